"""Hydra-compatible config composition and `_target_` instantiation for src/train.py.

Hydra / OmegaConf are not in this image, so this restates the subset the
reference's configs use (configs/train.yaml, configs/experiment/pretrain/*.yaml):
  * a primary config whose `defaults` list picks one file per group
    (`- data: pretrain`), `_self_`, and `- experiment: null`;
  * experiment files with `# @package _global_` merged at the root, whose own
    defaults `override /group: choice` replace a group choice and
    `/group@key: choice` load a group file under another key;
  * `${a.b}` interpolation (a whole-string reference keeps the referenced
    node's type; embedded references are substituted as text);
  * command-line overrides `experiment=pretrain/x`, `group=choice`, `a.b=value`;
  * group files with their own `defaults` list (configs/callbacks/*.yaml: plain
    names are options of the same group, merged in order around `_self_`);
  * the resolvers the reference configs use: `${oc.env:VAR[,default]}` (an
    unset PROJECT_ROOT falls back to the working directory) and
    `${hydra:runtime.output_dir}` / `${hydra:runtime.cwd}` (run directory
    logs/<task_name>/runs/<timestamp> under the working directory, as Hydra's);
    an interpolation whose key does not exist stays unresolved text (Hydra
    resolves lazily, so such a node only fails where it is used);
  * hydra.utils.instantiate semantics: `_target_` is imported and called with
    the other keys (recursively instantiated), `_partial_: true` returns a
    functools.partial.  Lightning targets resolve to src.utils.trainer
    (Trainer, ModelCheckpoint, EarlyStopping, LearningRateMonitor) when
    Lightning is absent.
"""
from __future__ import annotations

import copy
import functools
import importlib
import importlib.util
import os
import re
from typing import Any, Dict, List, Optional

import yaml

CONFIG_DIR = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "configs"))
_INTERP = re.compile(r"\$\{([^}]+)\}")
_FALLBACK_TARGETS = {"lightning.pytorch.trainer.Trainer": "src.utils.trainer.Trainer",
                     "lightning.Trainer": "src.utils.trainer.Trainer",
                     "lightning.pytorch.callbacks.ModelCheckpoint": "src.utils.trainer.ModelCheckpoint",
                     "lightning.pytorch.callbacks.EarlyStopping": "src.utils.trainer.EarlyStopping",
                     "lightning.pytorch.callbacks.LearningRateMonitor": "src.utils.trainer.LearningRateMonitor"}
_RUN_STAMP = None


def _load(path: str) -> dict:
    with open(path) as f:
        data = yaml.safe_load(f)
    return data or {}


def _group_file(root: str, group: str, choice: str) -> str:
    p = os.path.join(root, group, f"{choice}.yaml")
    if not os.path.exists(p):
        raise FileNotFoundError(f"config group {group!r} has no option {choice!r} ({p})")
    return p


def _load_group(root: str, group: str, choice: str) -> dict:
    """A group option, with its own defaults list (options of the same group)."""
    node = _load(_group_file(root, group, choice))
    if not isinstance(node, dict):
        return node
    defs = node.pop("defaults", None)
    if not defs:
        return node
    out: dict = {}
    if "_self_" not in defs:
        defs = list(defs) + ["_self_"]
    for e in defs:
        if e == "_self_":
            merge(out, node)
        elif isinstance(e, str):
            merge(out, _load_group(root, group, e))
        else:
            raise ValueError(f"unsupported defaults entry {e!r} in {group}/{choice}")
    return out


def merge(dst: dict, src: dict) -> dict:
    """Recursive dict merge, src wins (OmegaConf.merge for plain containers)."""
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _set_path(cfg: dict, dotted: str, value: Any) -> None:
    keys = dotted.split(".")
    node = cfg
    for k in keys[:-1]:
        node = node.setdefault(k, {})
    node[keys[-1]] = value


def _get_path(cfg: dict, dotted: str) -> Any:
    node = cfg
    for k in dotted.split("."):
        if not isinstance(node, dict) or k not in node:
            raise KeyError(f"interpolation ${{{dotted}}}: missing key {k!r}")
        node = node[k]
    return node


def _parse_defaults(entries) -> List[tuple]:
    """-> [(kind, group, package, choice)] kind in {self, group, override}."""
    out = []
    for e in entries or []:
        if e == "_self_":
            out.append(("self", None, None, None))
            continue
        if not isinstance(e, dict) or len(e) != 1:
            raise ValueError(f"unsupported defaults entry {e!r}")
        (key, choice), = e.items()
        kind = "group"
        if key.startswith("override "):
            kind, key = "override", key[len("override "):]
        key = key.lstrip("/")
        group, _, package = key.partition("@")
        out.append((kind, group, package or group, choice))
    return out


def compose(config_name: str = "train", overrides: Optional[List[str]] = None,
            config_dir: str = CONFIG_DIR) -> dict:
    overrides = list(overrides or [])
    primary = _load(os.path.join(config_dir, f"{config_name}.yaml"))
    entries = _parse_defaults(primary.pop("defaults", ["_self_"]))
    choices = {g: c for k, g, p, c in entries if k == "group" and p == g}
    plain, cli_choice = [], {}
    for o in overrides:
        k, _, v = o.partition("=")
        if not _:
            raise ValueError(f"override {o!r} is not key=value")
        add = len(k) - len(k.lstrip("+"))   # Hydra: +key appends a new key, ++key adds or sets
        k = k.lstrip("+")
        if add == 0 and "." not in k and (k in choices or os.path.isdir(os.path.join(config_dir, k))):
            cli_choice[k] = v
        else:
            plain.append((k, v, add))
    choices.update(cli_choice)
    if choices.get("experiment") not in (None, "null"):
        exp = _load(_group_file(config_dir, "experiment", choices["experiment"]))
        if "experiment" not in [g for _, g, _, _ in entries]:
            entries.append(("group", "experiment", "experiment", None))
        at = [g for _, g, _, _ in entries].index("experiment")
        for kind, g, p, c in _parse_defaults(exp.pop("defaults", [])):
            if kind == "override":
                if g not in cli_choice:          # the command line beats the experiment
                    choices[g] = c
            elif kind == "group":                # merged before the experiment's own keys (_self_ last)
                entries.insert(at, ("group", g, p, c))
                at += 1
    else:
        exp = None
    cfg: dict = {}
    for kind, g, pkg, c in entries:
        if kind == "self":
            merge(cfg, primary)
        elif g == "experiment":
            if exp is not None:
                merge(cfg, exp)                   # @package _global_
        else:
            choice = choices.get(g, c) if pkg == g else c
            if choice in (None, "null"):
                continue
            node = _load_group(config_dir, g, choice)
            if isinstance(node, dict):
                merge(cfg.setdefault(pkg, {}), node)
            else:
                cfg[pkg] = {} if node is None else node
    for k, v, add in plain:
        if add == 1:
            try:
                _get_path(cfg, k)
            except KeyError:
                pass
            else:
                raise ValueError(f"override +{k}: the key already exists (use ++{k}= or {k}=)")
        _set_path(cfg, k, yaml.safe_load(v))
    return resolve(cfg)


def resolve(cfg: dict) -> dict:
    """Resolve ${...} interpolations against the root (repeat until stable)."""
    root = copy.deepcopy(cfg)

    def lookup(key, depth):
        if key.startswith("oc.env:"):
            var, _, default = key[len("oc.env:"):].partition(",")
            val = os.environ.get(var.strip())
            if val is None:
                val = default.strip() if default else (os.getcwd() if var.strip() == "PROJECT_ROOT" else None)
            if val is None:
                raise KeyError(f"interpolation ${{{key}}}: environment variable {var} is not set")
            return val
        if key.startswith("hydra:"):
            what = key[len("hydra:"):].strip()
            if what == "runtime.cwd":
                return os.getcwd()
            if what == "runtime.output_dir":
                global _RUN_STAMP
                if _RUN_STAMP is None:
                    import time
                    _RUN_STAMP = time.strftime("%Y-%m-%d_%H-%M-%S")
                return os.path.join(os.getcwd(), "logs", str(root.get("task_name", "train")), "runs", _RUN_STAMP)
            raise KeyError(f"unsupported hydra resolver ${{{key}}}")
        return res(copy.deepcopy(_get_path(root, key)), depth + 1)

    def res(node, depth=0):
        if depth > 32:
            raise ValueError("interpolation cycle")
        if isinstance(node, dict):
            return {k: res(v, depth) for k, v in node.items()}
        if isinstance(node, list):
            return [res(v, depth) for v in node]
        if isinstance(node, str):
            m = _INTERP.fullmatch(node)
            try:
                if m:
                    return lookup(m.group(1).strip(), depth)
                if _INTERP.search(node):
                    return _INTERP.sub(lambda mm: str(lookup(mm.group(1).strip(), depth)), node)
            except KeyError as e:
                if "missing key" in str(e):
                    return node          # unresolvable: stays text until (unless) it is used
                raise
        return node

    return res(root)


def _import(path: str):
    path = _FALLBACK_TARGETS.get(path, path) if importlib.util.find_spec(path.split(".")[0]) is None else path
    mod, _, attr = path.rpartition(".")
    return getattr(importlib.import_module(mod), attr)


def instantiate(node: Any, **kwargs) -> Any:
    """hydra.utils.instantiate for plain containers."""
    if isinstance(node, list):
        return [instantiate(v) for v in node]
    if not isinstance(node, dict):
        return node
    if "_target_" not in node:
        return {k: instantiate(v) for k, v in node.items()}
    node = dict(node)
    target = _import(node.pop("_target_"))
    partial = bool(node.pop("_partial_", False))
    node.pop("_recursive_", None)
    args = {k: instantiate(v) for k, v in node.items()}
    args.update(kwargs)
    if partial:
        return functools.partial(target, **args)
    return target(**args)
