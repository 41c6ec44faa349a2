"""ctypes binding of libvlp_hip.so (the C ABI declared in include/vlp_hip.h).

The argument types are derived from the header itself, so the Python side and
the C ABI cannot drift apart.  Every entry point returns a hipError_t; a
non-zero code raises ``RuntimeError`` (the reference's own error behaviour for a
failed device op is a torch RuntimeError as well).

There is deliberately NO fallback: if the shared library is missing or was
built for another architecture, importing the device path fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Dict, List

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_REPO = os.path.dirname(_PKG)
LIB_PATH = os.environ.get("VLP_HIP_LIB", os.path.join(_HERE, "libvlp_hip.so"))
HEADER_PATH = os.path.join(_REPO, "include", "vlp_hip.h")

F32, BF16 = 0, 1
ABI_VERSION = 3     # vlp_abi_version() of the library this binding was written against

_CTYPE = {
    "int": ctypes.c_int,
    "long long": ctypes.c_longlong,
    "unsigned long long": ctypes.c_ulonglong,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
}


def parse_header(path: str = HEADER_PATH) -> Dict[str, dict]:
    """Return {name: {"ret": str, "args": [(ctype_name, arg_name)]}} for every
    prototype in the header."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    protos = {}
    for m in re.finditer(r"\b(int|void)\s+(vlp_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        parsed = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                is_ptr = "*" in a
                a2 = a.replace("*", " ").replace("const ", "").strip()
                toks = a2.split()
                argname = toks[-1]
                tname = " ".join(toks[:-1])
                parsed.append(("ptr" if is_ptr else tname, argname))
        protos[name] = {"ret": ret, "args": parsed}
    return protos


# entry points timed by ops.py under a kernel-family key (with algorithmic FLOPs)
_FAMILY_TIMED = {"vlp_conv_fwd", "vlp_conv_fwd_act", "vlp_conv_dgrad", "vlp_conv_dgrad_relu",
                 "vlp_conv_dgrad_bn_act", "vlp_conv_dgrad_relu_act", "vlp_conv_dgrad_relu_ds", "vlp_conv_dgrad_relu2", "vlp_conv_wgrad", "vlp_conv_wgrad_ws", "vlp_stem_fwd", "vlp_stem_wgrad", "vlp_stem_wgrad_ws",
                 "vlp_stem1_fwd", "vlp_stem1_wgrad_ws", "vlp_stem1_pool_fwd", "vlp_stem1_bwd_fused",
                 "vlp_linear_fwd", "vlp_linear_fwd_rs", "vlp_linear_dgrad", "vlp_linear_wgrad", "vlp_linear_wgrad_ws",
                 "vlp_nest_attn_fwd", "vlp_nest_attn_bwd"}


# host-side queries (no GPU work): never timed
_QUERIES = {"vlp_linear_wgrad_ws_floats", "vlp_clip_loss_ws_floats", "vlp_stem1_bwd_fused_ws_floats",
            "vlp_stem1_fused_ok", "vlp_conv_fwd_act_ok", "vlp_conv_dgrad_act_ok"}


class HipError(RuntimeError):
    pass


class _Lib:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            raise ImportError(
                f"libvlp_hip.so not found at {path}: build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        self._dll = ctypes.CDLL(path)
        self.protos = parse_header()
        self._fns = {}
        for name, p in self.protos.items():
            fn = getattr(self._dll, name)  # AttributeError => ABI mismatch, fail loudly
            argtypes: List = []
            for t, _ in p["args"]:
                argtypes.append(ctypes.c_void_p if t == "ptr" else _CTYPE[t])
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int if p["ret"] == "int" else None
            self._fns[name] = fn
        ver = self._fns["vlp_abi_version"]()
        if ver != ABI_VERSION:
            raise ImportError(f"{path}: C ABI version {ver}, this binding needs {ABI_VERSION} "
                              f"(rebuild the library: make -C vision-language-pretraining-for-bone-tumor-detection_amd/csrc)")

    def __getattr__(self, name):
        fns = self.__dict__.get("_fns")
        if fns is None or name not in fns:
            raise AttributeError(name)
        fn = fns[name]
        ret = self.protos[name]["ret"]
        if name == "vlp_abi_version":  # returns a value, not an error code
            self.__dict__[name] = fn
            return fn

        from . import ktimer
        timed_here = name not in _FAMILY_TIMED and name not in _QUERIES

        def call(*args):
            tk = ktimer.begin(name[4:]) if timed_here and ktimer._ENABLED else None
            r = fn(*args)
            if tk is not None:
                ktimer.end(tk)
            if ret == "int" and r != 0:
                raise HipError(f"{name} failed with hipError {r}")
            return r

        call.__name__ = name
        self.__dict__[name] = call
        return call


_LIB = None


def lib() -> _Lib:
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
