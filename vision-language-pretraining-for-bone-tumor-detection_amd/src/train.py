"""src/train.py for the MI355X pretraining path (reference src/train.py:56-340).

Same entry points and flow for the VLP pretraining experiments:
  main(argv)  Hydra-style command line (`experiment=pretrain/pretrain_resnet34_tinybert
              data.batch_size=256 ...`), configs composed from ../configs with the
              reference's group names (src/utils/config.py; Hydra is not in this image);
  train(cfg)  seed (train.yaml `seed`, :86-88) -> instantiate cfg.data (:90) -> for each
              (datamodule, label_weights) in get_cv_splits() (:105): set
              model.label_weights, instantiate cfg.model (:109-116) and cfg.trainer
              (:163) with the configured callbacks (:123; Lightning's ModelCheckpoint /
              EarlyStopping / LearningRateMonitor resolve to src/utils/trainer.py) ->
              trainer.fit(model, datamodule) (:171) -> per-fold metrics -> for a
              VisionLanguageModule with downstream data: reload the best checkpoint
              (:189-198) and evaluate downstream precision@k (:204) -> metrics
              aggregated over folds (:231-262).
The late-fusion finetune (FusionModule + DownstreamDataModule) runs through the
same path: `experiment=baseline_imaging_and_clinical/baseline_imaging_and_clinical_resnet_34`.
Out of scope: W&B loggers (configured loggers whose package is
absent are skipped with a warning), t-SNE / confusion-matrix plots, downstream
zero-shot evaluation and the OnlyImaging baseline module.

Multi-GPU: launch one process per GPU (`python -m torch.distributed.run
--nproc-per-node N src/train.py ...`); train() initialises torch.distributed
(nccl = RCCL over xGMI) from the launcher's environment and pins each rank to
LOCAL_RANK.  The module's fused step all-gathers embeddings for the global-batch
loss and all-reduces gradients itself.
"""
from __future__ import annotations

import logging
import os
import random
import sys
from typing import Any, Dict, List, Optional, Tuple

_PKG = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.utils.config import compose, instantiate  # noqa: E402

log = logging.getLogger("project")


def seed_everything(seed: int) -> None:
    """lightning.seed_everything(seed, workers=True) (train.py:87-88)."""
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
    os.environ["PL_GLOBAL_SEED"] = str(seed)


def _init_distributed() -> None:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and not torch.distributed.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        torch.distributed.init_process_group(backend)


def instantiate_callbacks(cb_cfg) -> List[Any]:
    """src/utils/instantiators.py:instantiate_callbacks: every node with a _target_."""
    out = []
    for name, node in (cb_cfg or {}).items():
        if isinstance(node, dict) and "_target_" in node:
            log.info("Train: Instantiating callback <%s>", node["_target_"])
            out.append(instantiate(node))
    return out


def instantiate_loggers(lg_cfg) -> List[Any]:
    """Loggers whose package is installed; the others (wandb here) are skipped."""
    import importlib.util
    out = []
    for name, node in (lg_cfg or {}).items():
        if not (isinstance(node, dict) and "_target_" in node):
            continue
        pkg = node["_target_"].split(".")[0]
        need = "wandb" if "wandb" in node["_target_"].lower() else pkg
        if importlib.util.find_spec(pkg) is None or importlib.util.find_spec(need) is None:
            log.warning("Train: logger <%s> skipped (%s is not installed)", node["_target_"], need)
            continue
        out.append(instantiate(node))
    return out


_PRECISION_DTYPE = {None: "fp32", "32": "fp32", "32-true": "fp32", "bf16": "bf16", "bf16-mixed": "bf16",
                    "bf16-true": "bf16"}


def compute_dtype_for(precision) -> str:
    """HIP compute dtype for a Lightning `trainer.precision`.  The reference sets no
    precision (configs/trainer/default.yaml), i.e. Lightning's fp32: its experiments
    keep fp32 arithmetic unless they opt in (the _mi355x experiments name
    model.compute_dtype: bf16).  The HIP towers have no fp16 path."""
    key = None if precision is None else str(precision)
    if key not in _PRECISION_DTYPE:
        raise ValueError(f"trainer.precision={precision!r}: the MI355X build computes in fp32 or bf16 "
                         f"(use 32-true or bf16-mixed)")
    return _PRECISION_DTYPE[key]


def model_config(cfg: Dict[str, Any], label_weights) -> Dict[str, Any]:
    """The model node train() instantiates for one fold (src/train.py:109-116)."""
    model_cfg = dict(cfg["model"])
    if not model_cfg.get("scheduler"):
        model_cfg["scheduler"] = None
    model_cfg["label_weights"] = label_weights
    if "compute_dtype" not in model_cfg:   # the reference's arithmetic unless the run opts in
        model_cfg["compute_dtype"] = compute_dtype_for((cfg.get("trainer") or {}).get("precision"))
    if "FusionModule" in model_cfg["_target_"]:
        model_cfg.pop("downstream_datamodule", None)
    elif not isinstance(model_cfg.get("downstream_datamodule"), dict) or not model_cfg["downstream_datamodule"]:
        # model/vision_language.yaml names the group option ("downstream"); the experiments
        # interpolate the composed ${downstream_data} node, anything else means none
        model_cfg["downstream_datamodule"] = None
    return model_cfg


def train(cfg: Dict[str, Any]) -> Tuple[Dict[str, Any], Dict[str, Any]]:
    if cfg.get("k_fold_cross_validation", False):
        log.info("Train: Doing k-fold cross validation.")
    if cfg.get("seed"):
        seed_everything(int(cfg["seed"]))
    _init_distributed()
    log.info("Train: Instantiating datamodule <%s>", cfg["data"]["_target_"])
    datamodule = instantiate(cfg["data"])
    all_fold_metrics: List[Dict[str, Any]] = []
    objects: Dict[str, Any] = {"cfg": cfg, "datamodule": datamodule}
    for i, (fold_dm, label_weights) in enumerate(datamodule.get_cv_splits()):
        model_cfg = model_config(cfg, label_weights)
        log.info("Train: Instantiating model <%s>", model_cfg["_target_"])
        model = instantiate(model_cfg)
        callbacks = instantiate_callbacks(cfg.get("callbacks"))
        if cfg.get("downstream_data") and "VisionLanguageModule" in model_cfg["_target_"]:   # :123-134
            from src.utils.LinearProbeCallback import LinearProbeCallback
            ds_dm = instantiate(cfg["downstream_data"])
            dm, _ = next(ds_dm.get_cv_splits())
            callbacks.append(LinearProbeCallback(dm.train_dataloader(), dm.val_dataloader()))
            log.info("Train: Added LinearProbeCallback to callbacks.")
        log.info("Train: Instantiating trainer <%s>", cfg["trainer"]["_target_"])
        loggers = instantiate_loggers(cfg.get("logger"))
        tkw = {"callbacks": callbacks, "logger": loggers or None}
        out_dir = (cfg.get("paths") or {}).get("output_dir")
        if out_dir and "default_root_dir" not in cfg["trainer"]:
            tkw["default_root_dir"] = out_dir
        trainer = instantiate(cfg["trainer"], **tkw)
        objects.update(model=model, trainer=trainer, callbacks=callbacks)
        if cfg.get("train", True):
            trainer.fit(model=model, datamodule=fold_dm)
            bs = getattr(fold_dm, "batch_size", 0)
            ws = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
            log.info("Train: %d steps in %.2f s (%.1f image-text pairs/s incl. data loading, %d rank(s))",
                     trainer.global_step, trainer.fit_seconds,
                     ws * bs * trainer.global_step / max(trainer.fit_seconds, 1e-9), ws)
        fold_metrics = dict(trainer.logged_metrics)
        if "VisionLanguageModule" in model_cfg["_target_"] and cfg.get("downstream_data"):   # :189-210
            ck = trainer.checkpoint_callback
            if ck is not None and ck.best_model_path and os.path.exists(ck.best_model_path):
                log.info("Train: Using best model path from trainer: %s", ck.best_model_path)
                ds = instantiate(cfg["downstream_data"])
                model = type(model).load_from_checkpoint(ck.best_model_path, downstream_datamodule=ds,
                                                         device=model.device)
                objects["best_model"] = model   # objects["model"] stays the trained module, as in the reference
            else:
                log.warning("Train: No best model path found in trainer, using current model weights.")
            if getattr(model, "downstream_datamodule", None) is not None:
                for k, v in model.evaluate_downstream_precision_at_k(mode="entire").items():
                    fold_metrics[f"downstream_entire/label_precision_at_{k}"] = v
        all_fold_metrics.append(fold_metrics)
        if not cfg.get("k_fold_cross_validation", False):
            break
    metrics: Dict[str, Any] = {}
    if all_fold_metrics:
        keys = set.intersection(*(set(m) for m in all_fold_metrics))
        for k in sorted(keys):
            vals = [m[k] for m in all_fold_metrics if isinstance(m[k], (int, float))]
            if vals:
                metrics[k] = float(np.mean(vals))
                metrics[k + "_std"] = float(np.std(vals))
    return metrics, objects


def main(argv: Optional[List[str]] = None) -> Dict[str, Any]:
    logging.basicConfig(level=os.environ.get("VLP_LOGLEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(message)s")
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = compose("train", argv)
    metrics, _ = train(cfg)
    return metrics


if __name__ == "__main__":
    main()
