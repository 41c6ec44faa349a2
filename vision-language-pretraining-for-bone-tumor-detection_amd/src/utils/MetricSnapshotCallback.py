"""SnapshotAllMetricsOnBestCallback (reference src/utils/MetricSnapshotCallback.py:10-103),
named by the reference callback configs (configs/callbacks/snapshot_metrics_*.yaml).

After each validation round: when `monitor` improves, every metric the trainer
holds is copied under "{monitor}_best_{name}".  The reference writes that copy
into wandb.summary; wandb is not in this image, so the snapshot is kept on the
callback (`snapshot`) and in the trainer's logged metrics, where src/train.py's
per-fold metrics pick it up.
"""
from __future__ import annotations

import torch


class SnapshotAllMetricsOnBestCallback:
    def __init__(self, monitor: str, mode: str):
        assert mode in ("min", "max"), "mode must be 'min' or 'max'"
        self.monitor, self.mode = monitor, mode
        self.best_val = float("-inf") if mode == "max" else float("inf")
        self.snapshot = {}

    def on_validation_end(self, trainer, pl_module) -> None:
        if getattr(trainer, "sanity_checking", False):
            return
        metrics = trainer.callback_metrics
        cur = metrics.get(self.monitor)
        if cur is None:
            return
        cur = cur.item() if isinstance(cur, torch.Tensor) else float(cur)
        better = cur > self.best_val if self.mode == "max" else cur < self.best_val
        if not better:
            return
        self.best_val = cur
        snap = {}
        for k, v in list(metrics.items()):
            if "_best_" in k:
                continue
            v = v.item() if isinstance(v, torch.Tensor) and v.numel() == 1 else v
            if isinstance(v, (int, float)):
                snap[f"{self.monitor}_best_{k}"] = float(v)
        self.snapshot = snap
        metrics.update(snap)
