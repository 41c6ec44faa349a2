"""The subset of lightning.pytorch.Trainer that src/train.py drives for pretraining
(SURVEY §8(b) "Loop semantics"): per step model.train(), optimizer.zero_grad(),
loss = training_step(batch, i), loss.backward(), optimizer.step(); epoch hooks;
validation over [lera_val, mura_val] with dataloader_idx; epoch-interval LR
schedulers.  Lightning is not in this image; configs/trainer/default.yaml's
`lightning.pytorch.trainer.Trainer` target resolves here (src/utils/config.py).

MI355X specifics: batches reach the device through DevicePrefetcher (copy of
batch i+1 on a side stream while step i runs); the loss is read back to the
host only every `log_every_n_steps` steps so the HIP queue is not drained per
step.  Multi-GPU: one process per GPU with torch.distributed initialised by
the launcher (backend nccl = RCCL); VisionLanguageModule's fused step performs
the embedding all-gather and the gradient all-reduce itself
(`handles_dp_collectives`), so the model is never wrapped in DDP.  For other
modules (FusionModule) the trainer averages gradients after backward as DDP
would: the module's `all_reduce_gradients()` when it has one (one RCCL call
over the ResNet34 tower's flat gradient arena), else one flat SUM all-reduce
over every gradient, divided by the world size.

Callbacks (the Lightning ones the reference configs name resolve here when
Lightning is absent, src/utils/config.py): ModelCheckpoint (best-k by a
monitored metric, Lightning checkpoint dict {state_dict, hyper_parameters,
epoch, global_step}; `trainer.checkpoint_callback.best_model_path` feeds
src/train.py's post-fit reload as in the reference :189-198), EarlyStopping
(patience on a monitored metric) and LearningRateMonitor.  Validation runs
every epoch over all batches unless limit_val_batches says otherwise
(Lightning's defaults).
"""
from __future__ import annotations

import functools
import logging
import math
import os
import re
import time
from typing import List, Optional

import torch

from src.data.PretrainDataModule import DevicePrefetcher

logger = logging.getLogger("project")


def _metric(trainer, key):
    v = trainer.logged_metrics.get(key)
    if v is None:
        return None
    return float(v.detach()) if torch.is_tensor(v) else float(v)


def _rank0():
    d = torch.distributed
    return not (d.is_available() and d.is_initialized()) or d.get_rank() == 0


def _dist_on():
    d = torch.distributed
    return d.is_available() and d.is_initialized() and d.get_world_size() > 1


def _dist_device():
    """Device of the collective's tensors: the rank's GPU for RCCL, the host for gloo."""
    d = torch.distributed
    if d.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def sync_val_metrics(metrics: dict) -> None:
    """Mean over ranks of every `val*` scalar (in place), as Lightning's
    sync_dist / torchmetrics sync does for the monitored metrics: every rank
    then takes the same checkpoint and early-stopping decisions.  The union of
    the ranks' keys is used; a key a rank lacks counts only where present."""
    if not _dist_on():
        return
    d = torch.distributed
    mine = sorted(k for k, v in metrics.items() if k.startswith("val") and isinstance(v, (int, float)))
    keys = [None] * d.get_world_size()
    d.all_gather_object(keys, mine)
    allk = sorted(set().union(*keys))
    if not allk:
        return
    t = torch.zeros(2, len(allk), dtype=torch.float64, device=_dist_device())
    for i, k in enumerate(allk):
        if k in metrics:
            t[0, i] = float(metrics[k])
            t[1, i] = 1.0
    d.all_reduce(t)
    for i, k in enumerate(allk):
        if t[1, i] > 0:
            metrics[k] = float(t[0, i] / t[1, i])


def _any_rank(flag: bool) -> bool:
    """MAX over ranks of a boolean (Lightning's reduce_boolean_decision)."""
    if not _dist_on():
        return flag
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=_dist_device())
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return bool(t.item() > 0)


def _barrier():
    if _dist_on():
        torch.distributed.barrier()


def serializable_hparams(hp) -> dict:
    """Module hyper-parameters as a weights_only-loadable dict: primitives kept,
    functools.partial (optimizer / scheduler factories) as a `_target_` /
    `_partial_` node that src/utils/config.instantiate rebuilds, other objects
    (the downstream datamodule) dropped -- load_from_checkpoint takes them as
    kwargs again, as src/train.py:198 does."""
    def conv(v):
        if v is None or isinstance(v, (bool, int, float, str)):
            return v
        if isinstance(v, (list, tuple)):
            out = [conv(x) for x in v]
            return None if any(x is _DROP for x in out) else out
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items() if conv(x) is not _DROP}
        if isinstance(v, functools.partial):
            f = v.func
            return {"_target_": f"{f.__module__}.{f.__qualname__}", "_partial_": True,
                    **{k: conv(x) for k, x in v.keywords.items()}}
        return _DROP
    out = {}
    for k, v in dict(hp or {}).items():
        c = conv(v)
        if c is not _DROP:
            out[k] = c
    return out


_DROP = object()


class ModelCheckpoint:
    """lightning.pytorch.callbacks.ModelCheckpoint (the options the reference
    configs use: monitor, mode, filename with {epoch} / {metric[:fmt]} fields,
    save_top_k, auto_insert_metric_name, dirpath).  monitor=None keeps the last
    epoch's checkpoint (Lightning's default checkpointing)."""

    def __init__(self, dirpath: Optional[str] = None, filename: Optional[str] = None, monitor: Optional[str] = None,
                 mode: str = "min", save_top_k: int = 1, auto_insert_metric_name: bool = True,
                 save_last: bool = False, verbose: bool = False, **unused):
        if mode not in ("min", "max"):
            raise ValueError(f"ModelCheckpoint: mode must be 'min' or 'max', got {mode!r}")
        self.dirpath, self.filename, self.monitor, self.mode = dirpath, filename, monitor, mode
        self.save_top_k, self.auto_insert_metric_name = save_top_k, auto_insert_metric_name
        self.best_model_path, self.best_model_score = "", None
        self._kept = []   # (score, path), best first

    def _format(self, trainer, score):
        name = self.filename or ("{epoch}-{step}" if self.monitor is None else "{epoch}-{" + self.monitor + "}")
        vals = {"epoch": trainer.current_epoch, "step": trainer.global_step}

        def sub(m):
            key, _, fmt = m.group(1).partition(":")
            v = vals.get(key, _metric(trainer, key))
            txt = "nan" if v is None else format(v, fmt) if fmt else str(v)
            return (f"{key}={txt}" if self.auto_insert_metric_name else txt).replace("/", "_")
        return re.sub(r"\{([^}]+)\}", sub, name) + ".ckpt"

    def _better(self, a, b):
        return b is None or (a < b if self.mode == "min" else a > b)

    def on_validation_end(self, trainer, pl_module):
        if self.save_top_k == 0:
            return
        score = None
        if self.monitor is not None:
            score = _metric(trainer, self.monitor)
            if score is None or not math.isfinite(score):
                return
            worst = self._kept[-1][0] if len(self._kept) >= self.save_top_k > 0 else None
            if worst is not None and not self._better(score, worst):
                return
        d = self.dirpath or os.path.join(trainer.default_root_dir, "checkpoints")
        path = os.path.join(d, self._format(trainer, score))
        if _rank0():
            os.makedirs(d, exist_ok=True)
            trainer.save_checkpoint(path, pl_module)
        _barrier()   # the file exists for every rank once it is named best_model_path
        if self.monitor is None:
            for _, old in self._kept:
                if old != path and _rank0() and os.path.exists(old):
                    os.remove(old)
            self._kept = [(None, path)]
        else:
            self._kept.append((score, path))
            self._kept.sort(key=lambda t: t[0], reverse=self.mode == "max")
            while self.save_top_k > 0 and len(self._kept) > self.save_top_k:
                _, old = self._kept.pop()
                if _rank0() and os.path.exists(old):
                    os.remove(old)
        self.best_model_path = self._kept[0][1]
        self.best_model_score = self._kept[0][0]


class EarlyStopping:
    """lightning.pytorch.callbacks.EarlyStopping: stop once the monitored metric
    has not improved (by more than min_delta) for `patience` validation rounds."""

    def __init__(self, monitor: str, mode: str = "min", patience: int = 3, min_delta: float = 0.0,
                 verbose: bool = False, **unused):
        self.monitor, self.mode, self.patience, self.min_delta, self.verbose = monitor, mode, patience, min_delta, verbose
        self.best, self.wait = None, 0

    def on_validation_end(self, trainer, pl_module):
        v = _metric(trainer, self.monitor)
        if v is None:
            return
        improved = self.best is None or (v < self.best - self.min_delta if self.mode == "min"
                                         else v > self.best + self.min_delta)
        if improved:
            self.best, self.wait = v, 0
            return
        self.wait += 1
        if self.wait >= self.patience:
            trainer.should_stop = True
            if self.verbose:
                logger.info("EarlyStopping: %s did not improve for %d rounds (best %.5f)", self.monitor,
                            self.wait, self.best)


class LearningRateMonitor:
    """lightning.pytorch.callbacks.LearningRateMonitor: logs each param group's lr."""

    def __init__(self, logging_interval: Optional[str] = None, **unused):
        self.logging_interval = logging_interval

    def on_train_epoch_end(self, trainer, pl_module):
        opt = getattr(trainer, "optimizer", None)
        if opt is None:
            return
        for i, g in enumerate(opt.param_groups):
            trainer.logged_metrics[f"lr-{type(opt).__name__}/{g.get('name', i)}"] = g["lr"]


class Trainer:
    def __init__(self, min_epochs: int = 1, max_epochs: int = 10, accelerator: str = "auto",
                 devices="auto", log_every_n_steps: int = 1, max_steps: int = -1,
                 limit_train_batches: Optional[int] = None, limit_val_batches: Optional[int] = None,
                 callbacks: Optional[List] = None, logger=None, enable_checkpointing: bool = True,
                 default_root_dir: Optional[str] = None, check_val_every_n_epoch: int = 1, **unused):
        if max_epochs is not None and min_epochs is not None and min_epochs > max_epochs:
            raise ValueError("min_epochs > max_epochs")
        self.min_epochs, self.max_epochs = min_epochs, max_epochs
        self.accelerator, self.devices = accelerator, devices
        self.log_every_n_steps = max(1, int(log_every_n_steps))
        self.max_steps = max_steps
        self.limit_train_batches, self.limit_val_batches = limit_train_batches, limit_val_batches
        self.callbacks = list(callbacks or [])
        self.default_root_dir = default_root_dir or os.getcwd()
        self.enable_checkpointing = enable_checkpointing
        self.check_val_every_n_epoch = max(1, int(check_val_every_n_epoch))
        if enable_checkpointing and not any(isinstance(c, ModelCheckpoint) for c in self.callbacks):
            self.callbacks.append(ModelCheckpoint())     # Lightning's default: the last epoch
        self.should_stop = False
        self.global_step = 0
        self.current_epoch = 0
        self.sanity_checking = False
        self.logged_metrics = {}
        self.history = []            # (global_step, loss) at every logging step
        self.step_times = []
        if unused:
            logger.info("Trainer: ignoring Lightning options %s", sorted(unused))

    def _device(self, model):
        return model.device

    @property
    def checkpoint_callback(self):
        return next((c for c in self.callbacks if isinstance(c, ModelCheckpoint)), None)

    @property
    def callback_metrics(self):
        return self.logged_metrics

    def _hook(self, name, model):
        for cb in self.callbacks:
            fn = getattr(cb, name, None)
            if fn is not None:
                fn(self, model)

    def save_checkpoint(self, path, model):
        """Lightning checkpoint dict, loadable with torch.load(weights_only=True)."""
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        torch.save({"state_dict": sd, "hyper_parameters": serializable_hparams(getattr(model, "hparams", {})),
                    "epoch": self.current_epoch, "global_step": self.global_step}, path)

    @staticmethod
    def _dp_world():
        d = torch.distributed
        return d.get_world_size() if d.is_available() and d.is_initialized() else 1

    @staticmethod
    def average_gradients(model, world: int) -> None:
        """DDP-equivalent gradient mean across ranks (one bucket)."""
        if hasattr(model, "all_reduce_gradients"):
            model.all_reduce_gradients(world)
            return
        params = [p for p in model.parameters() if p.requires_grad and p.grad is not None]
        if not params:
            return
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        torch.distributed.all_reduce(flat)
        flat.mul_(1.0 / world)
        off = 0
        for p in params:
            n = p.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n

    def _log(self, model, step_loss):
        rec = {"step": self.global_step, "epoch": self.current_epoch, "train/loss": float(step_loss)}
        for k, v in getattr(model, "logged", {}).items():
            if torch.is_tensor(v) and v.numel() == 1:
                rec[k] = float(v.detach())
        self.logged_metrics.update(rec)
        self.history.append((self.global_step, float(step_loss)))
        rank = int(os.environ.get("RANK", "0"))
        if rank == 0:
            logger.info("step %d epoch %d loss %.5f", self.global_step, self.current_epoch, float(step_loss))

    def fit(self, model, datamodule=None, train_dataloaders=None, val_dataloaders=None):
        model.trainer = self
        if datamodule is not None:
            train_dataloaders = datamodule.train_dataloader()
            if self.limit_val_batches != 0 and hasattr(datamodule, "val_dataloader"):
                val_dataloaders = datamodule.val_dataloader()
        conf = model.configure_optimizers()
        optimizer = conf["optimizer"] if isinstance(conf, dict) else conf
        sched = conf.get("lr_scheduler") if isinstance(conf, dict) else None
        self.optimizer = optimizer
        dev = self._device(model)
        world = self._dp_world()
        reduce_grads = world > 1 and not getattr(model, "handles_dp_collectives", False)
        stop = False
        # training-batch augmentation on the device (the reference's MONAI chain runs
        # in its DataLoader workers, PretrainDataModule.py:186-198)
        augment = getattr(datamodule, "device_augment", None) if datamodule is not None else None
        t_fit = time.perf_counter()
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            model.train()
            if hasattr(model, "on_train_epoch_start"):
                model.on_train_epoch_start()
            for i, batch in enumerate(DevicePrefetcher(train_dataloaders, dev)):
                if self.limit_train_batches is not None and i >= self.limit_train_batches:
                    break
                t0 = time.perf_counter()
                if augment is not None:
                    batch = augment(batch)
                optimizer.zero_grad(set_to_none=False)
                loss = model.training_step(batch, i)
                loss.backward()
                if reduce_grads:
                    self.average_gradients(model, world)
                optimizer.step()
                self.global_step += 1
                if self.global_step % self.log_every_n_steps == 0:
                    lv = loss.detach().item()
                    if not math.isfinite(lv):
                        raise FloatingPointError(f"non-finite loss {lv} at step {self.global_step}")
                    self._log(model, lv)
                self.step_times.append(time.perf_counter() - t0)
                if 0 < self.max_steps <= self.global_step:
                    stop = True
                    break
            if hasattr(model, "on_train_epoch_end"):
                model.on_train_epoch_end()
            self._hook("on_train_epoch_end", model)
            if (epoch + 1) % self.check_val_every_n_epoch == 0:
                self._hook("on_validation_start", model)   # e.g. LinearProbeCallback (every n-th epoch)
                if val_dataloaders and self.limit_val_batches != 0:
                    self.validate(model, val_dataloaders)
                self._hook("on_validation_end", model)    # checkpointing, early stopping
                self.should_stop = _any_rank(self.should_stop)
            if sched is not None:
                s = sched["scheduler"] if isinstance(sched, dict) else sched
                s.step()
            if (stop or self.should_stop) and epoch + 1 >= (self.min_epochs or 0):
                break
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.fit_seconds = time.perf_counter() - t_fit
        return self

    @torch.no_grad()
    def validate(self, model, val_dataloaders):
        model.eval()
        if hasattr(model, "on_validation_epoch_start"):
            model.on_validation_epoch_start()
        for idx, loader in enumerate(val_dataloaders):
            for j, batch in enumerate(DevicePrefetcher(loader, self._device(model))):
                if self.limit_val_batches is not None and j >= self.limit_val_batches:
                    break
                model.validation_step(batch, j, idx)
        if hasattr(model, "on_validation_epoch_end"):
            model.on_validation_epoch_end()
        for k, v in getattr(model, "logged", {}).items():
            if k.startswith("val") and torch.is_tensor(v) and v.numel() == 1:
                self.logged_metrics[k] = float(v.detach())
            elif k.startswith("val") and isinstance(v, (int, float)):
                self.logged_metrics[k] = float(v)
        # monitored metrics are identical on every rank before the callbacks read them
        sync_val_metrics(self.logged_metrics)
        model.train()
