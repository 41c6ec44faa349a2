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
"""
from __future__ import annotations

import logging
import math
import os
import time
from typing import List, Optional

import torch

from src.data.PretrainDataModule import DevicePrefetcher

logger = logging.getLogger("project")


class Trainer:
    def __init__(self, min_epochs: int = 1, max_epochs: int = 10, accelerator: str = "auto",
                 devices="auto", log_every_n_steps: int = 1, max_steps: int = -1,
                 limit_train_batches: Optional[int] = None, limit_val_batches: Optional[int] = 0,
                 callbacks: Optional[List] = None, logger=None, enable_checkpointing: bool = False,
                 default_root_dir: Optional[str] = None, **unused):
        if max_epochs is not None and min_epochs is not None and min_epochs > max_epochs:
            raise ValueError("min_epochs > max_epochs")
        self.min_epochs, self.max_epochs = min_epochs, max_epochs
        self.accelerator, self.devices = accelerator, devices
        self.log_every_n_steps = max(1, int(log_every_n_steps))
        self.max_steps = max_steps
        self.limit_train_batches, self.limit_val_batches = limit_train_batches, limit_val_batches
        self.callbacks = list(callbacks or [])
        self.default_root_dir = default_root_dir
        self.enable_checkpointing = enable_checkpointing
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
            if self.limit_val_batches:
                val_dataloaders = datamodule.val_dataloader()
        conf = model.configure_optimizers()
        optimizer = conf["optimizer"] if isinstance(conf, dict) else conf
        sched = conf.get("lr_scheduler") if isinstance(conf, dict) else None
        self.optimizer = optimizer
        dev = self._device(model)
        world = self._dp_world()
        reduce_grads = world > 1 and not getattr(model, "handles_dp_collectives", False)
        stop = False
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
            for cb in self.callbacks:               # e.g. LinearProbeCallback (every n-th epoch)
                if hasattr(cb, "on_validation_start"):
                    cb.on_validation_start(self, model)
            if val_dataloaders and self.limit_val_batches:
                self.validate(model, val_dataloaders)
            if sched is not None:
                s = sched["scheduler"] if isinstance(sched, dict) else sched
                s.step()
            if stop and epoch + 1 >= (self.min_epochs or 0):
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
        model.train()
