"""Drop-in for the reference's src/models/baseline/OnlyImagingModule.py: the
imaging-only binary tumour classifier (the default model of configs/train.yaml),
built on the MI355X image towers of the pretraining path.

Same constructor (model, optimizer, scheduler, label_weights, coral_lambda,
pretrained_vlp_module, :36-106), same `network` sub-module with timm key names
(`network.<timm resnet34 incl. fc>` / `network.<timm nest_small incl. head>`),
forward(x) -> flattened logits (:236-237), forward_features / forward_head
(:245-249), _compute_loss (:251-302: weighted BCE + optional CORAL between the
INTERNAL and BTXRD samples' pooled features, shared with FusionModule),
configure_optimizers (:108-120), training_step (:305-335), validation_step's
dataloader-index rule (:337-384) and on_validation_epoch_end's combined
evaluation over the cached probabilities, logits and features (:386-430).

The networks:
  * resnet34: `ResNet34Classifier` (timm resnet34(num_classes=1) on the HIP
    tower, vlp_amd/resnet34.py); its fused average pool emits the pooled
    features, so forward_features returns [B, 512, 1, 1] -- every consumer in
    the reference takes the spatial mean of that map (forward_head's global
    pool, _compute_loss :282-283), the identity on a 1x1 map;
  * nest_small: `NestClassifier` (timm nest_small(num_classes=1) on the HIP NesT
    tower, vlp_amd/nest.py; `image_size` sets timm's img_size, default 224 as
    timm's), features [B, 384, 1, 1] after the final LayerNorm and token mean.
Not built (NotImplementedError): vit_base/large_patch16_224, resnet50 and the
torchxrayvision resnet50-res512-all backbone.  Checkpoints of a pretrained
VisionLanguageModule load with torch.load(weights_only=True) (the reference uses
weights_only=False, :76).

Metrics: torchmetrics is absent from this image; `BinaryMetrics` restates the
Binary{Accuracy,Precision,Recall,F1Score,AUROC} values at threshold 0.5 that the
reference logs (AUROC as the Mann-Whitney rank statistic with tie averaging).
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Tuple

import torch
import torch.nn as nn

_PKG = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from src.models.baseline.FusionModule import FusionModule, ResNet34Classifier  # noqa: E402
from src.models.pretrain.VisionLanguageModule import _Base, _HAVE_LIGHTNING, _default_device  # noqa: E402
from vlp_amd.nest import NestTower  # noqa: E402

logger = logging.getLogger("project")

supported_models = ["vit_base_patch16_224", "vit_large_patch16_224", "resnet50", "resnet34", "nest_small",
                    "resnet50-res512-all"]


class NestClassifier(NestTower):
    """timm nest_small(num_classes) on the HIP tower: forward_features / forward_head / forward."""

    def __init__(self, num_classes: int = 1, img_size: int = 224, compute_dtype: str = "fp32", device=None,
                 drop_path_rate: float = 0.5):
        super().__init__("nest_small", img_size=img_size, drop_path_rate=drop_path_rate,
                         compute_dtype=compute_dtype, device=device)
        self.head = nn.Linear(self.dims[-1], num_classes, device=device)

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        self.head._apply(fn)
        return self

    def forward_features(self, x):
        return NestTower.forward(self, x)[:, :, None, None]

    def forward_head(self, x):
        return self.head(x.mean((2, 3)) if x.dim() == 4 else x)

    def forward(self, x):
        return self.forward_head(self.forward_features(x))


class BinaryMetrics:
    """Epoch accumulator for torchmetrics' Binary{Accuracy, Precision, Recall,
    F1Score, AUROC} (threshold 0.5; precision / recall / F1 are 0 when their
    denominator is 0, as torchmetrics' zero_division default)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self._p, self._y = [], []

    def update(self, probs, labels):
        self._p.append(probs.detach().float().reshape(-1).cpu())
        self._y.append(labels.detach().reshape(-1).cpu().long())

    def compute(self):
        if not self._p:
            return {}
        p, y = torch.cat(self._p), torch.cat(self._y)
        return binary_metrics(p, y)


def binary_metrics(p: torch.Tensor, y: torch.Tensor):
    pred = (p >= 0.5).long()
    tp = int(((pred == 1) & (y == 1)).sum())
    fp = int(((pred == 1) & (y == 0)).sum())
    fn = int(((pred == 0) & (y == 1)).sum())
    acc = int((pred == y).sum()) / y.numel() if y.numel() else 0.0
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * prec * rec / (prec + rec) if prec + rec else 0.0
    npos, nneg = int((y == 1).sum()), int((y == 0).sum())
    if npos and nneg:
        # Mann-Whitney U with average ranks for ties = the area under the ROC curve
        order = torch.argsort(p.double())
        ps = p.double()[order]
        ranks = torch.empty_like(ps)
        i, n = 0, ps.numel()
        while i < n:
            j = i
            while j + 1 < n and ps[j + 1] == ps[i]:
                j += 1
            ranks[i:j + 1] = 0.5 * (i + j) + 1.0
            i = j + 1
        r = torch.empty_like(ranks)
        r[order] = ranks
        auroc = float((r[y == 1].sum() - npos * (npos + 1) / 2) / (npos * nneg))
    else:
        auroc = 0.0
    return {"accuracy": acc, "precision": prec, "recall": rec, "f1": f1, "auroc": auroc}


class OnlyImagingModule(_Base):
    def __init__(
        self,
        model: str,
        optimizer,
        scheduler=None,
        label_weights: Tuple[float] = (1.0, 1.0),
        coral_lambda: float = 0.0,
        pretrained_vlp_module: str = None,
        compute_dtype: str = "fp32",
        image_size: int = 224,
        device=None,
        **kwargs,
    ):
        super().__init__()
        hp = dict(model=model, optimizer=optimizer, scheduler=scheduler, label_weights=label_weights,
                  coral_lambda=coral_lambda, pretrained_vlp_module=pretrained_vlp_module,
                  compute_dtype=compute_dtype, image_size=image_size, **kwargs)
        if _HAVE_LIGHTNING:  # pragma: no cover
            self.save_hyperparameters(logger=False)
        else:
            self.save_hyperparameters(hp, logger=False)
        if model not in supported_models:                                              # :49-52
            raise ValueError(f"OnlyImagingModule: Model {model} is not supported. Supported models are: "
                             f"{supported_models}")
        if model not in ("resnet34", "nest_small"):
            raise NotImplementedError(f"OnlyImagingModule: {model} is not built for MI355X "
                                      "(resnet34 and nest_small are)")
        dev = _default_device(device)
        if model == "resnet34":
            self.network = ResNet34Classifier(1, compute_dtype=compute_dtype, device=dev)
        else:
            self.network = NestClassifier(1, img_size=image_size, compute_dtype=compute_dtype, device=dev,
                                          drop_path_rate=kwargs.get("drop_path_rate", 0.5))   # timm's default
        if pretrained_vlp_module is not None:                                          # :75-98
            ckpt = torch.load(pretrained_vlp_module, map_location="cpu", weights_only=True)
            sd = {k.replace("image_encoder.model.", ""): v for k, v in ckpt["state_dict"].items()
                  if k.startswith("image_encoder.model.")}
            missing, unexpected = self.network.load_state_dict(sd, strict=False)
            used = sum(v.numel() for k, v in sd.items() if k not in unexpected)
            if unexpected:
                logger.warning("OnlyImagingModule: unexpected keys in the pretrained vision encoder: %s",
                               unexpected)
            logger.info("OnlyImagingModule: loaded %d pretrained vision-encoder parameters from %s "
                        "(%d missing keys: the classification head)", used, pretrained_vlp_module, len(missing))
        self.label_weights = torch.Tensor(label_weights)                               # :101
        self.train_metrics = BinaryMetrics()
        self.val_metrics = {"internal": BinaryMetrics(), "btxrd": BinaryMetrics(), "combined": BinaryMetrics()}
        self._clear_val_cache()
        logger.info("OnlyImagingModule (MI355X): initialized %s, compute_dtype=%s", model, compute_dtype)

    @property
    def device(self):
        return self.network.arena.data.device

    def _clear_val_cache(self):
        self.all_val_probs, self.all_val_labels, self.all_val_logits = [], [], []
        self.all_val_features, self.all_val_datset_labels = [], []

    def get_image_network(self):
        return self.network

    def all_reduce_gradients(self, world: int) -> None:
        """Data-parallel gradient mean (the trainer's DDP hook): the tower's flat
        gradient arena in one SUM all-reduce, the classification head in one
        more, both scaled by 1/world."""
        dist = torch.distributed
        tower = self.network
        slots = [(owner._parameters[attr], full) for owner, attr, full in tower._param_slots]
        tower_ids = {id(p) for p, _ in slots}
        aliased = all(p.grad is not None and p.grad.data_ptr() == tower.arena.gview(full).data_ptr()
                      for p, full in slots)
        if aliased:
            dist.all_reduce(tower.arena.grad)
            tower.arena.grad.mul_(1.0 / world)
            rest = [p for p in self.parameters() if p.grad is not None and id(p) not in tower_ids]
        else:
            rest = [p for p in self.parameters() if p.grad is not None]
        if rest:
            flat = torch.cat([p.grad.reshape(-1) for p in rest])
            dist.all_reduce(flat)
            flat.mul_(1.0 / world)
            off = 0
            for p in rest:
                p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                off += p.numel()

    # ---------------- optimizer (:108-120) ----------------
    def configure_optimizers(self):
        optimizer = self.hparams.optimizer(params=self.parameters())
        if self.hparams.scheduler is not None:
            scheduler = self.hparams.scheduler(optimizer=optimizer)
            return {"optimizer": optimizer,
                    "lr_scheduler": {"scheduler": scheduler, "interval": "epoch", "frequency": 1}}
        return {"optimizer": optimizer}

    # ---------------- forward / loss (:236-302) ----------------
    def forward(self, x):
        return self.network(x.to(self.device, non_blocking=True)).flatten()

    def forward_features(self, x):
        return self.network.forward_features(x.to(self.device, non_blocking=True))

    def forward_head(self, x):
        return self.network.forward_head(x).flatten()

    _compute_loss = FusionModule._compute_loss      # weighted BCE + CORAL, :251-302 == FusionModule :341-390

    def _unpack(self, batch):
        x = batch["x-ray"] if "x-ray" in batch else batch["x-ray-u8"]
        if hasattr(self.network, "u8_norm"):
            self.network.u8_norm = tuple(batch.get("x-ray-u8-norm", (127.5, 73.9)))
        return x, batch["tumor"], batch["dataset"]

    def training_step(self, batch, batch_idx=None):                                  # :305-335
        x, labels, dataset = self._unpack(batch)
        features = self.forward_features(x)
        logits = self.forward_head(features)
        loss, cls, cor = self._compute_loss(features, logits, labels, dataset)
        self.train_metrics.update(torch.sigmoid(logits), labels)
        bs = x.shape[0]
        self.log("train/classification_loss", cls, on_step=True, on_epoch=True, batch_size=bs)
        self.log("train/coral_loss", cor, on_step=True, on_epoch=True, batch_size=bs)
        self.log("train/loss", loss, on_step=True, on_epoch=True, batch_size=bs)
        return loss

    def on_train_epoch_end(self):
        for k, v in self.train_metrics.compute().items():
            self.log(f"train/{k}", v, on_step=False, on_epoch=True)
        self.train_metrics.reset()

    @torch.no_grad()
    def validation_step(self, batch, batch_idx, dataloader_idx=0):                   # :337-384
        x, labels, dataset = self._unpack(batch)
        features = self.forward_features(x)
        logits = self.forward_head(features)
        loss, _, _ = self._compute_loss(features, logits, labels, dataset)
        probs = torch.sigmoid(logits)
        self.all_val_probs.append(probs)
        self.all_val_labels.append(labels.to(probs.device))
        self.all_val_logits.append(logits)
        self.all_val_features.append(features)
        self.all_val_datset_labels.extend(dataset)
        if dataloader_idx == 0:
            key = "internal"
        elif dataloader_idx == 1:
            key = "btxrd"
        else:
            raise ValueError(f"OnlyImagingModule: Validation dataloader index {dataloader_idx} is not supported. "
                             "Supported indices are: 0, 1.")
        self.val_metrics[key].update(probs, labels)
        self.log(f"val/{key}/loss", loss, on_step=True, on_epoch=True, add_dataloader_idx=False,
                 batch_size=x.shape[0])
        return loss

    @torch.no_grad()
    def on_validation_epoch_end(self):                                               # :386-430
        for key in ("internal", "btxrd"):
            for k, v in self.val_metrics[key].compute().items():
                self.log(f"val/{key}/{k}", v, on_step=False, on_epoch=True, add_dataloader_idx=False)
            self.val_metrics[key].reset()
        if not self.all_val_probs:
            return
        probs, labels = torch.cat(self.all_val_probs), torch.cat(self.all_val_labels)
        logits, features = torch.cat(self.all_val_logits), torch.cat(self.all_val_features)
        loss, cls, cor = self._compute_loss(features, logits, labels, self.all_val_datset_labels)
        bs = features.shape[0]
        self.log("val/combined/loss", loss, on_step=False, on_epoch=True, add_dataloader_idx=False, batch_size=bs)
        self.log("val/combined/classification_loss", cls, on_step=False, on_epoch=True,
                 add_dataloader_idx=False, batch_size=bs)
        self.log("val/combined/coral_loss", cor, on_step=False, on_epoch=True, add_dataloader_idx=False,
                 batch_size=bs)
        for k, v in binary_metrics(probs.float().cpu(), labels.cpu().long()).items():
            self.log(f"val/combined/{k}", v, on_step=False, on_epoch=True, add_dataloader_idx=False, batch_size=bs)
        self._clear_val_cache()
