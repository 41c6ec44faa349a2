"""Drop-in for the reference's src/models/baseline/FusionModule.py (late fusion of
ResNet34 imaging logits with a clinical-data MLP; SURVEY §8(f) row 1, BASELINE
configs[4]) on MI355X.

Same constructor (model, optimizer, scheduler, label_weights, coral_lambda,
pretrained_vlp_module, vision_encoder_lr, :38-50), same sub-module names and
state-dict keys (tabular_network.*, image_network.<timm resnet34 incl. fc>,
combination_network.*), same forward(x, age, sex, anatomy_site) -> (logits,
image_features) (:318-326), _compute_loss (:341-390: weighted BCE + optional
CORAL), configure_optimizers (:127-201: image_backbone / head_and_remaining
groups), training_step (:392-420) and validation_step's dataloader index rule.

The image network is the HIP ResNet34 tower of the pretraining path
(vlp_amd/resnet34.py, every conv / BN / pool on the hand-written kernels, >99.9 %
of the step's FLOPs).  Its fused average-pool kernel produces the pooled features
directly, so forward_features returns them as [B, 512, 1, 1]: the reference's
consumers only take the spatial mean of that map (forward_head's global pool,
CORAL's mean over (2, 3), :366-369), which is the identity on a 1x1 map.  The
fc, the 15->32->20->10 tabular MLP with BatchNorm1d, the 20->1 combination and
the loss (a few kFLOP per sample) run as device tensor ops.

Not built: the vit / resnet50 / nest_small / torchxrayvision backbones
(NotImplementedError), torchmetrics accuracy/AUROC logging, t-SNE plots.
Pretrained VLP checkpoints load with torch.load(weights_only=True) (the
reference uses weights_only=False, :84).
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

_PKG = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from src.models.pretrain.VisionLanguageModule import _Base, _HAVE_LIGHTNING, _default_device  # noqa: E402
from src.utils.coral_loss.coral import coral  # noqa: E402
from vlp_amd.resnet34 import ResNet34Tower  # noqa: E402

logger = logging.getLogger("project")

supported_models = ["vit_base_patch16_224", "vit_large_patch16_224", "resnet50", "resnet34", "nest_small",
                    "resnet50-res512-all"]


class ResNet34Classifier(ResNet34Tower):
    """timm resnet34(num_classes) on the HIP tower: forward_features / forward_head / forward."""

    def __init__(self, num_classes: int = 10, compute_dtype: str = "fp32", device=None):
        super().__init__(drop_rate=0.0, compute_dtype=compute_dtype, device=device)
        self.fc = nn.Linear(512, num_classes, device=device)

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        self.fc._apply(fn)
        return self

    def forward_features(self, x):
        return ResNet34Tower.forward(self, x)[:, :, None, None]

    def forward_head(self, x):
        return self.fc(x.mean((2, 3)) if x.dim() == 4 else x)

    def forward(self, x):
        return self.forward_head(self.forward_features(x))


class FusionModule(_Base):
    def __init__(
        self,
        model: str,
        optimizer,
        scheduler=None,
        label_weights: Tuple[float] = (1.0, 1.0),
        coral_lambda: float = 0.0,
        pretrained_vlp_module: str = None,
        vision_encoder_lr: float = None,
        compute_dtype: str = "fp32",
        device=None,
        **kwargs,
    ):
        super().__init__()
        hp = dict(model=model, optimizer=optimizer, scheduler=scheduler, label_weights=label_weights,
                  coral_lambda=coral_lambda, pretrained_vlp_module=pretrained_vlp_module,
                  vision_encoder_lr=vision_encoder_lr, compute_dtype=compute_dtype, **kwargs)
        if _HAVE_LIGHTNING:  # pragma: no cover
            self.save_hyperparameters(logger=False)
        else:
            self.save_hyperparameters(hp, logger=False)
        assert vision_encoder_lr is None or vision_encoder_lr >= 0.0, \
            "FusionModule: vision_encoder_lr must be None or >= 0.0"                  # :52
        if model not in supported_models:
            raise ValueError(f"FusionModule: Model {model} is not supported. Supported models are: "
                             f"{supported_models}")
        if model != "resnet34":
            raise NotImplementedError(f"FusionModule: {model} is not built for MI355X (resnet34 is)")
        dev = _default_device(device)
        self.tabular_network = nn.Sequential(                                          # :60-70
            nn.Linear(15, 32), nn.BatchNorm1d(32), nn.ReLU(),
            nn.Linear(32, 20), nn.BatchNorm1d(20), nn.ReLU(),
            nn.Linear(20, 10), nn.BatchNorm1d(10), nn.ReLU()).to(dev)
        self.image_network = ResNet34Classifier(10, compute_dtype=compute_dtype, device=dev)
        if pretrained_vlp_module is not None:                                          # :82-113
            ckpt = torch.load(pretrained_vlp_module, map_location="cpu", weights_only=True)
            sd = {k.replace("image_encoder.model.", ""): v for k, v in ckpt["state_dict"].items()
                  if k.startswith("image_encoder.model.")}
            missing, unexpected = self.image_network.load_state_dict(sd, strict=False)
            used = sum(v.numel() for k, v in sd.items() if k not in unexpected)
            if unexpected:
                logger.warning("FusionModule: unexpected keys in the pretrained vision encoder: %s", unexpected)
            logger.info("FusionModule: loaded %d pretrained vision-encoder parameters from %s (%d missing keys)",
                        used, pretrained_vlp_module, len(missing))
        self.combination_network = nn.Linear(20, 1).to(dev)                            # :117
        self.label_weights = torch.Tensor(label_weights)                               # :119
        logger.info("FusionModule (MI355X): initialized %s, compute_dtype=%s", model, compute_dtype)

    @property
    def device(self):
        return self.combination_network.weight.device

    def all_reduce_gradients(self, world: int) -> None:
        """Data-parallel gradient mean (DDP semantics, called by the trainer after
        backward): one SUM all-reduce over the tower's flat gradient arena and one
        over the ~6.7k head gradients, both scaled by 1/world."""
        dist = torch.distributed
        tower = self.image_network
        slots = [(owner._parameters[attr], full) for owner, attr, full in tower._param_slots]
        aliased = all(p.grad is not None and p.grad.data_ptr() == tower.arena.gview(full).data_ptr()
                      for p, full in slots)
        if aliased:          # tower gradients live in the arena: one call over the flat buffer
            arena = tower.arena.grad
            dist.all_reduce(arena)
            arena.mul_(1.0 / world)
            head = [p for n, p in self.named_parameters()
                    if p.grad is not None and (not n.startswith("image_network.") or ".fc." in n)]
        else:
            head = [p for p in self.parameters() if p.grad is not None]
        if head:
            flat = torch.cat([p.grad.reshape(-1) for p in head])
            dist.all_reduce(flat)
            flat.mul_(1.0 / world)
            off = 0
            for p in head:
                p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                off += p.numel()

    def get_image_network(self):
        return self.image_network

    # ---------------- optimizer (:127-201) ----------------
    def configure_optimizers(self):
        lr_v = self.hparams.vision_encoder_lr
        if lr_v is not None and lr_v >= 0.0:
            backbone, head = [], []
            for name, p in self.image_network.named_parameters():
                (head if ("head" in name or "classifier" in name or "fc" in name) else backbone).append(p)
            img_ids = {id(p) for p in self.image_network.parameters()}
            remaining = [p for p in self.parameters() if id(p) not in img_ids]
            groups = [{"params": backbone, "lr": lr_v, "name": "image_backbone"},
                      {"params": head + remaining, "name": "head_and_remaining_parameters"}]
            optimizer = self.hparams.optimizer(params=groups)
        else:
            optimizer = self.hparams.optimizer(params=self.parameters())
        if self.hparams.scheduler is not None:
            scheduler = self.hparams.scheduler(optimizer=optimizer)
            return {"optimizer": optimizer,
                    "lr_scheduler": {"scheduler": scheduler, "interval": "epoch", "frequency": 1}}
        return {"optimizer": optimizer}

    # ---------------- forward / loss (:318-390) ----------------
    def forward(self, x, age_encoded, sex_encoded, anatomy_site_encoded):
        dev = self.device
        image_features = self.forward_image_features(x.to(dev, non_blocking=True))
        image_logits = self.forward_image_head(image_features)
        clinical = torch.cat((anatomy_site_encoded, age_encoded, sex_encoded), dim=1).to(dev, non_blocking=True)
        clinical_logits = self.tabular_network(clinical.float())
        logits = self.combination_network(torch.cat((image_logits, clinical_logits), dim=1)).flatten()
        return logits, image_features

    def forward_image_features(self, x):
        return self.image_network.forward_features(x)

    def forward_image_head(self, x):
        return self.image_network.forward_head(x)

    def _compute_loss(self, image_features, logits, labels, dataset):
        labels = labels.to(logits.device)
        lw = self.label_weights.to(logits.device)
        sample_weights = torch.where(labels == 0, lw[0], lw[1])
        classification_loss = F.binary_cross_entropy_with_logits(logits, labels.float(), weight=sample_weights)
        zero = torch.zeros((), device=logits.device)
        if self.hparams.coral_lambda == 0.0:
            return classification_loss, classification_loss, zero
        pooled = image_features.mean((2, 3)) if image_features.dim() == 4 else image_features
        internal = torch.tensor([d == "INTERNAL" for d in dataset], dtype=torch.bool)
        btxrd = torch.tensor([d == "BTXRD" for d in dataset], dtype=torch.bool)
        if internal.sum() <= 1 or btxrd.sum() <= 1:                                  # :375-376
            return classification_loss, classification_loss, zero
        dev = pooled.device
        coral_loss = self.hparams.coral_lambda * coral(pooled[internal.to(dev)], pooled[btxrd.to(dev)])
        return classification_loss + coral_loss, classification_loss, coral_loss

    def _unpack(self, batch):
        x = batch["x-ray"] if "x-ray" in batch else batch["x-ray-u8"]
        self.image_network.u8_norm = tuple(batch.get("x-ray-u8-norm", (127.5, 73.9)))
        return (x, batch["tumor"], batch["dataset"], batch["anatomy_site_encoded"], batch["age_encoded"],
                batch["sex_encoded"])

    def training_step(self, batch, batch_idx=None):
        x, labels, dataset, site, age, sex = self._unpack(batch)
        logits, image_features = self.forward(x, age, sex, site)
        loss, cls, cor = self._compute_loss(image_features, logits, labels, dataset)
        bs = x.shape[0]
        self.log("train/classification_loss", cls, on_step=True, on_epoch=True, batch_size=bs)
        self.log("train/coral_loss", cor, on_step=True, on_epoch=True, batch_size=bs)
        self.log("train/loss", loss, on_step=True, on_epoch=True, batch_size=bs)
        return loss

    def validation_step(self, batch, batch_idx, dataloader_idx=0):
        x, labels, dataset, site, age, sex = self._unpack(batch)
        logits, image_features = self.forward(x, age, sex, site)
        loss, _, _ = self._compute_loss(image_features, logits, labels, dataset)
        if dataloader_idx == 0:
            key = "internal"
        elif dataloader_idx == 1:
            key = "btxrd"
        else:
            raise ValueError(f"FusionModule: Validation dataloader index {dataloader_idx} is not supported.")
        self.log(f"val/{key}/loss", loss, on_step=False, on_epoch=True, batch_size=x.shape[0],
                 add_dataloader_idx=False)
        return loss
