"""Linear probe on the image encoder's features during pretraining (reference
src/utils/LinearProbeCallback.py:17-116).

Same constructor (train_dataloader, val_dataloaders, every_n_epochs=5), same gate
(every n-th epoch, skipped while sanity checking), same probe (eval-mode 512-d
features -> sklearn LogisticRegression(max_iter=1000, lbfgs) -> balanced accuracy
and AUROC on the concatenated validation sets), same two logged keys.

MI355X: the features come from the HIP ResNet34 tower (eval-mode BN from the
running statistics) on the uint8 upload when the loader provides it, with the
batches moved by the side-stream DevicePrefetcher; only the [B, 512] features
come back to the host.  As in the reference, the encoder is left in eval mode
(the trainer puts the module back in train mode before the next step).
"""
from __future__ import annotations

import logging

import numpy as np
import torch
from sklearn.linear_model import LogisticRegression
from sklearn.metrics import balanced_accuracy_score, roc_auc_score
from torch.utils.data import ConcatDataset, DataLoader

from src.data.PretrainDataModule import DevicePrefetcher

logger = logging.getLogger("project")


class LinearProbeCallback:
    def __init__(self, train_dataloader: DataLoader, val_dataloaders: list, every_n_epochs: int = 5):
        self.train_dataloader = train_dataloader
        val_dataset = ConcatDataset([dl.dataset for dl in val_dataloaders])
        self.val_dataloader = DataLoader(val_dataset, batch_size=train_dataloader.batch_size, shuffle=False,
                                         collate_fn=train_dataloader.collate_fn,
                                         pin_memory=torch.cuda.is_available())
        self.every_n_epochs = every_n_epochs

    def on_validation_start(self, trainer, pl_module) -> None:
        if trainer.current_epoch % self.every_n_epochs != 0:
            return
        if getattr(trainer, "sanity_checking", False):
            return
        bacc, auroc = self._linear_probe_training(pl_module.image_encoder, pl_module.device)
        pl_module.log("downstream_validation/linear_probe_balanced_accuracy", bacc, on_step=False, on_epoch=True)
        pl_module.log("downstream_validation/linear_probe_auroc", auroc, on_step=False, on_epoch=True)

    def _linear_probe_training(self, image_encoder, device):
        image_encoder = image_encoder.eval()
        X_train, y_train = self._extract_features(image_encoder, self.train_dataloader, device)
        X_val, y_val = self._extract_features(image_encoder, self.val_dataloader, device)
        clf = LogisticRegression(max_iter=1000, solver="lbfgs")
        clf.fit(X_train, y_train)
        y_pred = clf.predict(X_val)
        balanced_acc = balanced_accuracy_score(y_val, y_pred)
        auroc = roc_auc_score(y_val, clf.predict_proba(X_val)[:, 1])
        return balanced_acc, auroc

    def _extract_features(self, encoder, dataloader, device):
        feats, labels = [], []
        with torch.no_grad():
            for batch in DevicePrefetcher(dataloader, device):
                imgs = batch["x-ray"] if "x-ray" in batch else batch["x-ray-u8"]
                feats.append(encoder(imgs.to(device, non_blocking=True)).float().cpu().numpy())
                labels.append(batch["tumor"].cpu().numpy())
        return np.concatenate(feats, axis=0), np.concatenate(labels, axis=0)
