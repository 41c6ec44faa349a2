"""Drop-in for the reference's src/data/DownstreamDataModule.py feeding FusionModule
(SURVEY §8(f) row 1): synthetic INTERNAL / BTXRD radiographs with clinical data.

Kept: constructor kwargs (using_crops, batch_size, num_workers, num_channels,
try_with_only_n_samples, gaussian_noise_augmentation, scale_intensity_normalization,
DownstreamDataModule.py:98-107), num_channels not in {1, 3} -> ValueError (:119-125),
get_cv_splits() yielding (DataModuleFolds(train, [internal_val, btxrd_val]),
label_weights) with w_c = n / (2 * n_c) over the training labels (:256-337), and the
batch keys FusionModule reads: "x-ray", "tumor", "dataset", "anatomy_site_encoded"
[B,9], "age_encoded" [B,4], "sex_encoded" [B,2] (FusionModule.py:392-394).
MI355X: the image goes up as the uint8 1-channel "x-ray-u8" by default (normalised
on the device), upload="fp32" gives the normalised 3-channel "x-ray".
The BTXRD / INTERNAL readers and MONAI transforms are not built (no data in this
image): synthetic=False raises NotImplementedError.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch.utils.data import DataLoader, Dataset, Subset

from src.data.PretrainDataModule import normalize_u8

N_SITES, N_AGE, N_SEX = 9, 4, 2


class SyntheticClinicalRadiographs(Dataset):
    def __init__(self, n: int, image_size: int, seed: int = 0, tumor_rate: float = 0.35):
        self.n, self.H, self.seed, self.rate = n, image_size, seed, tumor_rate

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if not 0 <= i < self.n:
            raise IndexError(i)
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        oh = torch.nn.functional.one_hot
        return {
            "x-ray-u8": torch.randint(0, 256, (1, self.H, self.H), generator=g, dtype=torch.uint8),
            "tumor": int(torch.rand((), generator=g) < self.rate),
            "dataset": "INTERNAL" if i % 2 == 0 else "BTXRD",
            "anatomy_site_encoded": oh(torch.randint(0, N_SITES, (), generator=g), N_SITES).float(),
            "age_encoded": oh(torch.randint(0, N_AGE, (), generator=g), N_AGE).float(),
            "sex_encoded": oh(torch.randint(0, N_SEX, (), generator=g), N_SEX).float(),
            "image_path": f"synthetic://downstream/{i}.png",
        }


class ClinicalCollator:
    def __init__(self, upload: str = "u8", num_channels: int = 3):
        if upload not in ("u8", "fp32"):
            raise ValueError(f"upload must be 'u8' or 'fp32', got {upload!r}")
        self.upload, self.num_channels = upload, num_channels

    def __call__(self, samples: List[dict]) -> dict:
        if not samples:
            raise ValueError("empty batch")
        x_u8 = torch.stack([s["x-ray-u8"] for s in samples])
        b = {"tumor": torch.tensor([s["tumor"] for s in samples], dtype=torch.long),
             "dataset": [s["dataset"] for s in samples], "image_path": [s["image_path"] for s in samples]}
        for k in ("anatomy_site_encoded", "age_encoded", "sex_encoded"):
            b[k] = torch.stack([s[k] for s in samples])
        if self.upload == "u8":
            b["x-ray-u8"] = x_u8
        else:
            b["x-ray"] = normalize_u8(x_u8, self.num_channels)
        return b


class DataModuleFolds:
    """One fold: train loader + [internal_val, btxrd_val] (the reference's DataModuleFolds)."""

    def __init__(self, train_dataloader, val_dataloaders, batch_size):
        self._train, self._val, self.batch_size = train_dataloader, val_dataloaders, batch_size

    def train_dataloader(self):
        return self._train

    def val_dataloader(self):
        return self._val


class DownstreamDataModule:
    def __init__(self, using_crops: bool = False, batch_size: int = 32, num_workers: int = 2,
                 num_channels: int = 3, try_with_only_n_samples: Optional[int] = None,
                 gaussian_noise_augmentation: bool = True, scale_intensity_normalization: bool = False,
                 synthetic: bool = True, image_size: int = 224, n_samples: int = 512,
                 n_val_samples: int = 64, n_folds: int = 1, upload: str = "u8", seed: int = 0):
        if not (num_channels == 1 or num_channels == 3):
            raise ValueError(f"DownstreamDataModule: num_channels must be 1 or 3, but got {num_channels}")
        if not synthetic:
            raise NotImplementedError("DownstreamDataModule (MI355X build): BTXRD/INTERNAL readers are not "
                                      "part of this build; use synthetic=True")
        if scale_intensity_normalization:
            raise NotImplementedError("scale_intensity_normalization serves the torchxrayvision backbone only")
        self.using_crops, self.batch_size, self.num_workers = using_crops, batch_size, num_workers
        self.num_channels, self.try_with_only_n_samples = num_channels, try_with_only_n_samples
        self.image_size, self.n_samples, self.n_val, self.n_folds, self.seed = (
            image_size, n_samples, n_val_samples, n_folds, seed)
        self.collate = ClinicalCollator(upload if num_channels == 3 else "fp32", num_channels)

    @staticmethod
    def shard_indices(n, rank, world):
        """DistributedSampler(drop_last=False)'s split: the index list is padded by
        wrapping to ceil(n / world) * world, then rank r takes r, r + world, ...
        Every rank gets the same number of samples (hence batches), so the
        per-step gradient all-reduce never waits on a rank that has run out."""
        per = -(-n // world)
        idx = list(range(n))
        total = per * world
        while len(idx) < total:
            idx += idx[:total - len(idx)]
        return idx[rank:total:world]

    @classmethod
    def _shard(cls, ds):
        """Data parallel: each rank reads its own interleaved shard of the dataset
        (DistributedSampler's split, which Lightning's DDP inserts for the
        reference); the label weights stay those of the whole training set."""
        d = torch.distributed
        if not (d.is_available() and d.is_initialized()) or d.get_world_size() == 1:
            return ds
        return Subset(ds, cls.shard_indices(len(ds), d.get_rank(), d.get_world_size()))

    def _loader(self, ds, shuffle):
        return DataLoader(self._shard(ds), batch_size=self.batch_size, shuffle=shuffle,
                          num_workers=self.num_workers, collate_fn=self.collate,
                          pin_memory=torch.cuda.is_available())

    def get_cv_splits(self):
        for i in range(self.n_folds):
            n = self.n_samples if self.try_with_only_n_samples is None else self.try_with_only_n_samples
            nv = self.n_val if self.try_with_only_n_samples is None else self.try_with_only_n_samples
            train = SyntheticClinicalRadiographs(n, self.image_size, self.seed + 101 * i)
            vals = [SyntheticClinicalRadiographs(nv, self.image_size, self.seed + 101 * i + 1 + k) for k in (0, 1)]
            labels = torch.tensor([train[j]["tumor"] for j in range(len(train))])
            n0, n1 = int((labels == 0).sum()), int((labels == 1).sum())
            w0 = len(labels) / (2 * n0) if n0 else float("inf")                      # :330-332
            w1 = len(labels) / (2 * n1) if n1 else float("inf")
            yield DataModuleFolds(self._loader(train, True), [self._loader(v, False) for v in vals],
                                  self.batch_size), (float(w0), float(w1))
