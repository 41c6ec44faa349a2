"""Device-side radiograph preprocessing and training augmentation (SURVEY §8(f)
row 4): the host half of csrc/prep_ops.hip.

Reference: src/data/PretrainDataModule.py:157-198 runs, per sample in CPU
DataLoader workers, HistogramNormalized -> 3-channel repeat ->
CropLargerDimension(0.05) -> PadToSquaredEdgeAverage -> Resized(224, area) ->
NormalizeIntensityd, then for training RandAffined(p .3, translate +-20 px,
shear factors +-5, bilinear, border) -> RandRotated(p .3, +-pi/6) ->
RandFlipd(p .3, spatial axis 0) -> RandZoomd(p .3, 1.1-1.3) ->
RandGaussianNoised(p .5, std U(0, 0.01)).

`preprocess` runs the first chain for a list of decoded images of any size in
four launches.  `Augmenter` draws each sample's parameters on the host (same
probabilities and ranges; a torch.Generator instead of MONAI's RandomState),
composes the four geometric maps into one output->source 2x3 map and runs one
resample + noise kernel over the batch (MONAI resamples after each transform;
see DESIGN.md).
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from . import ops


def preprocess(images: Sequence, size: int, mean: float, std: float, channels: int = 3,
               device="cuda") -> torch.Tensor:
    """Decoded grayscale images [H_i, W_i] (uint8 or float; numpy or torch) ->
    fp32 [n, channels, size, size] on `device`."""
    ts = [torch.as_tensor(np.asarray(im) if not torch.is_tensor(im) else im) for im in images]
    if not ts:
        raise ValueError("preprocess: no images")
    for t in ts:
        if t.dim() != 2 or t.shape[0] < 1 or t.shape[1] < 1:
            raise ValueError(f"preprocess: expected 2-D grayscale images, got {tuple(t.shape)}")
    u8 = all(t.dtype == torch.uint8 for t in ts)
    dt = torch.uint8 if u8 else torch.float32
    flat = torch.cat([t.reshape(-1).to(dt) for t in ts])
    sizes = torch.tensor([t.numel() for t in ts], dtype=torch.int64)
    off = torch.cumsum(sizes, 0) - sizes
    hw = torch.tensor([[t.shape[0], t.shape[1]] for t in ts], dtype=torch.int32)
    n = len(ts)
    src = flat.pin_memory().to(device, non_blocking=True) if flat.device.type == "cpu" else flat.to(device)
    off_d, hw_d = off.to(device), hw.to(device)
    out = torch.empty(n, channels, size, size, dtype=torch.float32, device=device)
    work = torch.empty(n * ops.PREP_WORK_BYTES_PER_IMAGE // 4, dtype=torch.float32, device=device)
    ops.prep_images(src, u8, off_d, hw_d, n, size, mean, std, channels, out, work)
    return out


class Augmenter:
    """RandAffined / RandRotated / RandFlipd / RandZoomd / RandGaussianNoised with
    the reference's settings (PretrainDataModule.py:188-195) as one device pass."""

    def __init__(self, seed: int = 0, p_affine=0.3, p_rotate=0.3, p_flip=0.3, p_zoom=0.3, p_noise=0.5,
                 translate=20.0, shear=5.0, rotate=math.pi / 6, zoom=(1.1, 1.3), noise_std=0.01):
        self.gen = torch.Generator().manual_seed(seed)
        self.p = torch.tensor([p_affine, p_rotate, p_flip, p_zoom, p_noise], dtype=torch.float64)
        self.translate, self.shear, self.rotate = float(translate), float(shear), float(rotate)
        self.zoom, self.noise_std = (float(zoom[0]), float(zoom[1])), float(noise_std)
        self._calls = 0

    def draw(self, B: int) -> dict:
        u = lambda *s: torch.rand(*s, generator=self.gen, dtype=torch.float64)
        on = u(B, 5) < self.p
        return {"on": on, "shear": (u(B, 2) * 2 - 1) * self.shear, "translate": (u(B, 2) * 2 - 1) * self.translate,
                "angle": (u(B) * 2 - 1) * self.rotate, "zoom": self.zoom[0] + u(B) * (self.zoom[1] - self.zoom[0]),
                "noise_std": u(B) * self.noise_std}

    @staticmethod
    def maps(prm: dict) -> torch.Tensor:
        """[B, 2, 3] float64 output->source maps in (row, col), centred:
        zoom (1/z) -> flip (rows) -> rotate -> shear, translation t."""
        on = prm["on"]
        B = on.shape[0]
        M = torch.eye(2, dtype=torch.float64).repeat(B, 1, 1)
        z = torch.where(on[:, 3], 1.0 / prm["zoom"], torch.ones(B, dtype=torch.float64))
        M = M * z[:, None, None]
        M[:, 0, :] = torch.where(on[:, 2, None], -M[:, 0, :], M[:, 0, :])
        th = torch.where(on[:, 1], prm["angle"], torch.zeros(B, dtype=torch.float64))
        c, s = torch.cos(th), torch.sin(th)
        R = torch.stack([torch.stack([c, -s], -1), torch.stack([s, c], -1)], -2)
        M = R @ M
        sh = torch.where(on[:, 0, None], prm["shear"], torch.zeros(B, 2, dtype=torch.float64))
        Sh = torch.stack([torch.stack([torch.ones(B, dtype=torch.float64), sh[:, 0]], -1),
                          torch.stack([sh[:, 1], torch.ones(B, dtype=torch.float64)], -1)], -2)
        M = Sh @ M
        t = torch.where(on[:, 0, None], prm["translate"], torch.zeros(B, 2, dtype=torch.float64))
        return torch.cat([M, t[:, :, None]], -1)

    def __call__(self, x: torch.Tensor, channels: int = 3, mean: float = 0.0, std: float = 1.0,
                 prm: dict | None = None) -> torch.Tensor:
        """x: device fp32 [B, C, H, W] (normalised) or uint8 [B, 1, H, W] (normalised
        on load with mean / std) -> augmented fp32 [B, channels, H, W]."""
        B = x.shape[0]
        prm = self.draw(B) if prm is None else prm
        m = self.maps(prm)
        maps = torch.stack([m[:, 0, 0], m[:, 0, 1], m[:, 0, 2], m[:, 1, 0], m[:, 1, 1], m[:, 1, 2]], -1)
        ns = torch.where(prm["on"][:, 4], prm["noise_std"], torch.zeros(B, dtype=torch.float64))
        dev = x.device
        C = channels if x.shape[1] == 1 else x.shape[1]
        out = torch.empty(B, C, x.shape[2], x.shape[3], dtype=torch.float32, device=dev)
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())
        ops.aug_warp(x.contiguous(), out, maps.float().to(dev), ns.float().to(dev), seed, mean, std)
        self.last_params = prm
        return out
