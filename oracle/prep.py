"""ORACLE (test infrastructure): CPU restatement of the reference's image
preprocessing and augmentation (src/data/PretrainDataModule.py:157-198 and the
transforms it composes), the checker for csrc/prep_ops.hip.

Pre-normalisation chain (:157-178), per image, grayscale [H, W]:
  HistogramNormalized   MONAI 1.x histogram_normalize(num_bins=256, min=0, max=255):
                        np.histogram over [img.min(), img.max()], cumsum,
                        rescale_array to [0, 255], np.interp(img, bins[:-1], cum)
  CropLargerDimension   src/data/transform/CropLargerDimension.py:27-57
  PadToSquaredEdgeAverage src/data/transform/PadToSquaredEdgeAverage.py:29-76
  Resized(224)          MONAI Resize, default mode "area" = torch
                        F.interpolate(mode="area") = adaptive average pooling
  NormalizeIntensityd   (x - mean) / std (:288)
Augmentations (:186-198), applied after the normalisation (:291-295):
  RandAffined(p .3, translate +-20 px, shear factors +-5, bilinear, border),
  RandRotated(p .3, +-pi/6), RandFlipd(p .3, spatial axis 0),
  RandZoomd(p .3, 1.1-1.3, keep_size), RandGaussianNoised(p .5, std U(0, .01)).

MONAI (monai==1.x, environment.yaml) is not installed, so its transforms are
restated from their published algorithm -- PARITY UNPINNED against MONAI; the
two transforms the reference defines itself are restated line by line.  The
augmentation oracle is the continuous composition of the four geometric maps
sampled once (bilinear, border clamp), which is what the HIP kernel computes;
MONAI resamples after every transform (up to four bilinear passes) -- a
documented deviation, the parameter distributions are the same.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def rescale_array(arr, minv=0.0, maxv=1.0, dtype=np.float32):
    """MONAI rescale_array (transforms/utils.py): computed in float32."""
    arr = np.asarray(arr).astype(dtype)
    mina, maxa = arr.min(), arr.max()
    if mina == maxa:
        return arr * minv
    norm = (arr - mina) / (maxa - mina)
    return (norm * (maxv - minv)) + minv


def histogram_normalize(img, num_bins=256, minv=0, maxv=255):
    """MONAI histogram_normalize (transforms/utils.py) on a float32 array: the
    histogram range is the array's own float32 min / max (float32 bin edges)."""
    a = np.asarray(img, dtype=np.float32)
    hist, bins = np.histogram(a, num_bins, [a.min(), a.max()])
    cum = rescale_array(hist.cumsum(), minv, maxv)
    out = np.interp(a.flatten(), bins[:-1], cum)
    return out.reshape(a.shape).astype(np.float32)


def crop_larger_dimension(img, maximum_crop_ratio=0.05):
    """CropLargerDimension.__call__ :34-54 on [C, H, W]."""
    c, h, w = img.shape
    if h == w:
        return img
    if h > w:
        crop = int(h * maximum_crop_ratio)
        if h - crop < w:
            crop = h - w
        e = crop // 2
        return img[:, e:h - e, :]
    crop = int(w * maximum_crop_ratio)
    if w - crop < h:
        crop = w - h
    e = crop // 2
    return img[:, :, e:w - e]


def pad_to_square_edge_average(img):
    """PadToSquaredEdgeAverage.__call__ :36-73 on [C, H, W] (torch)."""
    c, h, w = img.shape
    if h == w:
        return img
    diff = abs(h - w)
    if h > w:
        lp, rp = diff // 2, diff - diff // 2
        le = img[:, :, 0].float().mean(dim=1)
        re = img[:, :, -1].float().mean(dim=1)
        return torch.cat([le[:, None, None].expand(-1, h, lp), img, re[:, None, None].expand(-1, h, rp)], dim=2)
    tp, bp = diff // 2, diff - diff // 2
    te = img[:, 0, :].float().mean(dim=1)
    be = img[:, -1, :].float().mean(dim=1)
    return torch.cat([te[:, None, None].expand(-1, tp, w), img, be[:, None, None].expand(-1, bp, w)], dim=1)


def preprocess(img_hw, size, mean, std, channels=3):
    """The pre-normalisation chain + NormalizeIntensityd for one grayscale image
    [H, W] (uint8 or float): returns fp32 [channels, size, size]."""
    eq = torch.from_numpy(histogram_normalize(np.asarray(img_hw, dtype=np.float32)))[None]
    eq = eq.repeat(channels, 1, 1)
    x = pad_to_square_edge_average(crop_larger_dimension(eq))
    x = F.interpolate(x[None], size=(size, size), mode="area")[0]
    return (x - mean) / std


# ---------------- augmentation ----------------
def draw_params(B, gen, p_affine=0.3, p_rotate=0.3, p_flip=0.3, p_zoom=0.3, p_noise=0.5, translate=20.0,
                shear=5.0, rotate=math.pi / 6, zoom=(1.1, 1.3), noise_std=0.01):
    """Per-sample parameters with the reference's probabilities and ranges
    (PretrainDataModule.py:188-195); torch.Generator draws, not MONAI's RNG."""
    u = lambda *s: torch.rand(*s, generator=gen, dtype=torch.float64)
    on = u(B, 5) < torch.tensor([p_affine, p_rotate, p_flip, p_zoom, p_noise], dtype=torch.float64)
    sh = (u(B, 2) * 2 - 1) * shear
    tr = (u(B, 2) * 2 - 1) * translate
    th = (u(B) * 2 - 1) * rotate
    z = zoom[0] + u(B) * (zoom[1] - zoom[0])
    ns = u(B) * noise_std
    return {"on": on, "shear": sh, "translate": tr, "angle": th, "zoom": z, "noise_std": ns}


def source_maps(prm):
    """[B, 2, 3] (row, col) maps: source = M @ (out - centre) + centre + t, the
    composition zoom -> flip -> rotate -> affine of the output-to-input maps
    (MONAI applies affine, rotate, flip, zoom in that order to the image)."""
    on = prm["on"]
    B = on.shape[0]
    out = torch.zeros(B, 2, 3, dtype=torch.float64)
    for b in range(B):
        M = torch.eye(2, dtype=torch.float64)
        if on[b, 3]:
            M = M / prm["zoom"][b]
        if on[b, 2]:
            M = torch.tensor([[-1.0, 0.0], [0.0, 1.0]], dtype=torch.float64) @ M
        if on[b, 1]:
            c, s = math.cos(prm["angle"][b]), math.sin(prm["angle"][b])
            M = torch.tensor([[c, -s], [s, c]], dtype=torch.float64) @ M
        t = torch.zeros(2, dtype=torch.float64)
        if on[b, 0]:
            Sh = torch.tensor([[1.0, prm["shear"][b, 0]], [prm["shear"][b, 1], 1.0]], dtype=torch.float64)
            M = Sh @ M
            t = prm["translate"][b].clone()
        out[b, :, :2] = M
        out[b, :, 2] = t
    return out


def warp(x, maps):
    """Bilinear resample of x [B, C, H, W] at source = M (p - c) + c + t, border
    clamp (grid_sample padding_mode="border")."""
    B, C, H, W = x.shape
    cy, cx = (H - 1) / 2.0, (W - 1) / 2.0
    r = torch.arange(H, dtype=torch.float64)[:, None].expand(H, W) - cy
    q = torch.arange(W, dtype=torch.float64)[None, :].expand(H, W) - cx
    out = torch.empty_like(x)
    for b in range(B):
        M = maps[b]
        sr = (M[0, 0] * r + M[0, 1] * q + M[0, 2] + cy).clamp(0, H - 1)
        sc = (M[1, 0] * r + M[1, 1] * q + M[1, 2] + cx).clamp(0, W - 1)
        r0, c0 = sr.floor().long().clamp(max=H - 2 if H > 1 else 0), sc.floor().long().clamp(max=W - 2 if W > 1 else 0)
        fr, fc = sr - r0, sc - c0
        r1, c1 = (r0 + 1).clamp(max=H - 1), (c0 + 1).clamp(max=W - 1)
        img = x[b].double()
        v = (img[:, r0, c0] * (1 - fr) * (1 - fc) + img[:, r0, c1] * (1 - fr) * fc
             + img[:, r1, c0] * fr * (1 - fc) + img[:, r1, c1] * fr * fc)
        out[b] = v.to(x.dtype)
    return out
