"""Device preprocessing / augmentation (csrc/prep_ops.hip, vlp_amd/augment.py)
against the CPU restatement oracle/prep.py of the reference's transform chain
(src/data/PretrainDataModule.py:157-198; MONAI absent, so parity vs MONAI is
unpinned -- the two transforms the reference defines itself,
CropLargerDimension and PadToSquaredEdgeAverage, are restated line by line).

Shapes cover height > width (crop + left/right pad), width > height (top/bottom),
square, upsampling (image smaller than the output), a constant image (numpy's
widened histogram range) and uint8 images full of values on bin edges.
Tolerances: preprocessing max |diff| <= 2e-4 in normalised units (the
equalisation LUT follows numpy's float32 / float64 arithmetic; the edge means
and window sums differ from torch's only in summation order); warp <= 1e-4
(float32 source coordinates against the fp64 oracle's).
"""
import math

import numpy as np
import pytest
import torch

import oracle.prep as op

pytestmark = pytest.mark.gpu
MEAN, STD = 127.5, 73.9


@pytest.fixture(scope="module")
def aug():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vlp_amd import augment
    return augment


def _images(kind):
    g = np.random.default_rng(3)
    if kind == "u8":
        return [g.integers(0, 256, (300, 200), dtype=np.uint8), g.integers(10, 60, (180, 261), dtype=np.uint8),
                g.integers(0, 256, (128, 128), dtype=np.uint8), g.integers(0, 256, (90, 100), dtype=np.uint8),
                np.full((50, 40), 77, dtype=np.uint8)]
    return [(g.standard_normal((257, 199)) * 300 + 1000).astype(np.float32),
            g.random((151, 240), dtype=np.float32) * 4095, np.full((33, 47), 3.25, dtype=np.float32)]


@pytest.mark.parametrize("kind", ["u8", "f32"])
@pytest.mark.parametrize("S,C", [(128, 3), (64, 1)])
def test_preprocess_vs_oracle(aug, kind, S, C):
    imgs = _images(kind)
    out = aug.preprocess(imgs, S, MEAN, STD, channels=C).cpu()
    for i, im in enumerate(imgs):
        ref = op.preprocess(im, S, MEAN, STD, channels=C)
        err = (out[i] - ref).abs().max().item()
        assert err < 2e-4, (kind, i, im.shape, err)


def test_histogram_equalisation_exact(aug):
    """Square images at S = side skip crop / pad / resize: the kernel output is
    then exactly (eq(x) - mean) / std of the numpy-exact equalisation."""
    g = np.random.default_rng(5)
    imgs = [g.integers(0, 256, (64, 64), dtype=np.uint8), (g.random((64, 64)) * 100).astype(np.float32)]
    for im in imgs:
        out = aug.preprocess([im], 64, 0.0, 1.0, channels=1).cpu()[0, 0].numpy()
        ref = op.histogram_normalize(im)
        assert np.array_equal(out, ref), np.abs(out - ref).max()


def _params(B, gen, on):
    u = lambda *s: torch.rand(*s, generator=gen, dtype=torch.float64)
    return {"on": on, "shear": (u(B, 2) * 2 - 1) * 0.3, "translate": (u(B, 2) * 2 - 1) * 20,
            "angle": (u(B) * 2 - 1) * math.pi / 6, "zoom": 1.1 + u(B) * 0.2, "noise_std": u(B) * 0.01}


def test_augment_warp_vs_oracle(aug):
    B, H, W = 6, 64, 48
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(B, 1, H, W, generator=gen)
    on = torch.tensor([[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 1, 0, 0], [0, 0, 0, 1, 0], [1, 1, 1, 1, 0],
                       [0, 0, 0, 0, 0]], dtype=torch.bool)
    prm = _params(B, gen, on)
    a = aug.Augmenter(seed=1)
    out = a(x.cuda(), channels=3, prm=prm).cpu()
    maps = op.source_maps(prm)
    assert torch.allclose(a.maps(prm), maps)
    ref = op.warp(x.expand(B, 3, H, W).contiguous(), maps)
    assert (out - ref).abs().max().item() < 1e-4
    assert torch.equal(out[5], x[5].expand(3, H, W))        # identity sample untouched


def test_augment_u8_input_normalises_on_load(aug):
    B, H, W = 3, 40, 40
    gen = torch.Generator().manual_seed(2)
    xu = torch.randint(0, 256, (B, 1, H, W), generator=gen, dtype=torch.uint8)
    on = torch.tensor([[1, 1, 0, 1, 0]] * B, dtype=torch.bool)
    prm = _params(B, gen, on)
    a = aug.Augmenter()
    out = a(xu.cuda(), channels=3, mean=MEAN, std=STD, prm=prm).cpu()
    ref = op.warp(((xu.float() - MEAN) / STD).expand(B, 3, H, W).contiguous(), op.source_maps(prm))
    assert (out - ref).abs().max().item() < 1e-4


def test_augment_noise_statistics(aug):
    B, H, W = 2, 256, 256
    x = torch.zeros(B, 1, H, W, device="cuda")
    on = torch.tensor([[0, 0, 0, 0, 1], [0, 0, 0, 0, 0]], dtype=torch.bool)
    prm = _params(B, torch.Generator().manual_seed(0), on)
    prm["noise_std"] = torch.tensor([0.5, 0.5], dtype=torch.float64)
    out = aug.Augmenter(seed=4)(x, channels=3, prm=prm).cpu()
    n = out[0]
    assert abs(n.mean().item()) < 8e-3 and abs(n.std().item() - 0.5) < 8e-3
    c = torch.corrcoef(torch.stack([n[0].flatten(), n[1].flatten()]))[0, 1].item()
    assert abs(c) < 0.02                                     # independent per channel, as MONAI's
    assert torch.equal(out[1], torch.zeros(3, H, W))         # noise off -> untouched


def test_augment_draw_protocol(aug):
    """Probabilities and ranges of the reference's transforms (PretrainDataModule.py:188-195)."""
    a = aug.Augmenter(seed=9)
    p = a.draw(20000)
    rate = p["on"].double().mean(0)
    assert torch.allclose(rate, torch.tensor([0.3, 0.3, 0.3, 0.3, 0.5], dtype=torch.float64), atol=0.015)
    assert p["translate"].abs().max() <= 20 and p["shear"].abs().max() <= 5
    assert p["angle"].abs().max() <= math.pi / 6 and p["zoom"].min() >= 1.1 and p["zoom"].max() <= 1.3
    assert p["noise_std"].max() <= 0.01


def _pad_mask(ref_shape, hw):
    """True on the padded columns (h > w after the crop) or rows (w > h)."""
    side = ref_shape[-1]
    m = torch.zeros(ref_shape, dtype=torch.bool)
    h, w = hw
    if h == w:
        return m
    # the crop leaves the larger side equal to `side`; the shorter one is padded
    short = w if h > w else h
    lo = (side - short) // 2
    idx = list(range(lo)) + list(range(lo + short, side))
    if h > w:
        m[:, idx] = True
    else:
        m[idx, :] = True
    return m


def test_crop_pad_vs_reference_transforms(aug):
    """vlp_prep_images' crop + pad stage against the reference's own
    CropLargerDimension / PadToSquaredEdgeAverage (tests/golden/make_prep_golden.py
    ran them on the equalised images): S = the padded side, so the area resize is
    the identity and mean / std are 0 / 1.  The image pixels must be bit-exact (the
    equalisation is numpy-exact and the crop moves no values); the padded columns
    or rows are edge means, summed in another order than torch's: <= 1e-4 of the
    0..255 range."""
    import os
    gd = torch.load(os.path.join(os.path.dirname(__file__), "golden", "prep_crop_pad.pt"), weights_only=True)
    assert len(gd["cases"]) == 8
    for c in gd["cases"]:
        u8, ref = c["u8"].numpy(), c["eq"]
        S = ref.shape[-1]
        out = aug.preprocess([u8], S, 0.0, 1.0, channels=1).cpu()[0, 0]
        assert out.shape == ref.shape
        pm = _pad_mask(ref.shape, u8.shape)
        assert torch.equal(out[~pm], ref[~pm]), (u8.shape, (out - ref).abs()[~pm].max().item())
        if pm.any():
            assert (out - ref).abs()[pm].max().item() <= 255 * 1e-4, u8.shape
