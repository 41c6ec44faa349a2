"""Golden vectors for the crop + pad stage of the preprocessing chain, made by
running the REFERENCE's own transforms.

Run in the build container (where /root/reference exists):
    python tests/golden/make_prep_golden.py
Writes tests/golden/prep_crop_pad.pt (inputs and outputs only; loaded with
torch.load(weights_only=True)).  The reference never travels to the GPU box.

The two transforms are imported unmodified from
  /root/reference/src/data/transform/CropLargerDimension.py   (:27-57)
  /root/reference/src/data/transform/PadToSquaredEdgeAverage.py (:29-76)
Their only third-party import is `monai.transforms.MapTransform`, a base class
with no arithmetic; MONAI is absent here, so it is replaced by a stand-in that
only stores `keys` (MapTransform.__init__'s role).

Each case is a uint8 grayscale image.  Two fixtures per case:
  raw      : the transforms applied to the image itself (float, 3 channels, as
             the reference's RepeatChanneld output) -- pins oracle/prep.py's
             restatement on CPU;
  eq       : the transforms applied after HistogramNormalized (MONAI absent:
             oracle.prep.histogram_normalize, the restatement that
             vlp_prep_images reproduces bit-exactly) -- the GPU test runs
             vlp_prep_images at S = the padded side (resize = identity),
             mean 0, std 1, and compares with this.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("VLP_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)

from oracle.prep import histogram_normalize  # noqa: E402

# (h, w): h > w with crop and odd pad; w > h; square; the crop that would undershoot
# (clamped to h - w, squares exactly); crop of 0 per side with a 1-pixel pad
CASES = [(64, 41), (41, 64), (48, 48), (80, 61), (61, 80), (62, 60), (61, 60), (37, 90)]


def _stub_monai():
    class MapTransform:
        def __init__(self, keys, allow_missing_keys=False):
            self.keys = (keys,) if isinstance(keys, str) else tuple(keys)
            self.allow_missing_keys = allow_missing_keys
    monai = types.ModuleType("monai")
    tr = types.ModuleType("monai.transforms")
    tr.MapTransform = MapTransform
    monai.transforms = tr
    sys.modules["monai"] = monai
    sys.modules["monai.transforms"] = tr


def _load(name):
    path = os.path.join(REF, "src", "data", "transform", name + ".py")
    spec = importlib.util.spec_from_file_location("ref_" + name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return getattr(mod, name)


def main():
    _stub_monai()
    Crop = _load("CropLargerDimension")
    Pad = _load("PadToSquaredEdgeAverage")
    crop, pad = Crop(keys=["x-ray"]), Pad(keys=["x-ray"])   # maximum_crop_ratio 0.05 (the default the data module uses)
    g = np.random.default_rng(20251128)
    out = {"cases": []}
    for h, w in CASES:
        u8 = g.integers(0, 256, (h, w), dtype=np.uint8)
        # a bright left / right / top / bottom edge band so the edge means differ per side
        u8[:, 0] = np.clip(u8[:, 0].astype(np.int32) // 2 + 128, 0, 255).astype(np.uint8)
        u8[0, :] = np.clip(u8[0, :].astype(np.int32) // 3, 0, 255).astype(np.uint8)
        raw = torch.from_numpy(u8.astype(np.float32))[None].repeat(3, 1, 1)
        eq = torch.from_numpy(histogram_normalize(u8.astype(np.float32)))[None].repeat(3, 1, 1)
        r_raw = pad(crop({"x-ray": raw}))["x-ray"]
        r_eq = pad(crop({"x-ray": eq}))["x-ray"]
        # the three channels are identical (per-channel transforms of a repeated channel): keep one
        assert torch.equal(r_raw[0], r_raw[2]) and torch.equal(r_eq[0], r_eq[2])
        out["cases"].append({"u8": torch.from_numpy(u8), "raw": r_raw[0].clone(), "eq": r_eq[0].clone()})
        print(f"{h}x{w} -> {tuple(r_raw.shape)}")
    torch.save(out, os.path.join(HERE, "prep_crop_pad.pt"))


if __name__ == "__main__":
    main()
