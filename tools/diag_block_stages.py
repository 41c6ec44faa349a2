"""Per-stage forward comparison of one HIP bf16 BasicBlock range against the
float64 bf16-storage emulation of tests/test_gpu_blocks.py: for every stored
tensor (y1, a1, y2, yd, out) the fraction of elements whose bf16 value differs
and the largest difference in bf16 ulps.  An exact bf16-storage implementation
differs only where an fp32 sum lands within rounding of a bf16 tie.

    python tools/diag_block_stages.py [layer1|layer2|layer3|layer4] [bs]
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
from tests.test_gpu_blocks import RANGES  # noqa: E402
from vlp_amd.resnet34 import ResNet34Tower  # noqa: E402


def ulps(a, b):
    """|a - b| in units of b's bf16 spacing (a, b bf16-valued)."""
    a, b = a.double(), b.double()
    e = torch.floor(torch.log2(b.abs().clamp_min(1e-30)))
    return (a - b).abs() / torch.pow(2.0, e - 7)


def main(name="layer1", bs=32):
    lo, hi, (H, W, C) = RANGES[name]
    dev = torch.device("cuda")
    t = ResNet34Tower(compute_dtype="bf16", device=dev)
    g = torch.Generator().manual_seed(500 + lo)
    P = {}
    blocks = []
    for bi in range(lo, hi):
        pre, has_ds = t._blocks[bi]
        blocks.append((pre, t._convs[pre + ".conv1"].S, has_ds))
        for k in [pre + ".conv1", pre + ".conv2"] + ([pre + ".downsample.0"] if has_ds else []):
            c = t._convs[k]
            P[k + ".weight"] = (torch.randn(c.Co, c.C, c.KH, c.KW, generator=g) * (2.0 / (c.Co * 9)) ** 0.5
                                ).to(torch.bfloat16).float()
        for k in [pre + ".bn1", pre + ".bn2"] + ([pre + ".downsample.1"] if has_ds else []):
            P[k + ".weight"] = torch.empty(t._bns[k].C).uniform_(0.3, 1.0, generator=g)
            P[k + ".bias"] = torch.empty(t._bns[k].C).uniform_(-0.1, 0.1, generator=g)
    with torch.no_grad():
        for k, v in P.items():
            t.arena.view(k).copy_(v)
    x = torch.relu(torch.randn(bs, C, H, W, generator=g)).to(torch.bfloat16)
    out, saved = t.run_block_range_forward(x.permute(0, 2, 3, 1).contiguous().to(dev), lo, hi)
    torch.cuda.synchronize()
    Pd = {k: v.to(dev, torch.float64) for k, v in P.items()}
    r = lambda v: v.to(torch.bfloat16).to(torch.float64)  # noqa: E731
    h = x.to(dev, torch.float64)
    for (pre, stride, has_ds), blk in zip(blocks, saved["blocks"][lo:]):
        def bn(v, k):
            return F.batch_norm(v, None, None, Pd[k + ".weight"], Pd[k + ".bias"], True, 0.1, 1e-5)
        hb = {k: (blk[k].permute(0, 3, 1, 2).double() if blk.get(k) is not None else None)
              for k in ("y1", "a1", "y2", "yd", "out")}
        # every stage from HIP's own stored inputs: each line judges one kernel
        st = {}
        st["y1"] = r(F.conv2d(h, Pd[pre + ".conv1.weight"], stride=stride, padding=1))
        st["a1"] = r(F.relu(bn(hb["y1"], pre + ".bn1")))
        st["y2"] = r(F.conv2d(hb["a1"], Pd[pre + ".conv2.weight"], padding=1))
        z = bn(hb["y2"], pre + ".bn2")
        if has_ds:
            st["yd"] = r(F.conv2d(h, Pd[pre + ".downsample.0.weight"], stride=stride))
            sc = bn(hb["yd"], pre + ".downsample.1")
        else:
            sc = h
        st["out"] = r(F.relu(z + sc))
        for k, v in st.items():
            hv = blk[k].permute(0, 3, 1, 2).double()
            u = ulps(hv, v)
            nz = (v != 0)
            print(f"{pre:10s} {k:4s} differ {((hv != v).double().mean().item()):.3e}  max ulp "
                  f"{u[nz].max().item() if nz.any() else 0:.1f}  rel-L2 "
                  f"{((hv - v).norm() / v.norm()).item():.2e}")
        # continue the chain from HIP's own output so each block is judged on its own
        h = blk["out"].permute(0, 3, 1, 2).double()
        # (stats) compare HIP's BN coefficients are implicit in a1 / out


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "layer1", int(sys.argv[2]) if len(sys.argv) > 2 else 32)
