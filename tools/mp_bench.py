"""Stem maxpool passes at bs=256, 512x512 in isolation (preallocated tensors):
maxpool_bwd (BN sums of the routed gradient), maxpool_bwd_apply (dy), maxpool_fwd."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
N, H, W, C = 256, 256, 256, 64
y0 = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
dp = torch.randn(N, H // 2, W // 2, C, device=dev).to(torch.bfloat16)
idx = torch.randint(0, 9, (N, H // 2, W // 2, C), device=dev, dtype=torch.uint8)
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
mu, ist, gam = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev)
s1 = torch.zeros(64 * C, dtype=torch.float64, device=dev)
s2 = torch.zeros_like(s1)
dy = torch.empty_like(y0)


def tm(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


print("maxpool_bwd (sums)  %.1f us" % tm(lambda: ops.maxpool_bwd(dp, idx, y0, sc, sh, mu, ist, s1, s2, stat_rep=64)))
print("maxpool_bwd_apply   %.1f us" % tm(lambda: ops.maxpool_bwd_apply(dp, idx, y0, sc, sh, mu, ist, gam, s1[:C], s2[:C], dy)))
po = torch.empty_like(dp)
pidx = torch.empty_like(idx)
yarg = torch.empty_like(dp)
rmask = torch.empty(dp.numel() // 8, dtype=torch.uint8, device=dev)
print("maxpool_fwd         %.1f us" % tm(lambda: ops.maxpool_fwd(y0, sc, sh, po, pidx, yarg, rmask)))
print("copy y0->dy (ref)   %.1f us" % tm(lambda: dy.copy_(y0)))
