"""Time the streaming BN elementwise kernels at the bs=256 ResNet34 sizes against
a plain device copy of the same bytes (torch copy_), to place them against the
achievable HBM rate.
  python tools/ew_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)


def tm(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1000


for (H, C) in [(128, 64), (64, 128), (32, 256), (16, 512)]:
    N = 256
    M = N * H * H
    y = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    idt = torch.randn_like(y)
    out = torch.empty_like(y)
    m = torch.empty(y.numel() // 8, dtype=torch.uint8, device=dev)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    mu, ist, gam = torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.ones(C, device=dev)
    sg = torch.zeros(C, dtype=torch.float64, device=dev)
    sgx = torch.zeros_like(sg)
    dy = torch.empty_like(y)
    B = y.numel() * 2
    tc = tm(lambda: out.copy_(y))
    t0 = tm(lambda: ops.bn_add_relu(y, sc, sh, None, None, None, out))
    t1 = tm(lambda: ops.bn_add_relu(y, sc, sh, idt, None, None, out, relu_mask=m))
    t2 = tm(lambda: ops.bn_bwd_apply(M, C, idt, None, 1, None, (y, mu, ist, gam, sg, sgx, dy), None, None, y))
    print(f"{H:3d}x{H:<3d}x{C:3d}: copy {tc:7.1f} us {2 * B / tc / 1e6:5.2f} TB/s | "
          f"bn_relu {t0:7.1f} us {2 * B / t0 / 1e6:5.2f} | bn_add_relu+mask {t1:7.1f} us {3.0625 * B / t1 / 1e6:5.2f} | "
          f"bn_bwd_apply {t2:7.1f} us {3 * B / t2 / 1e6:5.2f} TB/s", flush=True)
