"""Time the streaming BN elementwise kernels at the bs=256 layer-1 size
(bn_add_relu with identity + mask bits, bn_bwd_apply one side).
  python tools/ew_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
N, H, W, C = 256, 128, 128, 64
M = N * H * W
y = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
idt = torch.randn_like(y)
out = torch.empty_like(y)
m = torch.empty(y.numel() // 8, dtype=torch.uint8, device=dev)
sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
mu, ist, gam = torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.ones(C, device=dev)
sg = torch.zeros(C, dtype=torch.float64, device=dev)
sgx = torch.zeros_like(sg)
dy = torch.empty_like(y)


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


t1 = tm(lambda: ops.bn_add_relu(y, sc, sh, idt, None, None, out, relu_mask=m))
t2 = tm(lambda: ops.bn_bwd_apply(M, C, idt, None, 1, None, (y, mu, ist, gam, sg, sgx, dy), None, None, y))
print(f"bn_add_relu {t1:7.1f} us ({4 * y.numel() * 2 / t1 / 1e6:5.2f} TB/s)  "
      f"bn_bwd_apply {t2:7.1f} us ({3 * y.numel() * 2 / t2 / 1e6:5.2f} TB/s)")
