"""Time the TinyBERT linear GEMMs (bs = 256, T = 40: M = 10240 token rows) one by one.
  python tools/text_gemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
M = 10240


def tm(fn, it=20):
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


for (N, K) in [(936, 312), (312, 312), (1200, 312), (312, 1200)]:
    x = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(N, K, device=dev)
    fl = 2.0 * M * N * K
    t1 = tm(lambda: ops.linear_fwd(x, w, b, y, M, N, K))
    t2 = tm(lambda: ops.linear_dgrad(dy, w, dx, M, K, N))
    t3 = tm(lambda: ops.linear_wgrad(dy, x, dw, M, N, K))
    t4 = tm(lambda: ops.colsum(dy, b, M, N))
    print(f"N={N:5d} K={K:5d}: fwd {t1:6.1f} us {fl / t1 / 1e6:6.1f} TF/s | dgrad {t2:6.1f} us {fl / t2 / 1e6:6.1f} | "
          f"wgrad {t3:6.1f} us {fl / t3 / 1e6:6.1f} | colsum {t4:5.1f} us", flush=True)
