"""Flash-attention kernels of the NesT tower at the bs=128, 512x512 level shapes
(BT = B * blocks, H heads of 32, N = 1024 tokens per block).
  python tools/nest_attn_bench.py [--levels 0,1,2] [--iters 5]"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

LEVELS = {0: (128 * 16, 3), 1: (128 * 4, 6), 2: (128, 12)}


def tm(fn, it):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--levels", default="0,1,2")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--N", type=int, default=1024)
    a = ap.parse_args()
    for lv in [int(v) for v in a.levels.split(",")]:
        BT, H = LEVELS[lv]
        N, C = a.N, 32 * H
        qkv = (torch.randn(BT * N, 3 * C, device="cuda") * 0.5).to(torch.bfloat16)
        out = torch.empty(BT * N, C, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(BT * H * N, device="cuda")
        do = torch.randn_like(out)
        dqkv = torch.empty_like(qkv)
        delta = torch.empty_like(lse)
        s = 1 / math.sqrt(32)
        tf = tm(lambda: ops.nest_attn_fwd(qkv, out, lse, BT, H, N, s), a.iters)
        tb = tm(lambda: ops.nest_attn_bwd(qkv, out, do, lse, delta, dqkv, BT, H, N, s), a.iters)
        f = 4.0 * BT * H * N * N * 32
        print(f"level {lv} BT={BT} H={H} N={N}: fwd {tf:8.1f} us {f / tf / 1e6:6.1f} TF/s | "
              f"bwd {tb:8.1f} us {2.5 * f / tb / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
