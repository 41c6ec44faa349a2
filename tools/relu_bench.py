"""Time vlp_conv_dgrad_relu with the activation vs its sign-bit mask at the
bs=256 layer-1 (rows kernel) and layer-2 stride-2 (pixel-parity GEMMs) shapes.
  python tools/relu_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for name, (N, H, W, C, Co, S) in {"l1 s1": (256, 128, 128, 64, 64, 1), "l2 s2": (256, 128, 128, 64, 128, 2),
                                   "l2 s1": (256, 64, 64, 128, 128, 1), "l3 s1": (256, 32, 32, 256, 256, 1),
                                   "l4 s1": (256, 16, 16, 512, 512, 1)}.items():
    Ho, Wo = (H - 1) // S + 1, (W - 1) // S + 1
    dy = (torch.randn(N, Ho, Wo, Co, device=dev) * 0.5).to(torch.bfloat16)
    wt = (torch.randn(C, 3, 3, Co, device=dev) * 0.05).to(torch.bfloat16)
    pre = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    act = torch.empty_like(pre)
    m = torch.empty(pre.numel() // 8, dtype=torch.uint8, device=dev)
    ops.bn_add_relu(pre, torch.ones(C, device=dev), torch.zeros(C, device=dev), None, None, None, act, relu_mask=m)
    y = torch.randn_like(pre)
    add = torch.randn_like(pre)
    mu, ist = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    s1 = torch.zeros(64 * C, dtype=torch.float64, device=dev)
    s2 = torch.zeros_like(s1)
    for label, r in (("act", act), ("bits", m)):
        fn = lambda: ops.conv_dgrad_relu(dy, wt, H, W, C, 3, 3, S, 1, r, y, mu, ist, s1, s2, addend=add,  # noqa
                                         stat_rep=64)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:6s} {label:4s} {e0.elapsed_time(e1) / 10 * 1000:8.1f} us")
