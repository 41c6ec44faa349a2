"""Micro-benchmark of single implicit-GEMM conv launches at the bs=256, 512x512
ResNet34 shapes (for A/B work on the GEMM engine and for focused rocprofv3
PMC runs).

  python tools/conv_bench.py [--ops fwd,dgrad,wgrad] [--layers l1,l2,l3,l4] [--iters 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]

import torch  # noqa: E402
from vlp_amd import ops  # noqa: E402

# (name, N, H, W, C, Co, KH, KW, S, P) for the dominant 3x3 stride-1 convs
LAYERS = {
    "l1": (256, 128, 128, 64, 64, 3, 3, 1, 1),
    "l2": (256, 64, 64, 128, 128, 3, 3, 1, 1),
    "l3": (256, 32, 32, 256, 256, 3, 3, 1, 1),
    "l4": (256, 16, 16, 512, 512, 3, 3, 1, 1),
    # stride-2 stage entries (conv1 of layer2.0 / 3.0 / 4.0; dgrad_relu_ds folds the 1x1/2 downsample)
    "l2s": (256, 128, 128, 64, 128, 3, 3, 2, 1),
    "l3s": (256, 64, 64, 128, 256, 3, 3, 2, 1),
    "l4s": (256, 32, 32, 256, 512, 3, 3, 2, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--layers", default="l1,l2,l3,l4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--gemm", action="store_true")
    ap.add_argument("--text", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = {}
    for ln in [l for l in args.layers.split(",") if l]:
        N, H, W, C, Co, KH, KW, S, P = LAYERS[ln]
        Ho, Wo = (H + 2 * P - KH) // S + 1, (W + 2 * P - KW) // S + 1
        x = (torch.randn(N, H, W, C, device=dev) * 0.5).to(torch.bfloat16)
        dy = (torch.randn(N, Ho, Wo, Co, device=dev) * 0.5).to(torch.bfloat16)
        wp = (torch.randn(Co, KH, KW, C, device=dev) * 0.05).to(torch.bfloat16)
        wt = wp.permute(3, 1, 2, 0).contiguous()
        s1 = torch.zeros(64 * Co, dtype=torch.float64, device=dev)
        s2 = torch.zeros_like(s1)
        dws = torch.zeros(Co, KH * KW * C, device=dev)
        flop0 = 2.0 * N * Ho * Wo * Co * C * KH * KW
        for op in args.ops.split(","):
            flop = flop0
            if op == "fwd":
                fn = lambda: ops.conv_fwd(x, wp, Co, KH, KW, S, P, stat_sum=s1, stat_sumsq=s2, stat_rep=64)  # noqa: E731
            elif op == "fwd_bn":       # BN-apply + ReLU of the input on load (in_scale / in_shift)
                xsc, xsh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
                fn = lambda: ops.conv_fwd(x, wp, Co, KH, KW, S, P, in_scale=xsc, in_shift=xsh,  # noqa: E731
                                          stat_sum=s1, stat_sumsq=s2, stat_rep=64)
            elif op == "fwd_act":      # layer 1: bn + ReLU in the rows kernel's ring, activation written out
                xsc, xsh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
                xa = torch.empty_like(x)
                fn = lambda: ops.conv_fwd_act(x, wp, Co, KH, KW, S, P, xsc, xsh, xa, s1, s2, stat_rep=64)  # noqa: E731
            elif op == "pass_fwd":     # the unfused pair: bn_add_relu pass, then the forward
                xsc, xsh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
                xa = torch.empty_like(x)

                def fn():
                    ops.bn_add_relu(x, xsc, xsh, None, None, None, xa)
                    ops.conv_fwd(xa, wp, Co, KH, KW, S, P, stat_sum=s1, stat_sumsq=s2, stat_rep=64)
            elif op == "dgrad":
                fn = lambda: ops.conv_dgrad(dy, wt, H, W, C, KH, KW, S, P)  # noqa: E731
            elif op == "dgrad_bn":     # + ReLU-mask of bn(y), BN backward sums (EpiDgradBN)
                yb = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                cf = [torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1,
                      torch.zeros(C, device=dev), torch.ones(C, device=dev)]
                t1, t2 = torch.zeros(64 * C, dtype=torch.float64, device=dev), torch.zeros(64 * C, dtype=torch.float64, device=dev)
                fn = lambda: ops.conv_dgrad(dy, wt, H, W, C, KH, KW, S, P, y_bn=yb, bn=tuple(cf),  # noqa: E731
                                            stat1=t1, stat2=t2, stat_rep=64)
            elif op == "dgrad_relu":   # + addend, ReLU bit mask, BN backward sums (EpiDgradRelu<bits>)
                yb = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                ad = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                mk = torch.randint(0, 255, (N * H * W * C // 8,), dtype=torch.uint8, device=dev)
                mu, ist = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                t1, t2 = torch.zeros(64 * C, dtype=torch.float64, device=dev), torch.zeros(64 * C, dtype=torch.float64, device=dev)
                fn = lambda: ops.conv_dgrad_relu(dy, wt, H, W, C, KH, KW, S, P, mk, yb, mu, ist, t1, t2,  # noqa: E731
                                                 addend=ad, stat_rep=64)
            elif op == "dgrad_bn_act":   # layer 1: dy = k*g + b*y + c formed in the ring + EpiDgradBN
                coef = torch.randn(3, Co, device=dev) * 0.1
                yin = (torch.randn(N, Ho, Wo, Co, device=dev)).to(torch.bfloat16)
                dyo = torch.empty_like(dy)
                yb = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                bn = (torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1, torch.zeros(C, device=dev),
                      torch.ones(C, device=dev))
                t1, t2 = torch.zeros(64 * C, dtype=torch.float64, device=dev), torch.zeros(64 * C, dtype=torch.float64, device=dev)
                fn = lambda: ops.conv_dgrad_bn_act(dy, yin, coef, dyo, wt, H, W, C, KH, KW, S, P, yb, bn, t1, t2,  # noqa: E731
                                                   stat_rep=64)
            elif op == "dgrad_relu_act":  # layer 1: ring-formed dy + addend, ReLU bits, BN sums
                coef = torch.randn(3, Co, device=dev) * 0.1
                yin = (torch.randn(N, Ho, Wo, Co, device=dev)).to(torch.bfloat16)
                dyo = torch.empty_like(dy)
                yb = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                ad = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                mk = torch.randint(0, 255, (N * H * W * C // 8,), dtype=torch.uint8, device=dev)
                mu, ist = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                t1, t2 = torch.zeros(64 * C, dtype=torch.float64, device=dev), torch.zeros(64 * C, dtype=torch.float64, device=dev)
                fn = lambda: ops.conv_dgrad_relu_act(dy, yin, coef, dyo, wt, H, W, C, KH, KW, S, P, mk, yb, mu,  # noqa: E731
                                                     ist, t1, t2, addend=ad, stat_rep=64)
            elif op == "dgrad_relu_ds":   # stride-2 entry: conv1 + downsample data gradients in one GEMM
                pair = (torch.randn(2, N, Ho, Wo, Co, device=dev) * 0.5).to(torch.bfloat16)
                wpair = torch.empty(C * KH * KW * Co + C * Co, dtype=torch.bfloat16, device=dev)
                wpair[:C * KH * KW * Co].copy_(wt.reshape(-1))
                wpair[C * KH * KW * Co:].normal_(0, 0.05)
                wt1 = wpair[:C * KH * KW * Co].view(C, KH, KW, Co)
                wtd = wpair[C * KH * KW * Co:].view(C, 1, 1, Co)
                act = torch.relu(torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                yb = (torch.randn(N, H, W, C, device=dev)).to(torch.bfloat16)
                mu, ist = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                t1, t2 = torch.zeros(64 * C, dtype=torch.float64, device=dev), torch.zeros(64 * C, dtype=torch.float64, device=dev)
                fn = lambda: ops.conv_dgrad_relu_ds(pair[0], pair[1], wt1, wtd, H, W, C, KH, KW, S, P, act, yb,  # noqa: E731
                                                    mu, ist, t1, t2, stat_rep=64)
                flop = 2.0 * N * Ho * Wo * Co * C * (KH * KW + 1)
            elif op == "wgrad_a":      # the same atomic-epilogue engine on dy (MN operand)
                gw0 = torch.zeros(Co * KH * KW * C, device=dev)
                fn = lambda: ops.conv_wgrad(dy, x, KH, KW, S, P, gw0)  # noqa: E731
            else:
                gw = torch.empty(Co, C, KH, KW, device=dev)
                fn = lambda: ops.conv_wgrad_into(dy, x, KH, KW, S, P, gw)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            res[f"{op}_{ln}"] = {"us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}
            print(f"{op:6s} {ln}: {us:9.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)
    if args.gemm:
        # plain GEMMs with the three operand layouts at a conv-like size:
        # fwd (K-contig x K-contig), dgrad (K-contig x MN-contig), wgrad (MN x MN)
        M, N, K = 65536, 512, 4608
        flop = 2.0 * M * N * K
        a = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dyb = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device=dev)
        cases = {
            "gemm_kk": (lambda: ops.linear_fwd(a, w, None, y, M, N, K), 2.0 * M * N * K),
            "gemm_kmn": (lambda: ops.linear_dgrad(dyb, w, dx, M, K, N), 2.0 * M * N * K),
            "gemm_mnmn": (lambda: ops.linear_wgrad(dyb, a, dw, M, N, K), 2.0 * M * N * K),
        }
        for name, (fn, flop) in cases.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            res[name] = {"us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}
            print(f"{name:9s}: {us:9.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)
    if args.text:
        # TinyBERT weight gradients: dW[Nout][Kin] = dy^T x over M = B*T tokens
        for (M, Nout, Kin) in [(10240, 936, 312), (10240, 1200, 312), (10240, 312, 1200), (10240, 312, 312)]:
            dyb = (torch.randn(M, Nout, device=dev) * 0.1).to(torch.bfloat16)
            xb = (torch.randn(M, Kin, device=dev) * 0.1).to(torch.bfloat16)
            dw = torch.zeros(Nout, Kin, device=dev)
            fn = lambda: ops.linear_wgrad(dyb, xb, dw, M, Nout, Kin)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            flop = 2.0 * M * Nout * Kin
            print(f"linw {Nout}x{Kin}: {us:9.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
