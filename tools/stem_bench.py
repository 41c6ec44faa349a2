"""Stem kernels at the bench shape (bs = 256, 512^2, bf16): the unfused path
(K = 64 stem GEMM writing y0 + max-pool forward over y0, max-pool backward-apply
reading y0) against the fused one (vlp_stem1_pool_fwd + the pooled BN/ReLU pass,
vlp_stem1_route_bwd).  Median of HIP-event timings per kernel, us.

  python tools/stem_bench.py [--batch 256] [--size 512] [--iters 10]
(fused_bwd_all_us: vlp_stem1_bwd_fused, routing + BN backward + weight gradient in
one pass, the path the step runs; fused_route_bwd_us + stem_wgrad_us: the two-pass form)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]

import torch  # noqa: E402


def timeit(fn, iters):
    ts = []
    for _ in range(iters + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[2:])
    return round(ts[len(ts) // 2], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from vlp_amd import ops
    N, H = a.batch, a.size
    W = H
    dev = "cuda"
    bf = torch.bfloat16
    Ho, Wo, Hp, Wp1 = ops.stem1_geom(H, W)
    Hq, Wq = Ho // 2, Wo // 2
    xu = torch.randint(0, 256, (N, 1, H, W), dtype=torch.uint8, device=dev)
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.05
    gamma = torch.randn(64, device=dev)
    xs = torch.empty(4, N, Hp, Wp1, dtype=bf, device=dev)
    ops.stem1_prep_u8(xu, xs, 127.5, 73.9)
    wp1 = torch.empty(64, 64, dtype=bf, device=dev)
    ops.pack_stem1(w, wp1)
    rep = 64
    s = torch.zeros(rep, 64, dtype=torch.float64, device=dev)
    ss = torch.zeros_like(s)
    sc = torch.rand(64, device=dev) * gamma.sign()
    sh = torch.randn(64, device=dev)
    mean, istd = torch.randn(64, device=dev), torch.rand(64, device=dev) + 0.5
    sg = torch.randn(rep, 64, dtype=torch.float64, device=dev)
    sgx = torch.randn(rep, 64, dtype=torch.float64, device=dev)
    res = {"shape": f"N={N} {H}x{W} -> y0 {Ho}x{Wo}x64, pooled {Hq}x{Wq}x64"}
    # unfused
    y0 = torch.empty(N, Ho, Wo, 64, dtype=bf, device=dev)
    p = torch.empty(N, Hq, Wq, 64, dtype=bf, device=dev)
    idx = torch.empty(N, Hq, Wq, 64, dtype=torch.uint8, device=dev)
    yarg = torch.empty_like(p)
    pm = torch.empty(p.numel() // 8, dtype=torch.uint8, device=dev)
    dy0 = torch.empty_like(y0)
    dp = torch.randn(N, Hq, Wq, 64, device=dev).to(bf)
    res["unfused_stem_fwd_us"] = timeit(lambda: ops.stem1_fwd(xs, wp1, N, H, W, y0, s, ss, rep), a.iters)
    res["unfused_maxpool_fwd_us"] = timeit(lambda: ops.maxpool_fwd(y0, sc, sh, p, idx, yarg, relu_mask=pm), a.iters)
    res["unfused_maxpool_bwd_apply_us"] = timeit(
        lambda: ops.maxpool_bwd_apply(dp, idx, y0, sc, sh, mean, istd, gamma, sg[0], sgx[0], dy0), a.iters)
    del y0
    # fused
    res["fused_pool_fwd_us"] = timeit(
        lambda: ops.stem1_pool_fwd(xs, wp1, gamma, yarg, idx, N, H, W, s, ss, rep), a.iters)
    res["pooled_bn_relu_us"] = timeit(lambda: ops.bn_add_relu(yarg, sc, sh, None, None, None, p, relu_mask=pm),
                                      a.iters)
    res["fused_route_bwd_us"] = timeit(
        lambda: ops.stem1_route_bwd(xs, wp1, dp, idx, sc, sh, mean, istd, gamma, sg[0], sgx[0], dy0, N, H, W),
        a.iters)
    gw = torch.empty(64, 3, 7, 7, device=dev)
    res["stem_wgrad_us"] = timeit(lambda: ops.stem1_wgrad_into(dy0, xs, N, H, W, gw), a.iters)
    res["fused_bwd_all_us"] = timeit(
        lambda: ops.stem1_bwd_fused_into(xs, wp1, dp, idx, mean, istd, gamma, sg[0], sgx[0], N, H, W, gw), a.iters)
    res["stem1_prep_u8_us"] = timeit(lambda: ops.stem1_prep_u8(xu, xs, 127.5, 73.9), a.iters)
    res["unfused_total_us"] = round(res["unfused_stem_fwd_us"] + res["unfused_maxpool_fwd_us"]
                                    + res["unfused_maxpool_bwd_apply_us"], 1)
    res["fused_total_us"] = round(res["fused_pool_fwd_us"] + res["pooled_bn_relu_us"] + res["fused_route_bwd_us"], 1)
    res["unfused_with_wgrad_us"] = round(res["unfused_total_us"] + res["stem_wgrad_us"], 1)
    res["fused_one_pass_bwd_total_us"] = round(res["fused_pool_fwd_us"] + res["pooled_bn_relu_us"]
                                               + res["fused_bwd_all_us"], 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
