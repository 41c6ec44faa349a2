"""Time NesT-Small's per-layer kernels one by one at BASELINE configs[3]
(bs = 128, 512^2: level token rows M = 2.1 M / 524 k / 131 k at C = 96 / 192 / 384),
with the algorithmic FLOP and HBM-byte rates of each.

  python tools/nest_gemm_bench.py [--batch 128] [--levels 0,1,2] [--out F.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402


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
    return e0.elapsed_time(e1) / it * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--levels", default="0,1,2")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from vlp_amd import ops
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    res = []
    for lvl in [int(v) for v in a.levels.split(",")]:
        C = 96 << lvl
        M = a.batch * (128 >> lvl) ** 2
        F = 4 * C
        r = lambda *s: (torch.randn(*s, device=dev) * 0.1).to(bf)  # noqa: E731
        x, res_in = r(M, C), r(M, C)
        hid = r(M, F)
        out_c, out_3c = torch.empty(M, C, dtype=bf, device=dev), torch.empty(M, 3 * C, dtype=bf, device=dev)
        pre, act = torch.empty(M, F, dtype=bf, device=dev), torch.empty(M, F, dtype=bf, device=dev)
        w3, wc, w1, w2 = r(3 * C, C), r(C, C), r(F, C), r(C, F)
        b3, bc, b1 = torch.zeros(3 * C, device=dev), torch.zeros(C, device=dev), torch.zeros(F, device=dev)
        dw = torch.zeros(F, C, device=dev)
        g = torch.ones(C, device=dev)
        mu, rs = torch.empty(M, device=dev), torch.empty(M, device=dev)
        E = 2  # bytes per bf16 element

        def add(name, us, flop, byts):
            res.append({"level": lvl, "kernel": name, "M": M, "us": round(us, 1),
                        "TF/s": round(flop / us / 1e6, 1), "GB/s": round(byts / us / 1e3, 1)})
            print(json.dumps(res[-1]), flush=True)

        add("fwd qkv", tm(lambda: ops.linear_fwd(x, w3, b3, out_3c, M, 3 * C, C)), 2.0 * M * 3 * C * C,
            E * M * (C + 3 * C))
        add("fwd proj+res", tm(lambda: ops.linear_fwd(x, wc, bc, out_c, M, C, C, mode=2, res=res_in)),
            2.0 * M * C * C, E * M * 3 * C)
        add("fwd fc1+gelu", tm(lambda: ops.linear_fwd(x, w1, b1, act, M, F, C, mode=1, aux=pre)),
            2.0 * M * F * C, E * M * (C + 2 * F))
        add("fwd fc2+res", tm(lambda: ops.linear_fwd(hid, w2, bc, out_c, M, C, F, mode=2, res=res_in)),
            2.0 * M * F * C, E * M * (F + 2 * C))
        add("dgrad fc2 (gelu')", tm(lambda: ops.linear_dgrad(x, w2, act, M, F, C, mode=1, aux=hid)),
            2.0 * M * F * C, E * M * (C + 2 * F))
        add("dgrad fc1", tm(lambda: ops.linear_dgrad(hid, w1, out_c, M, C, F)), 2.0 * M * F * C, E * M * (F + C))
        add("dgrad qkv", tm(lambda: ops.linear_dgrad(out_3c, w3, out_c, M, C, 3 * C)), 2.0 * M * 3 * C * C,
            E * M * 4 * C)
        add("wgrad fc1", tm(lambda: ops.linear_wgrad(hid, x, dw, M, F, C)), 2.0 * M * F * C, E * M * (F + C))
        add("wgrad fc2", tm(lambda: ops.linear_wgrad(x, hid, dw, M, C, F)), 2.0 * M * F * C, E * M * (F + C))
        add("colsum F", tm(lambda: ops.colsum(hid, b1, M, F)), M * F, E * M * F)
        add("layernorm_fwd", tm(lambda: ops.layernorm_fwd(x, g, bc, 1e-6, out_c, mu, rs, M, C)), 0,
            E * M * 2 * C)
        del x, res_in, hid, out_c, out_3c, pre, act
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
