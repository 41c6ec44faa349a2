"""TinyBERT tower alone at the bench shape (bs = 256, T = 40, bf16, CLS-only last
layer as the training step runs it): forward + backward per step with HIP events,
and the per-family kernel time (ktimer), to size what the text stream costs the
step when it shares the CUs with the image tower.
  python tools/text_tower_bench.py [--batch 256] [--seq 40] [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=40)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from vlp_amd import ktimer
    from vlp_amd.tinybert import TinyBertConfig, TinyBertTower
    dev = torch.device("cuda", 0)
    t = TinyBertTower(TinyBertConfig(0.1, 0.1), compute_dtype="bf16", device=dev)
    t.train()
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(1, 30000, (a.batch, a.seq), generator=g).to(dev)
    mask = torch.ones(a.batch, a.seq, dtype=torch.long, device=dev)
    mask[:, a.seq * 3 // 4:] = 0
    tt = torch.zeros_like(ids)
    dcls = torch.randn(a.batch, t.cfg.hidden, device=dev) * 1e-3

    def step():
        h, sv = t.run_forward(ids, mask, tt, True, cls_only=True)
        t.run_backward(sv, dcls)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    ktimer.enable(None)
    step()
    torch.cuda.synchronize()
    fam = {k: round(v[0], 4) for k, v in sorted(ktimer.totals().items(), key=lambda kv: -kv[1][0])}
    ktimer.disable()
    print(json.dumps({"shape": f"bs={a.batch} T={a.seq}", "fwd_bwd_ms": round(ms, 3),
                      "kernel_ms_sum": round(sum(fam.values()), 3), "families_ms": fam}))


if __name__ == "__main__":
    main()
