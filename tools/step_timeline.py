"""Timeline of one bench step under the default (side-stream) schedule, from a
rocprofv3 kernel trace: which HIP queue carries which kernels, where the GPU is
idle, and which queue finishes the step.

  run      (GPU)  build the bench model, warm up, then run --steps steps between
                  two vlp_trace_marker dispatches:
                    rocprofv3 --kernel-trace -d DIR -o t -- python tools/step_timeline.py run
  analyze  (CPU)  python tools/step_timeline.py analyze DIR/.../t_kernel_trace.csv [--out F.json]
"""
import argparse
import csv
import functools
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]


def run(a):
    import torch
    import bench
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd._lib import lib
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                                 False, False, 512, 312, 128, compute_dtype="bf16", device=dev)
    model.train()
    opt = model.configure_optimizers()["optimizer"]
    batch = bench.make_batch(a.batch, 512, 40, dev, seed=0, form="u8")

    def step():
        opt.zero_grad()
        model.training_step(batch).backward()
        opt.step()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev).cuda_stream
    lib().vlp_trace_marker(0, s)
    for _ in range(a.steps):
        step()
    lib().vlp_trace_marker(1, s)
    torch.cuda.synchronize()
    print("ok")


def short(name):
    n = re.sub(r"^void ", "", name)
    n = n.split("(")[0]
    m = re.match(r"([\w:]+)<(.*)>$", n)
    if m:
        base, targs = m.group(1), m.group(2)
        return f"{base.split('::')[-1]}<{targs[:60]}>"
    return n.split("::")[-1][:80]


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def analyze(a):
    rows = []
    with open(a.trace_csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]))
    rows.sort()
    begins = [s for s, _, _, n in rows if "trace_marker_begin_kernel" in n]
    ends = [e for _, e, _, n in rows if "trace_marker_end_kernel" in n]
    t0 = begins[a.window]
    t1 = min(e for e in ends if e > t0)
    ks = [(s, e, q, n) for s, e, q, n in rows if t0 < s < t1 and "trace_marker" not in n]
    span = (t1 - t0) / 1e6
    queues = sorted({q for _, _, q, _ in ks})
    res = {"window_ms": round(span, 3), "kernels": len(ks), "queues": {}}
    for q in queues:
        iv = [(s, e) for s, e, qq, _ in ks if qq == q]
        u = union(iv)
        busy = sum(e - s for s, e in u) / 1e6
        fam = {}
        for s, e, qq, n in ks:
            if qq == q:
                k = short(n)
                fam[k] = fam.get(k, 0) + (e - s) / 1e6
        top = sorted(fam.items(), key=lambda kv: -kv[1])[:8]
        res["queues"][q] = {"launches": len(iv), "busy_ms": round(busy, 3),
                            "first_ms": round((u[0][0] - t0) / 1e6, 3), "last_end_ms": round((u[-1][1] - t0) / 1e6, 3),
                            "top": [(k, round(v, 3)) for k, v in top]}
    u_all = union([(s, e) for s, e, _, _ in ks])
    busy_all = sum(e - s for s, e in u_all) / 1e6
    gaps = []
    for (s0, e0), (s1, e1) in zip(u_all, u_all[1:]):
        gaps.append(((s1 - e0) / 1e6, (e0 - t0) / 1e6))
    gaps.sort(reverse=True)
    # time with two or more queues busy
    ev = []
    for q in queues:
        for s, e in union([(s, e) for s, e, qq, _ in ks if qq == q]):
            ev += [(s, 1), (e, -1)]
    ev.sort()
    depth, last, multi = 0, None, 0
    for t, d in ev:
        if depth >= 2 and last is not None:
            multi += t - last
        depth += d
        last = t
    res["gpu_busy_ms"] = round(busy_all, 3)
    res["gpu_idle_ms"] = round(span - busy_all, 3)
    res["overlap_ms"] = round(multi / 1e6, 3)
    res["largest_idle_gaps"] = [(round(g, 4), round(at, 3)) for g, at in gaps[:10]]
    # main-queue gaps (the queue of the first kernel): where it waits on another queue
    mq = ks[0][2]
    mu = union([(s, e) for s, e, q, _ in ks if q == mq])
    mg = sorted((((s1 - e0) / 1e6, (e0 - t0) / 1e6) for (s0, e0), (s1, e1) in zip(mu, mu[1:])), reverse=True)
    res["main_queue"] = mq
    res["main_queue_waits"] = [(round(g, 4), round(at, 3)) for g, at in mg[:12]]
    # the tail: last kernels per queue
    res["tail"] = {q: [(short(n), round((s - t0) / 1e6, 3), round((e - s) / 1e6, 3))
                       for s, e, qq, n in ks if qq == q][-a.tail:] for q in queues}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--batch", type=int, default=256)
    r.add_argument("--warmup", type=int, default=4)
    r.add_argument("--steps", type=int, default=1)
    z = sub.add_parser("analyze")
    z.add_argument("trace_csv")
    z.add_argument("--window", type=int, default=0)
    z.add_argument("--tail", type=int, default=8)
    z.add_argument("--out", default="")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else analyze(a)


if __name__ == "__main__":
    main()
