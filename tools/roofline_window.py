"""Average duration of the roofline kernel family's dispatches inside bench.py's
isolated roofline pass, from a rocprofv3 kernel trace of the bench command.

bench.py brackets that pass with two empty marker dispatches
(vlp_trace_marker -> trace_marker_begin_kernel / trace_marker_end_kernel); the
dispatches of the family (kernel names matching --include and not --exclude)
that start between the markers are the launches the bench line's
`roofline.avg_launch_us` averages with HIP events.

  python tools/roofline_window.py KERNEL_TRACE.csv [--include RX] [--exclude RX] [--out F.json]

Default family: conv_wgrad[raw]/wide = the ConvWgradB weight-gradient GEMMs
except the Co = 64 layer-1 tile (gemm_big_kernel<64,192>).
"""
import argparse
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_csv")
    ap.add_argument("--include", default=r"ConvWgradB")
    ap.add_argument("--exclude", default=r"gemm_big_kernelILi64ELi192E")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace_csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    begins = [s for s, _, n in rows if "trace_marker_begin_kernel" in n]
    ends = [s for s, _, n in rows if "trace_marker_end_kernel" in n]
    assert begins and ends, "no marker dispatches in the trace"
    t0, t1 = begins[-1], min(e for e in ends if e > begins[-1])
    inc, exc = re.compile(a.include), re.compile(a.exclude) if a.exclude else None
    per = {}
    durs = []
    for s, e, n in rows:
        if t0 < s < t1 and inc.search(n) and not (exc and exc.search(n)):
            durs.append(e - s)
            per.setdefault(n, []).append(e - s)
    assert durs, "no family dispatch inside the window"
    res = {"launches": len(durs), "avg_us": sum(durs) / len(durs) / 1e3,
           "window_ms": (t1 - t0) / 1e6,
           "per_kernel": {k: {"calls": len(v), "avg_us": sum(v) / len(v) / 1e3} for k, v in per.items()},
           "method": "rocprofv3 --kernel-trace; dispatches between bench.py's trace markers"}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
