"""Collect one A/B call's results (tools/gpu_ab.sh / gpu_envab.sh logs under
gpurun_out/) into a compact JSON record for profiles/:

    python tools/ab_summary.py TAG profiles/TAG_name.json [--note "..."] [--families f1,f2]

bench lines: gpurun_out/TAG_bench_<variant>_<rep>.log or TAG_<arm>_<rep>.log (value, ms_per_step);
conv_bench: gpurun_out/TAG_cb_<variant>.log (op/layer -> us, TF/s);
kernel reports: gpurun_out/TAG_kreport_<variant>_<rep>.json (ms per step of the named families).
"""
import argparse
import glob
import json
import os
import re


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("out")
    ap.add_argument("--note", default="")
    ap.add_argument("--families", default="")
    ap.add_argument("--dir", default="gpurun_out")
    a = ap.parse_args()
    rec = {"tag": a.tag, "note": a.note, "bench": {}, "conv_bench": {}, "kernel_report": {}}
    for p in sorted(glob.glob(os.path.join(a.dir, f"{a.tag}_*.log"))):
        base = os.path.basename(p)[len(a.tag) + 1:-4]
        if base.startswith("cb_"):
            rows = {}
            for line in open(p):
                m = re.match(r"(\S+)\s+(l\d|\S+)\s*:\s+([\d.]+) us\s+([\d.]+) TF/s", line.strip())
                if m:
                    rows[f"{m.group(1)}_{m.group(2)}"] = {"us": float(m.group(3)), "tflops": float(m.group(4))}
            rec["conv_bench"][base[3:]] = rows
            continue
        m = re.match(r"(?:bench_)?(.+)_(\d+)$", base)
        if not m:
            continue
        j = last_json(p)
        if j and "value" in j:
            rec["bench"].setdefault(m.group(1), []).append(
                {"rep": int(m.group(2)), "value": j["value"], "ms_per_step": j.get("ms_per_step")})
    fams = [f for f in a.families.split(",") if f]
    for p in sorted(glob.glob(os.path.join(a.dir, f"{a.tag}_kreport_*.json"))):
        base = os.path.basename(p)[len(a.tag) + len("_kreport_"):-5]
        d = json.load(open(p))
        rec["kernel_report"][base] = {k: round(v["ms"], 4) for k, v in d.items() if not fams or k in fams}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "kernel_report"}, indent=1)[:3000])


if __name__ == "__main__":
    main()
