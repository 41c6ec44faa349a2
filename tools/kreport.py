"""Pretty-print a bench.py --kernel-report JSON (per kernel family: time, launches, TF/s)."""
import json, sys
d = json.load(open(sys.argv[1]))
tot = sum(v["ms"] for v in d.values())
print(f"total timed kernel ms per step: {tot:.2f}")
for k, v in list(d.items())[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    tf = v["gflop"] / v["ms"] if v["ms"] else 0.0
    print(f"{k:40s} {v['ms']:9.3f} ms {100*v['ms']/tot:5.1f}%  n={v['launches']:4d}  TF/s={tf:8.1f}")
