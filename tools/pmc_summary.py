"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel (short name),
mean value of each counter over its dispatches.
  python tools/pmc_summary.py file1.csv [file2.csv ...]
(PMC_FILTER: regex of the kernel names to print; default gemm / conv kernels)"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(k):
    m = re.search(r"gemm_(\w+?)_kernelILi(\d+)ELi(\d+)E.*?NS_\d+(\w+?)I", k)
    if m:
        return f"gemm_{m.group(1)}{m.group(2)}x{m.group(3)}:{m.group(4)}"
    return k[:60]


vals = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
flt = re.compile(os.environ.get("PMC_FILTER", "gemm|conv|Conv"))
for k, d in vals.items():
    if not flt.search(k):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
