"""HBM traffic per launch from rocprofv3 PMC CSVs (separate FETCH_SIZE and
WRITE_SIZE passes, as MI355X_MICROARCH.md §HBM prescribes).

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  gfx950
correction: FETCH_SIZE tallies 128-B requests at 64 B, so wide coalesced reads
are reported at exactly half their bytes -> x2.  WRITE_SIZE is exact for
16-B-per-lane stores and float atomics.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv REGEX --family NAME [--out f.json]
  (--out merges the family's entry into the file's "families" map)
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("regex")
    ap.add_argument("--out", default="")
    ap.add_argument("--family", default="")
    args = ap.parse_args()
    fe = per_kernel(args.fetch_csv, "FETCH_SIZE")
    wr = per_kernel(args.write_csv, "WRITE_SIZE")
    rx = re.compile(args.regex)
    names = sorted(k for k in fe if rx.search(k))
    assert names, "no kernel matches"
    f_all = [v for k in names for v in fe[k]]
    w_all = [v for k in names for v in wr.get(k, [])]
    fetch = 2.0 * 1024.0 * sum(f_all) / len(f_all)
    write = 1024.0 * sum(w_all) / max(len(w_all), 1)
    res = {"family": args.family, "kernels": names, "launches": len(f_all),
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write,
           "method": "rocprofv3 --pmc FETCH_SIZE (x2 gfx950 correction, KiB->B) and a separate "
                     "--pmc WRITE_SIZE pass (KiB->B), averaged over the matching dispatches"}
    # calibration: the AdamW kernel streams 16 B/element in and 12 B/element out
    cal = [k for k in fe if "adamw_kernel" in k]
    if cal:
        res["calibration_adamw"] = {"fetch_bytes_mean": 2048.0 * sum(fe[cal[0]]) / len(fe[cal[0]]),
                                    "write_bytes_mean": 1024.0 * sum(wr.get(cal[0], [0])) / max(len(wr.get(cal[0], [])), 1)}
    print(json.dumps(res, indent=1))
    if args.out:
        # one file, one entry per kernel family (bench.py looks its roofline family up)
        try:
            with open(args.out) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            doc = {}
        if "families" not in doc:
            doc = {"families": {}}
        doc["families"][args.family or args.regex] = res
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
