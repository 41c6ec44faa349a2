"""Summarise `-Rpass-analysis=kernel-resource-usage` remarks of one hipcc compile:
one line per kernel (demangled, filtered by a substring) with VGPRs, AGPRs and
scratch bytes per lane.

    hipcc ... -c conv_ops.hip -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python tools/kernel_resources.py remarks.txt gemm_pp_kernel
    python tools/kernel_resources.py remarks.txt nest_attn --max-scratch 0   # build check: exit 1 on scratch
"""
import re
import subprocess
import sys


def main(path, filt="", max_scratch=None):
    cur, info, rows = None, {}, []
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            if cur:
                rows.append((cur, info))
            cur, info = m.group(1), {}
            continue
        for key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]"):
            m = re.search(re.escape(key) + r": (\d+)", line)
            if m and cur:
                info[key] = int(m.group(1))
    if cur:
        rows.append((cur, info))
    names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    over, seen = [], 0
    for name, (_, info) in zip(names, rows):
        if filt not in name:
            continue
        seen += 1
        if max_scratch is not None and info.get("ScratchSize [bytes/lane]", 0) > max_scratch:
            over.append(name)
        short = re.sub(r"vlp::|__hip_bfloat16|\(|\)|void ", "", name.replace("GemmShape, ", ""))
        print(f"V{info.get('VGPRs', '?'):>4} A{info.get('AGPRs', '?'):>4} "
              f"S{info.get('ScratchSize [bytes/lane]', '?'):>4}  {short[:170]}")


    if max_scratch is not None:
        if not seen:
            sys.exit(f"kernel_resources: no kernel matches {filt!r} in {path}")
        if over:
            sys.exit(f"kernel_resources: {len(over)} kernel(s) use scratch > {max_scratch} B/lane: {over}")


if __name__ == "__main__":
    args = sys.argv[1:]
    ms = None
    if "--max-scratch" in args:
        i = args.index("--max-scratch")
        ms = int(args[i + 1])
        del args[i:i + 2]
    main(args[0], args[1] if len(args) > 1 else "", ms)
