"""Summarise `-Rpass-analysis=kernel-resource-usage` remarks of one hipcc compile:
one line per kernel (demangled, filtered by a substring) with VGPRs, AGPRs and
scratch bytes per lane.

    hipcc ... -c conv_ops.hip -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python tools/kernel_resources.py remarks.txt gemm_pp_kernel
"""
import re
import subprocess
import sys


def main(path, filt=""):
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
    for name, (_, info) in zip(names, rows):
        if filt not in name:
            continue
        short = re.sub(r"vlp::|__hip_bfloat16|\(|\)|void ", "", name.replace("GemmShape, ", ""))
        print(f"V{info.get('VGPRs', '?'):>4} A{info.get('AGPRs', '?'):>4} "
              f"S{info.get('ScratchSize [bytes/lane]', '?'):>4}  {short[:170]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
