"""Instruction mix of a kernel's hottest basic blocks (the ones holding MFMAs)
from a hipcc --cuda-device-only -S listing.
  python tools/asm_loop.py listing.s KERNEL_SUBSTRING [KERNEL_SUBSTRING2 ...]"""
import os
import re
import sys
from collections import Counter


def kernel_body(lines, sub):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and l.rstrip().endswith(":") is False and ":" in l:
            pass
        if start is None and re.match(r"^_Z\S*:", l) and all(s in l for s in sub):
            start = i
        elif start is not None and (l.startswith(".Lfunc_end") or re.match(r"^\s*\.end_amdhsa_kernel", l)):
            return lines[start:i]
    return lines[start:] if start is not None else []


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    for p in ("v_", "s_waitcnt", "s_barrier", "s_", "ds_", "global_load_lds", "global_", "buffer_"):
        if op.startswith(p):
            return p.rstrip("_")
    return "other"


def main():
    lines = open(sys.argv[1]).read().splitlines()
    body = kernel_body(lines, sys.argv[2:])
    blocks, cur, name = [], [], "entry"
    for l in body:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        cur.append(t.split()[0])
    blocks.append((name, cur))
    tot = Counter()
    show_all = os.environ.get("ASM_ALL") == "1"
    for name, ins in blocks:
        c = Counter(classify(o) for o in ins)
        if show_all and not c["mfma"]:
            print("  ", name, len(ins), dict(c.most_common()))
        if c["mfma"]:
            print(name, len(ins), dict(c.most_common()))
            tot += c
    vgpr = [l for l in body if ".vgpr_count" in l or "NumVgprs" in l or "vgpr_count" in l]
    print("total over MFMA blocks:", dict(tot.most_common()))
    for l in body:
        if re.search(r"; (NumVgprs|NumAgprs|Occupancy|ScratchSize|LDSByteSize)", l):
            print(l.strip())


if __name__ == "__main__":
    main()
