#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a hipcc -S listing.

usage: isa_loops.py file.s kernel_substring
Finds the kernel's body, the basic blocks that end in a backward branch
(loops), and prints per loop the count of MFMA / VALU / LDS / VMEM / SALU /
waitcnt instructions -- the VALU-per-MFMA budget of cdna_hip_programming.md.
"""
import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_write", "ds_bpermute", "ds_swizzle")):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", ln))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = i
    for i, ln in enumerate(body):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\d+_\d+)", ln) or re.match(r"\s+s_branch\s+(\.LBB\d+_\d+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            lo = labels[m.group(1)]
            c = Counter()
            for x in body[lo:i + 1]:
                x = x.strip()
                if not x or x.startswith((";", ".")) or x.endswith(":"):
                    continue
                c[classify(x.split()[0])] += 1
            mf = max(1, c["mfma"])
            if "--hist" in sys.argv:
                lines_ = (y.strip() for y in body[lo:i + 1])
                h = Counter(x.split()[0] for x in lines_
                            if x and not x.startswith((";", ".")) and not x.endswith(":"))
                print("   ", ", ".join(f"{k} {v}" for k, v in h.most_common(40)))
            mix = " ".join(f"{k}={v}" for k, v in sorted(c.items()))
            print(f"loop {m.group(1)} lines {start + lo + 1}-{start + i + 1}: {mix}  valu/mfma={c['valu'] / mf:.2f}")


if __name__ == "__main__":
    main()
