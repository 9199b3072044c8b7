#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a gfx950 assembly dump
(hipcc --save-temps ... -> *-gfx950.s), for reading where a kernel's issue
slots go without a GPU:

  python tools/isa_stats.py <file.s> <kernel-name-substring> [--blocks]

Prints the kernel's VGPR/SGPR/scratch use, instruction classes (VALU, SALU,
LDS, VMEM load/store, DPP, waitcnt, branches) in total and, with --blocks, per
basic block with the branch targets, so the loop body of a kernel can be
picked out and its per-iteration cost counted.
"""
from __future__ import annotations

import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic")):
        return "vmem_st"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def body(lines: list[str], name: str) -> tuple[str, list[str]]:
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^(\S+):\s*(;.*)?$", l)
        if m and name in m.group(1) and not m.group(1).startswith("."):
            start, sym = i, m.group(1)
            break
    if start is None:
        raise SystemExit(f"no kernel matching {name!r}")
    out = []
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or re.match(r"^\s*\.Lfunc_end", l):
            break
        out.append(l)
    return sym, out


def main() -> int:
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    sym, b = body(lines, name)
    print(sym)
    meta = "\n".join(lines)
    for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size"):
        m = re.search(rf"\.set {re.escape(sym)}\.num_vgpr, (\d+)", meta) if key == "vgpr_count" else None
    tot = Counter()
    blocks = []
    cur = ["entry", Counter(), []]
    for l in b:
        s = l.strip()
        if not s or s.startswith((";", ".")):
            m = re.match(r"^(\.LBB\S+):", s)
            if m:
                blocks.append(cur)
                cur = [m.group(1), Counter(), []]
            continue
        op = s.split()[0]
        c = classify(op)
        if "_dpp" in s or " dpp" in s or "row_" in s or "quad_perm" in s:
            cur[1]["dpp"] += 1
        cur[1][c] += 1
        tot[c] += 1
        if c == "branch":
            cur[2].append(s)
    blocks.append(cur)
    print("total", dict(tot))
    if "--blocks" in sys.argv:
        for lab, cnt, br in blocks:
            n = sum(v for k, v in cnt.items() if k != "dpp")
            print(f"{lab:>14} n={n:4d} " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())) +
                  ("  -> " + "; ".join(br) if br else ""))
    return 0


if __name__ == "__main__":
    sys.exit(main())
