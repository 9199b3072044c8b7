#!/usr/bin/env python3
"""Log-record verify (nova_log_verify_records) on one log image under several
pre-sort variants, in one process, so that one rocprofv3 --pmc pass covers
them all (the sorted windows' over-fetch):

  python tools/log_sort_ab.py --variants 2:0:0,2:128:0,2:256:1,0 [--payload-max 4096]
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o pmc -- python3 tools/log_sort_ab.py ...
  python tools/log_sort_ab.py --split DIR --variants ... [--steps K --warmup W]

A variant is "sort[:window[:key]]" (nova_diag_set_rounds_sort / _log_window /
_log_key; 2:0:0 is the product).  Each variant runs `warmup` then `steps`
launches in order, so --split can cut the counter CSV's dispatches of the
rounds kernel (and the sort / unperm pre- and post-passes) back into variants
and report HBM read bytes per launch (FETCH_SIZE x 2, the gfx950 correction)
against the algorithmic bytes.  Every variant's statuses are checked (all OK).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
HBM_PEAK_GBS = 8000.0


def parse_variants(s: str):
    out = []
    for v in [x for x in s.split(",") if x]:
        so, win, key = (v.split(":") + ["0", "0"])[:3]
        out.append((v, int(so), int(win or 0), int(key or 0)))
    return out


def split(args) -> int:
    """Per-variant HBM read bytes per launch from a --pmc FETCH_SIZE run."""
    rows = []
    for path in glob.glob(os.path.join(args.split, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != "FETCH_SIZE":
                    continue
                rows.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0), r["Kernel_Name"],
                             float(r["Counter_Value"])))
    rows.sort()
    per = collections.defaultdict(float)
    count = collections.Counter()
    # log verify's rounds dispatches (MODE 4; the image's one log write is MODE 3)
    import re
    seq = [r for r in rows if re.search(r"crc32c_rounds_kernel<\d+, 4", r[1])]
    var = parse_variants(args.variants)
    k = args.steps + args.warmup
    info = json.load(open(args.info)) if args.info and os.path.exists(args.info) else {}
    alg = info.get("alg_bytes")
    # rounds-kernel dispatches in launch order: the first (1 + k) are the check
    # launch and variant 0, then k per variant
    starts = [1 + i * k for i in range(len(var))]
    for i, (name, *_r) in enumerate(var):
        lo, hi = starts[i] + args.warmup, starts[i] + k
        sel = seq[lo:hi]
        if not sel:
            continue
        fb = sum(x[2] for x in sel) / len(sel) * 1024 * 2  # KiB, x2 (MI355X_MICROARCH.md)
        # the pre-/post-passes between the variant's first and last rounds dispatch
        d0, d1 = sel[0][0], sel[-1][0]
        aux = [r for r in rows if d0 - 3 <= r[0] <= d1 + 3 and ("log_sort_kernel" in r[1] or "log_unperm_kernel" in r[1])]
        aux_b = sum(x[2] for x in aux) / len(sel) * 1024 * 2 if aux else 0.0
        out = {"variant": name, "launches": len(sel), "rounds_read_GB": round(fb / 1e9, 4),
               "aux_read_GB": round(aux_b / 1e9, 4)}
        if alg:
            out["rounds_read_over_alg"] = round(fb / alg, 4)
            out["all_read_over_alg"] = round((fb + aux_b) / alg, 4)
        print(json.dumps(out), flush=True)
    return 0


def aligned_layout(total_target: int, seed: int, pmax: int, align: int):
    """FULL records of U[1,pmax] B payloads, each at a multiple of `align`
    bytes, none crossing a 32 KiB log block (the gap bytes are zeros)."""
    from novalsm_amd.synth import splitmix64_words
    blk = 32768
    mean = 7 + (pmax + 1) // 2
    slot_mean = (mean + align - 1) // align * align
    n = total_target // slot_mean
    r = splitmix64_words(seed, 0, n)
    plens = ((r % np.uint64(pmax)) + np.uint64(1)).astype(np.int64)
    slots = (7 + plens + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    pos = 0
    sl = slots.tolist()
    rec = (7 + plens).tolist()
    for i in range(n):
        if pos // blk != (pos + rec[i] - 1) // blk:  # would cross a block: next block
            pos = (pos // blk + 1) * blk
        offs[i] = pos
        pos += sl[i]
    return (offs.astype(np.uint64), plens.astype(np.uint64), np.ones(n, np.uint8), int(pos))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="2:0:0")
    ap.add_argument("--payload-max", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1, help="alternations of the variant list (timing only)")
    ap.add_argument("--split", default="", help="rocprofv3 output dir to split per variant")
    ap.add_argument("--info", default="gpurun_out/log_sort_ab_info.json")
    ap.add_argument("--align", type=int, default=0,
                    help="place every record at a multiple of this many bytes (no line shared "
                         "by two records: an A/B of the boundary lines' cost), records never "
                         "crossing a 32 KiB block")
    args = ap.parse_args()
    if args.split:
        return split(args)
    import torch
    from novalsm_amd import crc32c as C
    from bench_ops import log_layout, timed

    assert C.load().nova_device_init() == 0
    if args.align:
        offs_np, lens_np, types_np, total = aligned_layout(4 << 30, args.seed, args.payload_max, args.align)
    else:
        offs_np, lens_np, types_np, total = log_layout(4 << 30, args.seed, args.payload_max)
    n = len(offs_np)
    buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 41)
    o = torch.from_numpy(offs_np.view(np.int64)).cuda()
    ln = torch.from_numpy(lens_np.astype(np.int64)).cuda()
    buf[o + 4] = (ln & 0xFF).to(torch.uint8)
    buf[o + 5] = (ln >> 8).to(torch.uint8)
    buf[o + 6] = torch.from_numpy(types_np).cuda()
    alg = int(lens_np.sum()) + 7 * n
    stream = torch.cuda.current_stream()
    C.log_write_crcs(buf, o, stream=stream)
    okb = torch.empty(n, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")

    def lv():
        C.log_verify_records(buf, o, stream=stream, ok=okb, bad=bad)

    lv()  # the check launch (one rounds dispatch before the variants)
    torch.cuda.synchronize()
    assert int(bad.item()) == 0 and bool((okb.cpu().numpy() == C.LOG_OK).all())
    os.makedirs(os.path.dirname(args.info) or ".", exist_ok=True)
    json.dump({"alg_bytes": alg, "records": n, "payload_max": args.payload_max}, open(args.info, "w"))
    print(json.dumps({"image": f"{n} records, payload U[1,{args.payload_max}] B, {total / 2**30:.2f} GiB",
                      "alg_bytes": alg}), flush=True)
    for rnd in range(args.rounds):
        for name, so, win, key in parse_variants(args.variants):
            with C.diagnostics() as D:
                D.nova_diag_set_rounds_sort(so)
                D.nova_diag_set_log_window(win)
                D.nova_diag_set_log_key(key)
                okb.fill_(0xEE)
                sec = timed(torch, lv, args.steps, args.warmup, stream)
            good = bool((okb.cpu().numpy() == C.LOG_OK).all()) and int(bad.item()) == 0
            gbs = alg / sec / 1e9
            print(json.dumps({"round": rnd, "variant": name, "ms": round(sec * 1e3, 4), "GBps": round(gbs, 1),
                              "frac": round(gbs / HBM_PEAK_GBS, 4), "statuses_ok": good}), flush=True)
            if not good:
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
