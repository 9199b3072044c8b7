#!/usr/bin/env python3
"""Per-call latency of log-record CRC write/verify (db/log_writer.cc:99-125,
db/log_reader.cc:251-262) on small log images, across rounds-kernel chunk
settings (tools/sweep_flat.py variants).  Device-resident, HIP events, medians.
Each variant's verify must pass on the records the default variant wrote."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,1048576,16777216,268435456,4294967296")
    ap.add_argument("--variants", default="auto,rounds:8:131:12:0,rounds:8:67:12:0,rounds:16:67:12:0")
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from tools.bench_ops import log_layout
    from tools.sweep_flat import set_variant
    assert C.load().nova_device_init() == 0
    s = torch.cuda.current_stream()
    for size in [int(x) for x in args.sizes.split(",")]:
        offs_np, lens_np, types_np, total = log_layout(size, 6)
        n = len(offs_np)
        buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 41)
        o = torch.from_numpy(offs_np.view(np.int64)).cuda()
        ln = torch.from_numpy(lens_np.astype(np.int64)).cuda()
        buf[o + 4] = (ln & 0xFF).to(torch.uint8)
        buf[o + 5] = (ln >> 8).to(torch.uint8)
        buf[o + 6] = torch.from_numpy(types_np).cuda()
        set_variant(C, "auto")
        C.log_write_crcs(buf, o, stream=s)
        row = {"records": n, "MiB": round(total / 2**20, 2)}
        for v in args.variants.split(","):
            set_variant(C, v)
            res = []
            for fn in (lambda: C.log_write_crcs(buf, o, stream=s),
                       lambda: C.log_verify_records(buf, o, stream=s)):
                ev = []
                for i in range(60):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    fn()
                    b.record(s)
                    b.synchronize()
                    if i >= 10:
                        ev.append(a.elapsed_time(b) * 1e3)
                res.append(round(statistics.median(ev), 1))
            ok, bad = C.log_verify_records(buf, o, stream=s)
            res.append(int(bad.item()) == 0 and bool(ok.cpu().numpy().all()))
            row[v] = res  # [write us, verify us, verified]
        set_variant(C, "auto")
        print(json.dumps(row), flush=True)
        del buf
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
