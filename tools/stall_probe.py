#!/usr/bin/env python3
"""Host-visible GPU stalls without the engine (tail latency).

Times a loop of tiny kernels (nova_fill_splitmix64 of 4 KiB, each waited on)
for --seconds and prints the slowest iterations with their start times, the
count over 1 ms, and the gaps between those.  A stall that hits every caller
at once at a fixed period, with no engine running, is the box's, not the
library's.

  python tools/stall_probe.py [--seconds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    C.load()
    assert C.load().nova_device_init() == 0
    x = torch.empty(4096, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    L = C.load()
    for _ in range(100):
        L.nova_fill_splitmix64(x.data_ptr(), 4096, 1, 0, s.cuda_stream)
        s.synchronize()
    t_start = time.perf_counter()
    rows = []
    while True:
        t0 = time.perf_counter()
        if t0 - t_start > args.seconds:
            break
        L.nova_fill_splitmix64(x.data_ptr(), 4096, 1, 0, s.cuda_stream)
        s.synchronize()
        rows.append((time.perf_counter() - t0, t0 - t_start))
    lat = sorted(r[0] for r in rows)
    slow = sorted((r for r in rows if r[0] > 1e-3), key=lambda r: r[1])
    starts = [round(r[1], 4) for r in slow]
    print(json.dumps({"iterations": len(rows), "p50_us": round(lat[len(lat) // 2] * 1e6, 1),
                      "p99_us": round(lat[int(len(lat) * 0.99)] * 1e6, 1), "max_us": round(lat[-1] * 1e6, 1),
                      "over_1ms": len(slow),
                      "over_1ms_at_s_ms": [[a, round(b[0] * 1e3, 2)] for a, b in zip(starts, slow)][:40],
                      "gaps_s": [round(b - a, 4) for a, b in zip(starts, starts[1:])][:40]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
