#!/usr/bin/env python3
"""Phase timeline of the one-SSTable burst kernel (diagnostics build, variant
kVarStamps): per wave, s_memrealtime (100 MHz) at entry, once the first
block's descriptors are used, once the tables and first data have landed,
after the first block's fold, after its result is written.  For each batch
size: the event-timed kernel, the stamped span (first entry -> last write),
the entry skew over waves and the median of each phase.

    python tools/burst_stamps.py [--sizes 1,64,1024,4096] [--lanes 64]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,1024,4096")
    ap.add_argument("--lanes", type=int, default=0, help="burst lanes (0 = automatic)")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_words
    L = C.enable_diagnostics()
    L.nova_diag_set_stamps.argtypes = [ctypes.c_void_p]
    assert L.nova_device_init() == 0
    for n in [int(x) for x in args.sizes.split(",")]:
        r = splitmix64_words(5, 0, n)
        lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
        total = int(offs[-1]) + int(lens[-1]) + 5
        buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 9)
        o = torch.from_numpy(offs.view(np.int64)).cuda()
        ln = torch.from_numpy(lens.view(np.int32)).cuda()
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        with C.diagnostics() as D:
            if args.lanes:
                D.nova_diag_set_burst_lanes(args.lanes)
            C.write_trailers(buf, o, ln, 0, False)
            # event-timed launches without stamps
            ev = []
            for _ in range(args.iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                C.verify_blocks(buf, o, ln, ok=ok, bad=bad)
                b.record()
                ev.append((a, b))
            torch.cuda.synchronize()
            ev_us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ev[5:])
            # stamped launches
            st = torch.zeros(8 * max(4096, n), dtype=torch.int64, device="cuda")
            D.nova_diag_set_stamps(st.data_ptr())
            D.nova_diag_set_variant(4)  # kVarStamps
            spans, ph = [], {k: [] for k in ("desc", "land", "fold", "write")}
            skews = []
            for _ in range(10):
                st.zero_()
                C.verify_blocks(buf, o, ln, ok=ok, bad=bad)
                torch.cuda.synchronize()
                s = st.cpu().numpy().reshape(-1, 8)
                s = s[s[:, 4] > 0]
                t0 = s[:, 0].min()
                spans.append((s[:, 4].max() - t0) * TICK_US)
                skews.append((np.percentile(s[:, 0], 90) - t0) * TICK_US)
                for k, (i, j) in zip(ph, ((0, 1), (1, 2), (2, 3), (3, 4))):
                    ph[k].append(float(np.median(s[:, j] - s[:, i])) * TICK_US)
            D.nova_diag_set_variant(0)
            D.nova_diag_set_stamps(None)
        assert int(bad.item()) == 0
        print(json.dumps({"n_blocks": n, "waves": int(len(s)), "event_us": round(ev_us, 2),
                          "stamped_span_us": round(statistics.median(spans), 2),
                          "entry_skew_p90_us": round(statistics.median(skews), 2),
                          "phase_median_us": {k: round(statistics.median(v), 2) for k, v in ph.items()}}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
