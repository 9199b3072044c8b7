#!/usr/bin/env python3
"""Burst (one-SSTable) kernel: kernel time of nova_sstable_verify_blocks on n
SSTable-like blocks (4096+U[0,255] B, 5-B trailers) per table set -- 64 lanes
per block (compact tables), 16 lanes per block (replicated tables), or the
burst kernel off (the rounds kernel) -- through the diagnostics library's
nova_diag_set_burst_lanes.  HIP events on the launch stream, median of R
launches per size; one JSON line per (n, lanes).  Picks the dispatcher's
kBurstWideMax threshold."""
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
    ap.add_argument("--sizes", default="1,16,64,128,256,512,1024,2048,4096,6144")
    ap.add_argument("--lanes", default="64,16,-1")
    ap.add_argument("--waves", default="0", help="comma list of waves per workgroup (0 = default)")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_words
    L = C.enable_diagnostics()
    assert L.nova_device_init() == 0
    stream = torch.cuda.current_stream()
    for n in [int(x) for x in args.sizes.split(",")]:
        r = splitmix64_words(5, 0, n)
        lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
        total = int(offs[-1]) + int(lens[-1]) + 5
        dev = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(dev, 31)
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        C.write_trailers(dev, do, dl, 0, False, stream=stream)
        okb = torch.empty(n, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        for lanes, waves in [(int(a), int(w)) for a in args.lanes.split(",")
                             for w in args.waves.split(",")]:
            L.nova_diag_set_burst_lanes(lanes)
            L.nova_diag_set_stream_waves(waves)
            for _ in range(20):
                C.verify_blocks(dev, do, dl, stream=stream, ok=okb, bad=bad)
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                C.verify_blocks(dev, do, dl, stream=stream, ok=okb, bad=bad)
                b.record(stream)
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ok = int(bad.item()) == 0 and bool(okb.cpu().numpy().all())
            print(json.dumps({"n_blocks": n, "lanes": lanes, "waves": waves, "kernel_us": round(statistics.median(ts), 2),
                              "min_us": round(min(ts), 2), "verified": ok}), flush=True)
        L.nova_diag_set_burst_lanes(0)
        L.nova_diag_set_stream_waves(0)
        del dev
    return 0


if __name__ == "__main__":
    sys.exit(main())
