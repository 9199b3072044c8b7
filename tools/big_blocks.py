#!/usr/bin/env python3
"""Batches of FEW, LARGE blocks: the kernel time of nova_crc32c_batch_strided
and of nova_crc32c_batch (with and without NOVA_CRC32C_HINT_LARGE_BLOCKS) when
the batch holds fewer blocks than the machine has lane groups -- one 256 MiB
block, 16 x 64 MiB, 256 x 4 MiB, 4096 x 256 KiB, 65536 x 64 KiB (every case
1 GiB but the first).  One JSON line per case and path: the dispatched kernel
(nova_crc32c_describe), median kernel time (HIP events on the launch stream)
and GB/s against the 8 TB/s HBM peak.  The first and last block of every
launch are checked against the CPU oracle (test tooling: the oracle is the
checker only).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
CASES = [(1, 256 << 20), (16, 64 << 20), (256, 4 << 20), (4096, 256 << 10), (65536, 64 << 10)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="")
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from tests.oracle_lib import load_oracle
    orc = load_oracle()
    stream = torch.cuda.current_stream()
    cases = CASES
    if args.cases:
        cases = [tuple(int(x) for x in c.split("x")) for c in args.cases.split(",")]
    for n, L in cases:
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 9)
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
        lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        ends = [0, n - 1]
        want = {i: orc.value(buf[i * L:(i + 1) * L].cpu().numpy().tobytes()) for i in ends}
        paths = [
            ("strided", lambda: C.batch_strided(buf, L, L, n, out=out, stream=stream),
             C.describe(n, L, L)),
            ("variable", lambda: C.batch(buf, offs, lens, out=out, stream=stream),
             C.describe(n, L, L, variable=True)),
            ("variable_hint", lambda: C.batch(buf, offs, lens, flags=C.HINT_LARGE_BLOCKS, out=out,
                                              stream=stream),
             C.describe(n, L, L, variable=True, large=True)),
        ]
        for name, fn, desc in paths:
            fn()
            torch.cuda.synchronize()
            ms = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn()
                b.record(stream)
                torch.cuda.synchronize()
                ms.append(a.elapsed_time(b))
            got = out.cpu().numpy().view(np.uint32)
            ok = all(int(got[i]) == want[i] for i in ends)
            med = statistics.median(ms)
            gbs = n * L / (med * 1e-3) / 1e9
            print(json.dumps({"n_blocks": n, "block_bytes": L, "path": name,
                              "kernel": desc.get("kernel"), "ms": round(med, 4),
                              "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                              "verified_ends": ok}), flush=True)
        del buf, offs, lens, out
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
