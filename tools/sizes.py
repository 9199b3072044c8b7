#!/usr/bin/env python3
"""Throughput vs total bytes and block size (one process, interleaved rounds):
separates per-launch fixed costs from per-byte costs of the access pattern."""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from novalsm_amd import crc32c as C
    L = C.enable_diagnostics()
    L.nova_diag_read_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p]
    assert L.nova_device_init() == 0
    big = torch.empty(32 << 30, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(big, 2)
    out = torch.empty(8 << 20, dtype=torch.int32, device="cuda")
    rs = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
    cases = []
    for gib in (1, 2, 4, 8, 16, 32):
        for blk in (4096, 16384, 65536):
            cases.append(("crc", gib, blk))
        cases.append(("read", gib, 0))
    times = {}

    def run(kind, gib, blk):
        nbytes = gib << 30
        if kind == "crc":
            n = nbytes // blk
            return lambda: C.batch_strided(big, blk, blk, n, out=out[:n])
        return lambda: L.nova_diag_read_stream(big.data_ptr(), nbytes, rs.data_ptr(), 8192, None)

    for _ in range(3):
        for c in cases:
            f = run(*c)
            f()
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(4)]
            for a, b in ev:
                a.record()
                f()
                b.record()
            torch.cuda.synchronize()
            times.setdefault(c, []).append(statistics.median(a.elapsed_time(b) for a, b in ev))
    res = []
    for c, ts in times.items():
        t = statistics.median(ts) / 1e3
        gbs = (c[1] << 30) / t / 1e9
        res.append({"kind": c[0], "GiB": c[1], "block": c[2], "ms": t * 1e3, "GBps": gbs})
        print(f"{c[0]:5s} {c[1]:3d} GiB blk {c[2]:6d}  {t*1e3:8.3f} ms  {gbs:7.1f} GB/s "
              f"{100 * gbs / 8000:5.1f}%", flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "sizes.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
