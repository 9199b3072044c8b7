#!/usr/bin/env python3
"""Tuning / roofline sweep in ONE process (interleaved rounds, median of rounds).

Variants: lanes per unit G, segment size, kernel variant (0 production,
1 no-lookup ablation = memory-side ceiling of the access pattern, 2 default-policy
loads instead of nt),
and the plain coalesced streaming-read kernel (chip read ceiling).
Writes gpurun_out/sweep.json.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--configs", default="2,4")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.json"))
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    import bench

    L = C.enable_diagnostics()
    L.nova_diag_set_variant.argtypes = [ctypes.c_int]
    L.nova_diag_read_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p]
    L.nova_diag_read_stream.restype = ctypes.c_int
    L.nova_diag_set_static_pct.argtypes = [ctypes.c_int]
    L.nova_diag_set_blocks_per_group.argtypes = [ctypes.c_int]
    L.nova_diag_set_chunk_blocks.argtypes = [ctypes.c_int]
    assert L.nova_device_init() == 0
    results = []

    def timeit(fn, iters):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters)]
        fn()
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in ev) / 1e3

    for cfg in [int(c) for c in args.configs.split(",")]:
        n = 1 << 20
        if cfg in (2, 4):
            Lb = 4096 if cfg == 2 else 16384
            total = n * Lb
            buf = torch.empty(total, dtype=torch.uint8, device="cuda")
            C.fill_splitmix64(buf, cfg)
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            nbytes = total
            ref = C.batch_strided(buf, Lb, Lb, n).clone()

            def mk(g, seg, var, bpg=1):
                def f():
                    C.set_tuning(g, seg)
                    L.nova_diag_set_variant(var)
                    L.nova_diag_set_blocks_per_group(bpg)
                    C.batch_strided(buf, Lb, Lb, n, out=out)
                return f
            # seg 0 -> streaming kernel; seg == block length -> units kernel
            variants = [(g, 0, 0, b) for g in (4, 8, 16) for b in (1, 2, 4, 8)]
            variants += [(g, 0, 1, b) for g in (8, 16) for b in (1, 4)]
            variants += [(8, Lb, 0, 1)]
        else:
            offs_np, lens_np, total = bench.config3_layout(n, 3)
            buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
            C.fill_splitmix64(buf, 3)
            offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
            lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            nbytes = int(lens_np.astype(np.uint64).sum())
            ref = C.batch(buf, offs, lens).clone()

            def mk(g, seg, var, chunk=0, waves=0):
                def f():
                    C.set_tuning(g, seg)
                    L.nova_diag_set_variant(var)
                    L.nova_diag_set_chunk_blocks(chunk)
                    L.nova_diag_set_stream_waves(waves)
                    C.batch(buf, offs, lens, out=out)
                return f
            variants = [(16, s, v, 8, w) for s in (16384, 32768, 65536) for v in (0, 2)
                        for w in (8, 12, 16)]
        rs_out = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
        stream_variants = [8192]
        times: dict = {}
        for r in range(args.rounds):
            for key in variants:
                times.setdefault(("units",) + key, []).append(timeit(mk(*key), args.iters))
            for w in stream_variants:
                f = lambda w=w: L.nova_diag_read_stream(buf.data_ptr(), (buf.numel() // 16) * 16,
                                                        rs_out.data_ptr(), w, None)
                times.setdefault(("stream", w), []).append(timeit(f, args.iters))
        # correctness of production variants
        for key in variants:
            if key[2] != 1:
                mk(*key)()
                torch.cuda.synchronize()
                assert torch.equal(out, ref), ("mismatch", cfg, key)
        C.set_tuning(0, 0)
        L.nova_diag_set_variant(0)
        L.nova_diag_set_static_pct(-1)
        L.nova_diag_set_blocks_per_group(0)
        L.nova_diag_set_chunk_blocks(0)
        L.nova_diag_set_stream_waves(0)
        for key, ts in times.items():
            t = statistics.median(ts)
            b = nbytes if key[0] == "units" else (buf.numel() // 16) * 16
            row = {"config": cfg, "kind": key[0], "params": list(key[1:]), "sec": t,
                   "GBps": b / t / 1e9, "GiBps": b / t / 2**30, "frac_8TBs": b / t / 8e12}
            results.append(row)
            print(f"cfg{cfg} {key[0]:6s} {str(key[1:]):18s} {t*1e3:8.3f} ms  "
                  f"{b / t / 1e9:8.1f} GB/s  {100 * b / t / 8e12:5.1f}%", flush=True)
        del buf, out
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
