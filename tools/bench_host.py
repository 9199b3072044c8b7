#!/usr/bin/env python3
"""Host-resident SSTable paths: rates that
include the PCIe copies, next to the zero-copy form (kernels reading and
writing pinned host memory directly) and the device-resident kernel.

Image: n SSTable-like blocks of 4096+U[0,255] B with 5-B trailers, packed
(the Format() buffer / ReadAll() slab of ltc/stoc_file_client_impl.cpp:183-377,
:843-882), in pinned host memory.  Ops:
  crc       nova_crc32c_batch_host            (H2D blocks -> CRC -> D2H 4 B/block)
  trailers  nova_sstable_write_trailers_host  (H2D -> CRC -> D2H; host stores 5 B/block)
  verify    nova_sstable_verify_blocks_host   (H2D blocks+trailers -> verify -> D2H 1 B/block)
  zc_*      the device entry points on the pinned image itself (zero-copy)
  dev_verify the device-resident image (HBM), for scale
Rates are payload GB/s = sum(block bytes) / wall time of the synchronous call
(median of --iters).  One JSON line per op; also a per-SSTable (4K blocks) row.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--streams", type=int, default=3)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_bytes, splitmix64_words
    from tests.oracle_lib import load_oracle

    assert C.load().nova_device_init() == 0
    orc = load_oracle()

    def layout(n, seed):
        r = splitmix64_words(seed, 0, n)
        lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
        return offs, lens, int(offs[-1]) + int(lens[-1]) + 5

    def wall(fn, iters):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    chunk = args.chunk_mib << 20
    rows = []
    for n, iters in ((args.n, args.iters), (4096, 30)):
        offs, lens, total = layout(n, 5)
        payload = int(lens.astype(np.uint64).sum())
        img = torch.from_numpy(splitmix64_bytes(31, total)).pin_memory()
        C.write_trailers_host(img, offs, lens, 0, False, chunk_bytes=chunk, n_streams=args.streams)
        # sample check against the oracle
        idx = np.linspace(0, n - 1, 33).astype(np.int64)
        h = img.numpy()
        ok = all(orc.verify(h[int(offs[i]):int(offs[i]) + int(lens[i]) + 5].tobytes()) for i in idx)
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        okd = torch.empty(n, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        outd = torch.empty(n, dtype=torch.int32, device="cuda")
        L = C.load()
        ops = {
            "crc": lambda: C.batch_host(img, offs, lens, chunk_bytes=chunk, n_streams=args.streams),
            "trailers": lambda: C.write_trailers_host(img, offs, lens, 0, False, chunk_bytes=chunk,
                                                      n_streams=args.streams),
            "verify": lambda: C.verify_blocks_host(img, offs, lens, chunk_bytes=chunk,
                                                   n_streams=args.streams),
            "zc_crc": lambda: L.nova_crc32c_batch(img.data_ptr(), do.data_ptr(), dl.data_ptr(), None,
                                                  outd.data_ptr(), n, 0, None),
            "zc_trailers": lambda: L.nova_sstable_write_trailers(img.data_ptr(), do.data_ptr(),
                                                                 dl.data_ptr(), n, 0, None),
            "zc_verify": lambda: L.nova_sstable_verify_blocks(img.data_ptr(), do.data_ptr(),
                                                              dl.data_ptr(), n, okd.data_ptr(),
                                                              bad.data_ptr(), None),
        }
        dimg = img.cuda()
        ops["dev_verify"] = lambda: C.verify_blocks(dimg, do, dl, ok=okd, bad=bad)
        for name, fn in ops.items():
            sec = wall(fn, iters)
            row = {"op": name, "n_blocks": n, "payload_bytes": payload,
                   "ms": round(sec * 1e3, 3), "GBps": round(payload / sec / 1e9, 2),
                   "GiBps": round(payload / sec / 2**30, 2), "verified_sample": bool(ok),
                   "chunk_mib": args.chunk_mib, "streams": args.streams}
            rows.append(row)
            print(json.dumps(row), flush=True)
        okh, nb = C.verify_blocks_host(img, offs, lens, chunk_bytes=chunk)
        assert okh.all() and nb == 0
        del img, dimg
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_host.json"), "w") as f:
        json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
