#!/usr/bin/env python3
"""Per-call latency of one SSTable-sized batch, the way NovaLSM would call it.

NovaLSM checksums one SSTable at a time: all data blocks of a table at the end
of TableBuilder::Finish / StoCWritableFileClient::Format (write side,
ltc/stoc_file_client_impl.cpp:274-289) or a whole prefetched table before its
per-block Table::ReadBlock verify (read side, table/table.cc:425-441,
ltc/stoc_file_client_impl.cpp:843-882).  A call is synchronous for the
calling thread.  For batches of n SSTable-like blocks (4096+U[0,255] B each,
5-B trailers, packed) this prints, per n, one JSON line with:

  dev_wall_us     nova_sstable_verify_blocks on a device-resident image, call +
                  stream sync, host wall clock (launch + kernel + sync)
  dev_kernel_us   the same launch timed with HIP events on the launch stream
  trailers_kernel_us  nova_sstable_write_trailers on the same image (events)
  host_wall_us    image in pinned host memory: H2D copy, verify, D2H of the
                  per-block flags, sync (what an LTC with the table in its
                  RDMA-registered buffer would see)
  cpu_ref_us      reference util/crc32c.cc (oracle/_ref) on one host core over
                  the same blocks (Value over n+1 bytes per block, the verify
                  work of table/table.cc:434-436); the oracle restatement if the
                  reference build is absent

Medians over repeated calls.  Test tooling: the CPU leg is a timed baseline,
never the product path.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sst_layout(n: int, seed: int = 5):
    from novalsm_amd.synth import splitmix64_words
    r = splitmix64_words(seed, 0, n)
    lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    total = int(offs[-1]) + int(lens[-1]) + 5
    return offs, lens, total


def cpu_ref():
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    if os.path.exists(ref):
        lib, fn, kind = ctypes.CDLL(ref), "ref_batch", "reference"
    else:
        from tests.oracle_lib import load_oracle
        lib, fn, kind = load_oracle().lib, "oracle_batch", "port"
    f = getattr(lib, fn)
    f.restype = None
    if kind == "reference":
        f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
    else:  # oracle_batch(base, offsets, lengths, init, out, n, flags)
        f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_uint32]
    return f, kind


def sweep_variants(args, C, torch, stream) -> int:
    from tools.sweep_flat import set_variant
    for n in [int(x) for x in args.sizes.split(",")]:
        offs_np, lens_np, total = sst_layout(n)
        dev = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(dev, 31)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
        set_variant(C, "auto")
        C.write_trailers(dev, offs, lens, 0, False, stream=stream)
        okb = torch.empty(n, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        row = {"n_blocks": n}
        for v in args.variants.split(","):
            set_variant(C, v)
            bad.zero_()
            okb.zero_()
            evs, walls = [], []
            for i in range(120):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                a.record(stream)
                C.verify_blocks(dev, offs, lens, stream=stream, ok=okb, bad=bad)
                b.record(stream)
                b.synchronize()
                if i >= 20:
                    walls.append(time.perf_counter() - t0)
                    evs.append(a.elapsed_time(b) * 1e3)
            good = int(bad.item()) == 0 and bool(okb.cpu().numpy().all())
            row[v] = [round(statistics.median(evs), 1), round(statistics.median(walls) * 1e6, 1), good]
        set_variant(C, "auto")
        print(json.dumps(row), flush=True)
        del dev
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,64,256,1024,4096,16384,65536,262144")
    ap.add_argument("--budget-s", type=float, default=1.0, help="time per leg per size")
    ap.add_argument("--variants", default="",
                    help="comma list of tools/sweep_flat.py variants: device leg only (tuning)")
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    assert C.load().nova_device_init() == 0
    stream = torch.cuda.current_stream()
    fref, kind = cpu_ref()
    if args.variants:
        return sweep_variants(args, C, torch, stream)

    for n in [int(x) for x in args.sizes.split(",")]:
        offs_np, lens_np, total = sst_layout(n)
        dev = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(dev, 31)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
        C.write_trailers(dev, offs, lens, 0, False, stream=stream)  # StoC order: verifiable
        okb = torch.empty(n, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        host = torch.empty(total + 64, dtype=torch.uint8).pin_memory()
        host.copy_(dev.cpu())
        ok_host = torch.empty(n, dtype=torch.uint8).pin_memory()
        bad_host = torch.empty(1, dtype=torch.int32).pin_memory()
        torch.cuda.synchronize()
        sum_len = int(lens_np.astype(np.uint64).sum())

        def reps_for(sec_guess):
            return int(min(2000, max(5, args.budget_s / max(sec_guess, 1e-6))))

        # device-resident, synchronous
        def dev_call():
            C.verify_blocks(dev, offs, lens, stream=stream, ok=okb, bad=bad)
            stream.synchronize()
        for _ in range(20):
            dev_call()
        t0 = time.perf_counter()
        dev_call()
        R = reps_for(time.perf_counter() - t0)
        walls = []
        for _ in range(R):
            t0 = time.perf_counter()
            dev_call()
            walls.append(time.perf_counter() - t0)
        evs = []
        for _ in range(min(R, 200)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            C.verify_blocks(dev, offs, lens, stream=stream, ok=okb, bad=bad)
            b.record(stream)
            b.synchronize()
            evs.append(a.elapsed_time(b) * 1e3)
        assert int(bad.item()) == 0 and bool(okb.cpu().numpy().all()), "verify failed"
        tw = []  # trailer writer (StoC order), same device-resident image
        for i in range(min(R, 200) + 10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            C.write_trailers(dev, offs, lens, 0, False, stream=stream)
            b.record(stream)
            b.synchronize()
            if i >= 10:
                tw.append(a.elapsed_time(b) * 1e3)

        # host-resident: H2D, verify, D2H flags
        def host_call():
            dev.copy_(host, non_blocking=True)
            bad.zero_()
            C.verify_blocks(dev, offs, lens, stream=stream, ok=okb, bad=bad)
            ok_host.copy_(okb, non_blocking=True)
            bad_host.copy_(bad, non_blocking=True)
            stream.synchronize()
        for _ in range(5):
            host_call()
        t0 = time.perf_counter()
        host_call()
        Rh = reps_for(time.perf_counter() - t0)
        hwalls = []
        for _ in range(Rh):
            t0 = time.perf_counter()
            host_call()
            hwalls.append(time.perf_counter() - t0)
        assert int(bad_host[0]) == 0 and bool(ok_host.numpy().all()), "host verify failed"

        # reference on one core: Value over block + type byte
        hb = host.numpy()
        lens1 = (lens_np + np.uint32(1)).astype(np.uint32)
        out = np.empty(n, np.uint32)
        args_c = [hb.ctypes.data, offs_np.ctypes.data, lens1.ctypes.data, None, out.ctypes.data, n]
        if kind != "reference":
            args_c.append(0)
        t0 = time.perf_counter()
        fref(*args_c)
        Rc = max(3, min(200, int(args.budget_s / max(time.perf_counter() - t0, 1e-6))))
        cw = []
        for _ in range(Rc):
            t0 = time.perf_counter()
            fref(*args_c)
            cw.append(time.perf_counter() - t0)
        # the reference's CRCs must match the trailers the GPU wrote
        stored = np.array([int.from_bytes(hb[int(o) + int(l) + 1:int(o) + int(l) + 5].tobytes(), "little")
                           for o, l in zip(offs_np[:64], lens_np[:64])], np.uint32)
        mask = lambda c: ((((c >> np.uint32(15)) | (c << np.uint32(17))) + np.uint32(0xa282ead8))
                          & np.uint32(0xFFFFFFFF))
        assert np.array_equal(mask(out[:64].astype(np.uint64)).astype(np.uint32), stored), "ref mismatch"

        med = statistics.median
        row = {"n_blocks": n, "bytes": sum_len, "MiB": round(sum_len / 2**20, 2),
               "dev_wall_us": round(med(walls) * 1e6, 1),
               "dev_kernel_us": round(med(evs), 1),
               "trailers_kernel_us": round(med(tw), 1),
               "host_wall_us": round(med(hwalls) * 1e6, 1),
               "cpu_ref_us": round(med(cw) * 1e6, 1),
               "cpu_kind": kind,
               "dev_wall_GiBps": round(sum_len / med(walls) / 2**30, 1),
               "host_wall_GiBps": round(sum_len / med(hwalls) / 2**30, 1),
               "cpu_ref_GiBps": round(sum_len / med(cw) / 2**30, 2)}
        print(json.dumps(row), flush=True)
        del dev, host
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
