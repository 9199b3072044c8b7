#!/usr/bin/env python3
"""Variable-length kernels: tuning sweep in ONE process (interleaved rounds,
median launch time per round, median over rounds).

Workloads (all device-resident, splitmix64 data):
  cfg3   BASELINE config 3: 1M blocks {4,16,64} KiB + U[1,64] B, packed (unaligned)
  sst4k  an SSTable-like image: 1M blocks of 4096 + U[0,255] B, 5-B trailer gaps
  log    a log image: 2M records, payload U[1,4096] B, 7-B headers (log write CRC)

Variants: "flat:G:chunk:waves:var" (flat kernel), "units:G:seg:waves:var"
(units kernel, segment size forced) or "rounds:G:chunk*4+sort:waves:var"
(sort 0 none, 1 batch pre-pass, 2 or 3 per chunk; chunk 0 = default), or
"logstream:0:0:0:0" (the whole-image log-record kernel).  var 1 = no-lookup ablation (timing only).
Prints one line per (workload, variant); writes gpurun_out/sweep_flat.json.
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


def make_workload(wl: str, stream):
    """-> (launch fn, algorithmic bytes per launch, tensors to keep alive)."""
    import torch
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_words
    import bench
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_ops import log_layout
    mode = ""
    if wl.endswith("_tw") or wl.endswith("_vf"):  # sst4k_tw / sst4k_vf / log_vf: trailers / verify
        wl, mode = wl[:-3], wl[-2:]
    if wl == "cfg2":
        n, ln = 1 << 20, 4096
        buf = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 2)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        return (lambda: C.batch_strided(buf, ln, ln, n, out=out, stream=stream)), n * ln, (buf, out)
    if wl == "cfg3":
        offs, lens, total = bench.config3_layout(1 << 20, 3)
    elif wl == "sst4k":
        n = 1 << 20
        r = splitmix64_words(5, 0, n)
        lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
        total = int(offs[-1]) + int(lens[-1]) + 5
    elif wl == "c2var":  # config 2's aligned layout through the variable-length path
        n = 1 << 20
        lens = np.full(n, 4096, np.uint32)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(4096)
        total = n * 4096
    elif wl == "sst4k_a":  # sst4k sizes rounded to 128 B, every block 128-B aligned
        n = 1 << 20
        r = splitmix64_words(5, 0, n)
        lens = (np.uint64(4096) + np.uint64(128) * (r % np.uint64(3))).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(128))
        total = int(offs[-1]) + int(lens[-1]) + 128
    elif wl == "log":
        offs, lens, types, total = log_layout(4 << 30, 6)
    elif wl.startswith("log_"):  # log_uN: payload U[1,N]; log_fN: every payload N (4 GiB)
        from novalsm_amd.synth import log_layout as writer_layout
        k, v = wl[4], int(wl[5:])
        n = (4 << 30) // (7 + (v // 2 if k == "u" else v))
        r = splitmix64_words(6, 0, n)
        plens = (r % np.uint64(v) + np.uint64(1)).astype(np.int64) if k == "u" else np.full(n, v, np.int64)
        offs, lens, types, _, total = writer_layout(plens)
        lens = lens.astype(np.uint64)
        wl = "log"
    else:
        raise SystemExit(wl)
    buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 77)
    o = torch.from_numpy(offs.view(np.int64)).cuda()
    if wl == "log":
        ln = torch.from_numpy(lens.astype(np.int64)).cuda()
        buf[o + 4] = (ln & 0xFF).to(torch.uint8)
        buf[o + 5] = (ln >> 8).to(torch.uint8)
        buf[o + 6] = torch.from_numpy(types).cuda()
        alg = int(lens.astype(np.uint64).sum()) + 7 * len(offs)
        if mode == "vf":  # log_vf: verify the records the writer just checksummed
            C.log_write_crcs(buf, o, stream=stream)
            st = torch.empty(len(offs), dtype=torch.uint8, device="cuda")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda")
            return (lambda: C.log_verify_records(buf, o, stream=stream, ok=st, bad=bad)), alg, \
                (buf, o, st, bad)
        return (lambda: C.log_write_crcs(buf, o, stream=stream)), alg, (buf, o)
    ls = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
    alg = int(lens.astype(np.uint64).sum())
    if mode == "tw":  # trailer writer (TableBuilder ordering): reads sum(len), writes 5 B/block
        return (lambda: C.write_trailers(buf, o, ls, 0, True, stream=stream)), alg + 5 * len(offs), \
            (buf, o, ls)
    if mode == "vf":  # read-verify over the same image: reads sum(len + 5)
        C.write_trailers(buf, o, ls, 0, False, stream=stream)
        okb = torch.empty(len(offs), dtype=torch.uint8, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        return (lambda: C.verify_blocks(buf, o, ls, stream=stream, ok=okb, bad=bad)), \
            alg + 5 * len(offs), (buf, o, ls, okb, bad)
    return (lambda: C.batch(buf, o, ls, out=out, stream=stream)), alg, (buf, o, ls, out)


def set_variant(C, v: str) -> None:
    """"flat:G:chunk:waves:var" | "units:G:seg:waves:var" | "auto"."""
    L = C.enable_diagnostics()
    if v == "auto":
        v = "auto:0:0:0:0"
    kind, g, x, w, var = v.split(":")
    g, x, w, var = int(g), int(x), int(w), int(var)
    L.nova_diag_set_variant(var)
    L.nova_diag_set_stream_waves(w)
    if kind == "logstream":  # whole-image log kernel (log workloads only)
        L.nova_diag_set_variable_kernel(4)
        C.set_tuning(0, 0)
        L.nova_diag_set_chunk_blocks(0)
    elif kind == "flat":
        L.nova_diag_set_variable_kernel(2)
        C.set_tuning(g, 0)
        L.nova_diag_set_chunk_blocks(x)
    elif kind == "rounds":  # x: chunk blocks * 4 + sort mode (sort 3 = default 2)
        L.nova_diag_set_variable_kernel(3)
        L.nova_diag_set_rounds_sort(2 if (x & 3) == 3 else (x & 3))
        C.set_tuning(g, 0)
        L.nova_diag_set_chunk_blocks(x >> 2)
    else:
        L.nova_diag_set_variable_kernel(1 if kind == "units" else 0)
        C.set_tuning(g, x)
        L.nova_diag_set_chunk_blocks(0)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg3,sst4k,log")
    ap.add_argument("--variants", default="flat:16:0:0:0,units:16:32768:0:0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=15)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C

    L = C.enable_diagnostics()
    assert L.nova_device_init() == 0
    stream = torch.cuda.current_stream()

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.iters)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in ev) / 1e3

    def setv(v):
        set_variant(C, v)

    rows = []
    for wl in args.workloads.split(","):
        fn, alg, keep = make_workload(wl, stream)
        variants = args.variants.split(",")
        times = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                setv(v)
                times[v].append(timeit(fn))
        for v in variants:
            t = statistics.median(times[v])
            row = {"workload": wl, "variant": v, "ms": round(t * 1e3, 4),
                   "GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 8e12, 4)}
            rows.append(row)
            print(json.dumps(row), flush=True)
        setv("auto")
        del keep, fn
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sweep_flat.json"), "w") as f:
        json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
