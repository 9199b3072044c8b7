#!/usr/bin/env python3
"""Device-resident batched CRC32C throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config 2|3|4|5|sst4k_trailers|sst4k_verify|log*|parity]
                    [--secondary 3,4,...,sst_engine|none] [--settle-ms MS] [--detail-out F]

One step = one pass of the hot path (a nova_crc32c_batch* call through the
C-ABI) over one batch of synthetic SSTable blocks already resident in HBM.

Workloads (BASELINE.json configs; per GPU, weak scaling):
  2  1M x 4 KiB uniform blocks (4 GiB) -- the headline `value` (configs[1])
  3  1M mixed {4,16,64} KiB + U[1,64] B unaligned blocks (~28 GiB), the
     variable-length kernel with NOVA_CRC32C_HINT_LARGE_BLOCKS
  4  1M x 16 KiB (16 GiB; 8M x 16 KiB over 8 GPUs)
  5  host-resident (pinned) 16 KiB blocks streamed H2D -> CRC -> D2H; its own
     line, never the device-resident value
  sst4k_trailers / sst4k_verify  NovaLSM's live block shape: 1M x (4096+U[0,255])
     B blocks back to back with 5-B trailers, unaligned -- the trailer writer
     (nova_sstable_write_trailers, TableBuilder ordering, table/table_builder.cc:
     192-212) and the read-verify (nova_sstable_verify_blocks, table/table.cc:
     434-440) over that image
  log4k_* / log512_* / parity  SURVEY 8(f) rows 3-4
  sst_engine  8 and 16 native threads calling nova_sst_queue_* on one 16.5 MiB
     SSTable each, back to back, through the persistent engine (N = 1 only)
By default the line carries config 2 as `value` and configs 3, 4 and the two
SSTable-shape workloads as `secondary` objects measured in the same run, each
with its own roofline.

Multi-GPU: one process per GPU.  Run under torchrun (WORLD_SIZE set) each rank
takes its device from LOCAL_RANK; run as `python bench.py --gpus N` without
torchrun, this process starts `torch.distributed.run` with N ranks as a CHILD
process before anything touches the GPU, and exits with its code.  Ranks
checksum their own shards (no data-path collective); RCCL carries only the
barriers, the max-over-ranks time and the per-rank kernel times.

Timing: a time-based settle (--settle-ms of back-to-back launches: the first
~25 launches of a burst run up to 30% slower in a power-management transient,
DESIGN.md 3.6), then W untimed warmup launches, then K launches bracketed by
barrier + synchronize; `value` = bytes of all ranks / max-over-ranks wall time.
`roofline.achieved` = algorithmic bytes per launch (sum of block lengths;
SURVEY.md 8(d)) / the average launch time from HIP events recorded on the
launch stream.  `cpu_baseline` = the reference util/crc32c.cc (oracle/_ref,
compiled from the reference sources) or the oracle restatement, timed on this
host's cores (rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s device-resident batched CRC32C, 4-64 KiB blocks; % HBM-read roofline"


def config3_layout(n: int, seed: int = 3):
    """BASELINE config 3: sizes uniform over {4096,16384,65536} + U[1,64] bytes,
    chosen by splitmix64(seed), packed back to back (unaligned starts/lengths)."""
    from novalsm_amd.synth import splitmix64_words
    r = splitmix64_words(seed, 0, n)
    cls = np.array([4096, 16384, 65536], dtype=np.uint64)[(r % np.uint64(3)).astype(np.int64)]
    jit = ((r >> np.uint64(8)) % np.uint64(64)) + np.uint64(1)
    lens = (cls + jit).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    total = int(offs[-1]) + int(lens[-1])
    return offs, lens, total


SST_WORKLOADS = ("sst4k_trailers", "sst4k_verify")
# NovaLSM's many-caller shape through the persistent engine
ENGINE_WORKLOAD = "sst_engine"
# SURVEY 8(f) rows 3-4 as driver-measured secondaries
LOG_WORKLOADS = ("log4k_write", "log4k_verify", "log512_write", "log512_verify")
OPS_WORKLOADS = LOG_WORKLOADS + ("parity",)


def sst4k_layout(n: int, seed: int = 5):
    """NovaLSM's data blocks: 4096+U[0,255] B (a 4 KiB block_size block closes
    past 4 KiB, table/block_builder.cc:56-60), back to back with their 5-B
    trailers, from splitmix64(seed)."""
    from novalsm_amd.synth import splitmix64_words
    r = splitmix64_words(seed, 0, n)
    lens = (np.uint64(4096) + (r % np.uint64(256))).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + np.uint64(5))
    total = int(offs[-1]) + int(lens[-1]) + 5
    return offs, lens, total


def log_bench_layout(pmax: int, total_target: int = 4 << 30, seed: int = 6):
    """A ~4 GiB log file as log::Writer lays it out (db/log_writer.cc:53-97):
    logical records of U[1,pmax] B payload from splitmix64(seed), fragmented at
    32 KiB blocks.  (offsets u64, payload lengths u64, types u8, total bytes)."""
    from novalsm_amd.synth import log_layout_fast, splitmix64_words
    n = total_target // (7 + (pmax + 1) // 2)
    r = splitmix64_words(seed, 0, n)
    plens = ((r % np.uint64(pmax)) + np.uint64(1)).astype(np.int64)
    offs, lens, types, _, total = log_layout_fast(plens)
    return offs, lens.astype(np.uint64), types, total


def workload(cfg):
    if cfg in LOG_WORKLOADS:
        pmax = 4096 if cfg.startswith("log4k") else 512
        op = "write" if cfg.endswith("write") else "verify"
        what = ("record CRC write (db/log_writer.cc:99-114)" if op == "write"
                else "record verify (db/log_reader.cc:196-262)")
        return {"workload": f"{cfg}: ~4 GiB log image per GPU, log::Writer layout of U[1,{pmax}] B payloads, "
                            f"{what}", "n_blocks": None, "block_bytes": None, "kind": f"log_{op}",
                "pmax": pmax}
    if cfg == "parity":
        return {"workload": "parity: XOR parity of 8 fragments x 512 MiB per GPU "
                            "(ltc/stoc_file_client_impl.cpp:334-349)",
                "n_blocks": 8, "block_bytes": 512 << 20, "kind": "parity"}
    if cfg == "sst4k_trailers":
        return {"workload": "sst4k_trailers: 1M x (4096+U[0,255]) B blocks + 5-B trailers per GPU, "
                            "trailer writer (TableBuilder ordering)",
                "n_blocks": 1 << 20, "block_bytes": None, "kind": "sst_trailers"}
    if cfg == "sst4k_verify":
        return {"workload": "sst4k_verify: 1M x (4096+U[0,255]) B blocks + 5-B trailers per GPU, "
                            "read-verify",
                "n_blocks": 1 << 20, "block_bytes": None, "kind": "sst_verify"}
    if cfg == 2:
        return {"workload": "config2: 1M x 4 KiB uniform blocks per GPU (BASELINE configs[1])",
                "n_blocks": 1 << 20, "block_bytes": 4096, "kind": "strided"}
    if cfg == 3:
        return {"workload": "config3: 1M mixed {4,16,64} KiB + U[1,64] B unaligned blocks per GPU",
                "n_blocks": 1 << 20, "block_bytes": None, "kind": "variable"}
    if cfg == 4:
        return {"workload": "config4: 1M x 16 KiB per GPU (8M x 16 KiB over 8 GPUs)",
                "n_blocks": 1 << 20, "block_bytes": 16384, "kind": "strided"}
    if cfg == 5:
        return {"workload": "config5: pinned-host 16 KiB blocks streamed H2D->CRC->D2H",
                "n_blocks": 1 << 18, "block_bytes": 16384, "kind": "host"}
    raise SystemExit(f"unknown config {cfg}")


# ---- host CPU share ---------------------------------------------------------

def host_cpus():
    """(threads to use, description): the CPUs this process may run on
    (sched_getaffinity), capped by a cgroup v2 CPU quota and by the host's
    stated per-job CPU share (OMP_NUM_THREADS: 16 per GPU on the GPU boxes)
    when those are set.  All three are reported."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    share = None
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "")) or None
    except ValueError:
        pass
    threads = aff
    if quota is not None:
        threads = min(threads, int(math.ceil(quota)))
    if share is not None:
        threads = min(threads, share)
    return max(1, threads), {"affinity_cpus": aff, "cgroup_quota_cpus": quota,
                             "omp_num_threads": share}


def cpu_baseline(seconds: float = 4.0):
    """Reference util/crc32c.cc (oracle/_ref) if built, else the oracle restatement,
    on BASELINE config 1: 1024 x 4 KiB splitmix64(seed 1) blocks, repeated,
    on 1 thread and on all of this process's CPUs; plus the reference's own
    db_bench crc32c method (benchmarks/db_bench.cc:635-652: Value() over the
    same 4 KiB of 'x' until 500 MiB, 1 thread)."""
    import ctypes
    from novalsm_amd.synth import splitmix64_bytes
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    n, L = 1024, 4096
    buf = splitmix64_bytes(1, n * L)
    out = np.empty(n, dtype=np.uint32)
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        fn, dbb = lib.ref_batch_strided_mt, lib.ref_dbbench_crc32c
        kind = "reference"
    else:
        from tests.oracle_lib import load_oracle
        lib = load_oracle().lib
        fn, dbb = lib.oracle_batch_strided_mt, lib.oracle_dbbench_crc32c
        kind = "port"
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    dbb.restype = ctypes.c_uint32
    dbb.argtypes = [ctypes.c_int64]

    def rate(th):
        reps = 1
        while True:
            t0 = time.perf_counter()
            fn(buf.ctypes.data, L, L, n, out.ctypes.data, th, reps)
            dt = time.perf_counter() - t0
            if dt > seconds / 4 or reps > 1 << 20:
                break
            reps *= 4
        reps = max(1, int(reps * seconds / max(dt, 1e-6)))
        t0 = time.perf_counter()
        fn(buf.ctypes.data, L, L, n, out.ctypes.data, th, reps)
        dt = time.perf_counter() - t0
        return n * L * reps / dt / 2**30, reps

    threads, share = host_cpus()
    one, r1 = rate(1)
    allc, r2 = rate(threads)
    db_bytes = 500 * 1048576
    t0 = time.perf_counter()
    crc = dbb(db_bytes)
    db_s = time.perf_counter() - t0
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(allc, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "single_core": round(one, 3), "cpu": model, **share,
            "product_host_extend": product_host_extend(seconds / 4),
            "sample": f"BASELINE config 1: 1024 x 4 KiB splitmix64(seed 1) blocks, "
                      f"{r2} reps on {threads} threads (+{r1} reps on 1 thread), g++ -O2",
            "db_bench_crc32c": {"value": round(db_bytes / db_s / 2**30, 3), "unit": "GiB/s",
                                "threads": 1, "crc": f"0x{crc:08x}",
                                "sample": "benchmarks/db_bench.cc:635-652: Value(4 KiB of 'x') "
                                          "until 500 MiB, 1 thread"}}


def product_host_extend(seconds: float = 1.0) -> dict:
    """The product's own scalar drop-in (leveldb::crc32c::Extend in
    crc32c_host.cpp, what every Extend() of an unmodified NovaLSM runs after
    INTEGRATION.md level 1), 1 thread, on 4 KiB and 1 MiB buffers; the loop
    runs natively (nova_diag_host_extend_loop: the same object code)."""
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_bytes
    fn = C.load_diag().nova_diag_host_extend_loop
    buf = splitmix64_bytes(9, 1 << 20)
    res = {"threads": 1, "unit": "GiB/s",
           "impl": "3 interleaved SSE4.2 crc32 chains joined by GF(2) shifts (crc32c_host.cpp)"}
    for size, key in ((4096, "4KiB"), (1 << 20, "1MiB")):
        reps = max(1, int(16 * 2**20 // size))
        while True:
            t0 = time.perf_counter()
            fn(buf.ctypes.data, size, reps)
            dt = time.perf_counter() - t0
            if dt >= seconds / 2:
                break
            reps *= 2
        res[key] = round(reps * size / dt / 2**30, 3)
    return res


# ---- the persistent engine under many callers ------------------------------------

def engine_measure(args, ctx: Ctx) -> dict:
    """NovaLSM's per-SSTable calls as they arrive: T native
    threads (8, 16; and one verify caller alone for the per-request latency,
    `lone`), each with its own stream and 4096-block SSTable image
    (4096+U[0,255] B + 5-B trailers, ~16.5 MiB: one table per call), calling
    nova_sst_queue_verify_blocks / nova_sst_queue_write_trailers back to back on
    the resident engine (crc32c_engine.hip), 0.3 s warm then a 1 s window
    (novalsm_amd/callers.py -> sst_callers.cpp).  Every verify call's mismatch
    count and flags and every table's final trailers are checked natively
    after the window.  Aggregate GB/s = algorithmic bytes of the calls that
    completed in the window / the window; latencies are per call, host clock."""
    from novalsm_amd import callers
    runs = []
    # one caller alone: the per-request latency host to host
    r1 = callers.run("verify", 1, 4096, args.engine_secs, "engine", warm_s=0.3, seed=10)
    lone = {"p50_us": r1["p50_us"], "p99_us": r1["p99_us"], "max_us": r1["max_us"],
            "GBps": r1["aggregate_GBps"], "verified": r1["verified"] and r1["engine"]["fallbacks"] == 0}
    for op in ("verify", "trailers"):
        for t in (8, 16):
            r = callers.run(op, t, 4096, args.engine_secs, "engine", warm_s=0.3, seed=11 + t)
            e = r["engine"]
            runs.append({"op": op, "threads": t, "GBps": r["aggregate_GBps"], "frac": r["frac_of_8TBps"],
                         "p50_us": r["p50_us"], "p99_us": r["p99_us"], "max_us": r["max_us"],
                         "calls": r["calls_in_window"], "launches": e["launches"],
                         "fallbacks": e["fallbacks"], "exits_yield": e["exits_yield"],
                         "cpu_throttled_us": r["cpu_throttled_us"], "verified": r["verified"]})
    ok = all(x["verified"] and x["fallbacks"] == 0 for x in runs) and lone["verified"]
    best = max(runs, key=lambda x: x["GBps"])
    return {"metric": "GB/s of 16.5 MiB SSTables through nova_sst_queue_* from 8/16 threads (persistent "
                      "engine); % of 8 TB/s", "config": ENGINE_WORKLOAD,
            "value": round(best["GBps"] * 1e9 / 2**30, 2), "unit": "GiB/s", "runs": runs, "lone": lone,
            "table": "4096 x (4096+U[0,255]) B + 5-B trailers per call; window %.1f s" % args.engine_secs,
            "verified_sample": ok}


# ---- launcher -----------------------------------------------------------------

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """Start n ranks under torch.distributed.run as a child process (this
    process has not touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ---- same-run ceilings ------------------------------------------------------------

def _events_avg_s(torch, fn, stream, warmup: int = 10, reps: int = 30) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / reps / 1e3


def parity_copy_ceiling(torch, C, buf, fo, plen, stream, args) -> dict:
    """The XOR parity kernel's own bound, in the same run: a copy kernel of the
    same traffic shape -- the 8 fragments read and the 512 MiB written, nothing
    computed (copy_ceiling_kernel of the diagnostics library) --
    at 1-8 chunks per lane (8: the product's own shape), non-temporal loads
    and stores, one-pass grid -- and the runtime's device-to-device copy of
    one fragment.  The fastest form is the ceiling."""
    D = C.load_diag()
    sink = torch.empty(256, dtype=torch.int32, device=buf.device)
    tmp = torch.empty(plen, dtype=torch.uint8, device=buf.device)
    best = None
    forms = {}
    for u in (1, 2, 4, 8):
        v = u | 1 << 4 | 1 << 5  # kind 0 (8 reads + 1 write), nt loads, nt stores

        def f(v=v):
            rc = D.nova_diag_copy_ceiling(buf.data_ptr(), fo.data_ptr(), plen, tmp.data_ptr(),
                                          sink.data_ptr(), 0, v, stream.cuda_stream)
            assert rc == 0, rc
        sec = _events_avg_s(torch, f, stream)
        gbs = 9 * plen / sec / 1e9
        forms[f"copy_kernel_{u}_chunks"] = round(gbs, 1)
        if best is None or gbs > best["achieved"]:
            best = {"kind": "8-read + 1-write copy, no XOR (copy_ceiling_kernel, diagnostics library)",
                    "chunks_per_lane": u, "achieved": round(gbs, 1), "unit": "GB/s",
                    "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4)}
    # the runtime's own device-to-device copy of one fragment (1 read + 1 write:
    # HBM's mixed read/write rate as the driver's copy engine-free path reaches it)
    src = buf[int(fo[0].item()):int(fo[0].item()) + plen]
    sec = _events_avg_s(torch, lambda: tmp.copy_(src), stream)
    gbs = 2 * plen / sec / 1e9
    forms["hip_d2d_copy"] = round(gbs, 1)
    if gbs > best["achieved"]:
        best = {"kind": "hipMemcpyAsync device-to-device copy of one fragment (torch copy_)",
                "achieved": round(gbs, 1), "unit": "GB/s", "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4)}
    best["forms_GBps"] = forms
    del tmp, sink
    return best


def read_ceiling(torch, C, buf, nbytes: int, stream) -> dict:
    """Config 2's own bound, in the same run ("also report against
    a measured device read-only streaming ceiling"): a kernel that only reads
    the same bytes and XOR-folds them (read_ceiling_kernel of the diagnostics
    library), non-temporal loads, 4-16 in flight per lane, over a few grids; the
    fastest form is the ceiling (tools/read_probe.hip swept 72 shapes: 88.9 %
    at best, profiles/r05_read_ceiling.log)."""
    D = C.load_diag()
    sink = torch.empty(1024 * 1024, dtype=torch.int32, device=buf.device)
    best, forms = None, {}
    for u, wgs, t1024 in ((8, 256, False), (4, 1024, False), (16, 256, False), (8, 256, True)):
        v = u | 0x100 | (0x200 if t1024 else 0)

        def f(v=v, wgs=wgs):
            rc = D.nova_diag_read_ceiling(buf.data_ptr(), nbytes, sink.data_ptr(), wgs, v, stream.cuda_stream)
            assert rc == 0, rc
        sec = _events_avg_s(torch, f, stream)
        gbs = nbytes / sec / 1e9
        forms[f"u{u}_wg{wgs}_t{1024 if t1024 else 256}"] = round(gbs, 1)
        if best is None or gbs > best["achieved"]:
            best = {"kind": "read-only nt stream of the same bytes (read_ceiling_kernel, diagnostics library)",
                    "achieved": round(gbs, 1), "unit": "GB/s", "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4)}
    best["forms_GBps"] = forms
    del sink
    return best


def h2d_ceiling(torch, host, dev_tmp, chunk: int, n_streams: int = 3) -> dict:
    """Config 5's own bound, in the same run: pinned-host -> HBM copies of the
    same bytes with hipMemcpyAsync (torch copy_, non_blocking), as one copy and
    as chunk-sized copies over n_streams streams; the faster is the ceiling."""
    total = host.numel()
    res = {}

    def one():
        dev_tmp.copy_(host, non_blocking=True)

    streams = [torch.cuda.Stream() for _ in range(n_streams)]

    def chunked():
        for i, o in enumerate(range(0, total, chunk)):
            with torch.cuda.stream(streams[i % n_streams]):
                dev_tmp[o:o + chunk].copy_(host[o:o + chunk], non_blocking=True)

    for name, fn in (("one_copy", one), (f"chunks_{chunk >> 20}MiB_x{n_streams}_streams", chunked)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = total * reps / (time.perf_counter() - t0) / 1e9
    best = max(res, key=res.get)
    return {"kind": "pinned H2D hipMemcpyAsync of the same bytes", "form": best,
            "achieved": round(res[best], 2), "unit": "GB/s",
            "forms": {k: round(v, 2) for k, v in res.items()}}


# ---- HBM preflight -----------------------------------------------------------------

def hbm_need(wl) -> int:
    """Device bytes a workload allocates (its image, descriptors and outputs)."""
    n = wl["n_blocks"]
    if wl["kind"] == "strided":
        return n * wl["block_bytes"] + 4 * n
    if wl["kind"] in ("sst_trailers", "sst_verify"):
        return n * (4096 + 128 + 5) + 17 * n
    if wl["kind"] == "variable":
        return n * (28 << 10) + 16 * n
    if wl["kind"] in ("log_write", "log_verify"):
        return (4 << 30) + (4 << 30) // (7 + (wl["pmax"] + 1) // 2) * 26
    if wl["kind"] == "parity":
        return 9 * wl["block_bytes"]
    if wl["kind"] == "host":
        return 2 * (4096 * wl["block_bytes"]) * 4
    return 0


def hbm_preflight(cfg, wl, ctx) -> None:
    """Fail loudly, on every rank, when this GPU cannot hold the workload (a
    shape the driver's first 8-GPU run may meet untried), instead of a late
    out-of-memory inside a kernel launch or a silent partial run."""
    import torch
    free, total = torch.cuda.mem_get_info(ctx.dev)
    need = hbm_need(wl)
    if need + (512 << 20) > free:
        msg = {"error": "HBM preflight", "config": cfg, "rank": ctx.rank, "need_bytes": need,
               "free_bytes": free, "total_bytes": total}
        print(json.dumps(msg), file=sys.stderr, flush=True)
        raise SystemExit(4)


# ---- one device-resident config ------------------------------------------------

class Ctx:
    """world/rank of this run; `on` when a process group exists (every run
    started by torch.distributed.run, a world of 1 included, so the RCCL path
    is the one a 1-GPU torchrun exercises)."""

    def __init__(self, world, rank, dev, dist, on):
        self.world, self.rank, self.dev, self.dist, self.on = world, rank, dev, dist, on

    def barrier(self):
        if self.on:
            self.dist.barrier()

    def all_gather_f64(self, x: float):
        import torch
        if not self.on:
            return [x]
        t = torch.tensor([x], dtype=torch.float64, device=self.dev)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [float(p.item()) for p in parts]


def run_device_config(cfg: int, args, ctx: Ctx) -> dict:
    import torch
    from novalsm_amd import crc32c as C
    wl = workload(cfg)
    hbm_preflight(cfg, wl, ctx)
    stream = torch.cuda.current_stream()
    n = wl["n_blocks"]
    seed = cfg
    ceiling = None
    if wl["kind"] in ("log_write", "log_verify"):
        offs_np, lens_np, types_np, total = log_bench_layout(wl["pmax"])
        n = len(offs_np)
        buf = torch.empty(total + 64, dtype=torch.uint8, device=ctx.dev)
        C.fill_splitmix64(buf, 41, first_word=ctx.rank * (total // 8))
        offs = torch.from_numpy(offs_np.view(np.int64)).to(ctx.dev)
        ln_t = torch.from_numpy(lens_np.view(np.int64)).to(ctx.dev)
        buf[offs + 4] = (ln_t & 0xFF).to(torch.uint8)  # header length (LE16) and type
        buf[offs + 5] = (ln_t >> 8).to(torch.uint8)
        buf[offs + 6] = torch.from_numpy(types_np).to(ctx.dev)
        del ln_t
        sum_rec = int(lens_np.sum()) + 7 * n
        if wl["kind"] == "log_write":
            def step():
                C.log_write_crcs(buf, offs, stream=stream, buf_len=total)
            bytes_step = sum_rec  # type + payload + length/type header read, CRC field written
            out = None
        else:
            C.log_write_crcs(buf, offs, stream=stream, buf_len=total)
            out = torch.empty(n, dtype=torch.uint8, device=ctx.dev)
            bad = torch.zeros(1, dtype=torch.int32, device=ctx.dev)

            def step():
                C.log_verify_records(buf, offs, stream=stream, ok=out, bad=bad, buf_len=total)
            bytes_step = sum_rec + n  # the whole records read, one status byte written
        dispatch = C.describe(n, total // n, 0, log=True, log_verify=wl["kind"] == "log_verify")
        dispatch["op"] = "nova_log_write_crcs" if wl["kind"] == "log_write" else "nova_log_verify_records"
        dispatch["records"] = n
        dispatch["mean_record_span"] = round(total / n, 1)
        lens_np = None
    elif wl["kind"] == "parity":
        k, plen = wl["n_blocks"], wl["block_bytes"]
        buf = torch.empty(k * plen, dtype=torch.uint8, device=ctx.dev)
        C.fill_splitmix64(buf, 51, first_word=ctx.rank * (k * plen // 8))
        fo = torch.arange(k, dtype=torch.int64, device=ctx.dev) * plen
        out = torch.empty(plen, dtype=torch.uint8, device=ctx.dev)

        def step():
            C.xor_parity(buf, fo, plen, out=out, stream=stream)
        bytes_step = (k + 1) * plen  # k fragments read, the parity written
        dispatch = {"op": "nova_xor_parity", "kernel": "xor_parity_kernel<8, 1>", "fragments": k,
                    "fragment_bytes": plen}
        offs_np = lens_np = None
        ceiling = parity_copy_ceiling(torch, C, buf, fo, plen, stream, args)
    elif wl["kind"] == "strided":
        L = wl["block_bytes"]
        total = n * L
        buf = torch.empty(total, dtype=torch.uint8, device=ctx.dev)
        # rank r's shard of the global batch: words [r*total/8, (r+1)*total/8)
        C.fill_splitmix64(buf, seed, first_word=ctx.rank * (total // 8))
        out = torch.empty(n, dtype=torch.int32, device=ctx.dev)

        def step():
            C.batch_strided(buf, L, L, n, out=out, stream=stream)
        lens_np = offs_np = None
        bytes_step = total
        dispatch = C.describe(n, L, L, variable=False)
    elif wl["kind"] in ("sst_trailers", "sst_verify"):
        offs_np, lens_np, total = sst4k_layout(n, 5)
        buf = torch.empty(total + 64, dtype=torch.uint8, device=ctx.dev)
        C.fill_splitmix64(buf, 31, first_word=ctx.rank * (total // 8))
        offs = torch.from_numpy(offs_np.view(np.int64)).to(ctx.dev)
        lens = torch.from_numpy(lens_np.view(np.int32)).to(ctx.dev)
        sum_len = int(lens_np.astype(np.uint64).sum())
        if wl["kind"] == "sst_trailers":
            def step():  # TableBuilder's ordering ('!' after the encode)
                C.write_trailers(buf, offs, lens, 0, True, stream=stream)
            # algorithmic bytes: the blocks read and the trailers written
            bytes_step = sum_len + 5 * n
            out = None
        else:
            C.write_trailers(buf, offs, lens, 0, False, stream=stream)  # StoC order: verifiable
            out = torch.empty(n, dtype=torch.uint8, device=ctx.dev)
            bad = torch.zeros(1, dtype=torch.int32, device=ctx.dev)

            def step():
                C.verify_blocks(buf, offs, lens, stream=stream, ok=out, bad=bad)
            # algorithmic bytes: block + type byte + stored CRC read, one flag written
            bytes_step = sum_len + 6 * n
        dispatch = C.describe(n, 4096 + 128, 0, variable=True)
        if wl["kind"] == "sst_trailers":  # two passes: the CRC pass in store mode
            dispatch.update({"op": "nova_sstable_write_trailers",
                             "kernels": ["trailer_layout_kernel", dispatch["kernel"], "trailer_rmw_kernel"]})
        else:
            dispatch.update({"op": "nova_sstable_verify_blocks",
                             "kernel": dispatch["kernel"].replace(", 0>", ", 2>")})  # MODE 2: verify
    else:
        offs_np, lens_np, total = config3_layout(n, seed)
        buf = torch.empty(total + 64, dtype=torch.uint8, device=ctx.dev)
        C.fill_splitmix64(buf, seed, first_word=ctx.rank * (total // 8))
        offs = torch.from_numpy(offs_np.view(np.int64)).to(ctx.dev)
        lens = torch.from_numpy(lens_np.view(np.int32)).to(ctx.dev)
        out = torch.empty(n, dtype=torch.int32, device=ctx.dev)
        # config 3 is LevelDB's block_size sweep (mean ~28 KiB): the caller
        # knows its block_size and passes the scheduling hint (results are
        # identical without it; include/nova_crc32c.h)
        hint = C.HINT_LARGE_BLOCKS

        def step():
            C.batch(buf, offs, lens, flags=hint, out=out, stream=stream)
        bytes_step = int(lens_np.astype(np.uint64).sum())
        dispatch = C.describe(n, 0, 0, variable=True, large=True)

    # settle: back-to-back launches for >= settle_ms (time-based), then warmup
    torch.cuda.synchronize()
    ctx.barrier()
    t_s = time.perf_counter()
    settle_launches = 0
    while (time.perf_counter() - t_s) * 1e3 < args.settle_ms:
        for _ in range(8):
            step()
        settle_launches += 8
        torch.cuda.synchronize()
    settle_ms = (time.perf_counter() - t_s) * 1e3
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    ctx.barrier()
    dt = time.perf_counter() - t0
    dts = ctx.all_gather_f64(dt)
    dt_max = max(dts)
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    rank_kernel_ms = ctx.all_gather_f64(avg_launch_s * 1e3)

    # sample verification against the CPU oracle (outside the timed region)
    verified = None
    if args.verify:
        from tests.oracle_lib import load_oracle
        orc = load_oracle()
        idx = np.linspace(0, n - 1, 257).astype(np.int64)
        ok = True
        if wl["kind"] == "log_write":
            idx = np.linspace(0, n - 1, 257).astype(np.int64)
            offs_h = offs.cpu().numpy().view(np.uint64)
            for i in idx:
                a = int(offs_h[i])
                L_ = int(buf[a + 4].item()) | (int(buf[a + 5].item()) << 8)
                rec = buf[a:a + 7 + L_].cpu().numpy()
                want = orc.mask(orc.value(rec[6:].tobytes()))  # type byte + payload
                ok &= int.from_bytes(rec[:4].tobytes(), "little") == want
        elif wl["kind"] == "log_verify":
            ok = int(bad.item()) == 0 and bool((out.cpu().numpy() == C.LOG_OK).all())
        elif wl["kind"] == "parity":
            k, plen = wl["n_blocks"], wl["block_bytes"]
            for i in np.linspace(0, plen - 4097, 33).astype(np.int64):
                want = np.zeros(4096, np.uint8)
                for f in range(k):
                    want ^= buf[f * plen + i:f * plen + i + 4096].cpu().numpy()
                ok &= bool(np.array_equal(out[i:i + 4096].cpu().numpy(), want))
        elif wl["kind"] == "sst_trailers":
            for i in idx:
                o, ln = int(offs_np[i]), int(lens_np[i])
                blk = buf[o:o + ln + 5].cpu().numpy().tobytes()
                ok &= orc.trailer(blk[:ln], 0, True) == blk[ln:]
        elif wl["kind"] == "sst_verify":
            ok = bool(out.cpu().numpy().all()) and int(bad.item()) == 0  # every block, every step
        else:
            got = out.cpu().numpy().view(np.uint32)
            for i in idx:
                if wl["kind"] == "strided":
                    o, ln = int(i) * L, L
                else:
                    o, ln = int(offs_np[i]), int(lens_np[i])
                blk = buf[o:o + ln].cpu().numpy().tobytes()
                ok &= orc.value(blk) == int(got[i])
        oks = ctx.all_gather_f64(1.0 if ok else 0.0)  # every rank learns whether any shard failed
        verified = bool(min(oks) > 0)

    if cfg == 2 and not ctx.on and not getattr(args, "no_read_ceiling", False):
        ceiling = read_ceiling(torch, C, buf, bytes_step, stream)
    achieved = bytes_step / avg_launch_s / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4)}
    roof.update(traffic_of(cfg, dispatch))
    if ceiling:
        roof["ceiling"] = ceiling
        roof["frac_of_ceiling"] = round(achieved / ceiling["achieved"], 4)
    roof.update({"kernel_ms_avg": round(avg_launch_s * 1e3, 4),
                 "kernel_ms_min": round(min(kernel_ms), 4),
                 "kernel_ms_median": round(sorted(kernel_ms)[len(kernel_ms) // 2], 4)})
    if ctx.on:
        roof["kernel_ms_avg_per_rank"] = [round(x, 4) for x in rank_kernel_ms]
    del buf, out
    torch.cuda.empty_cache()
    res_wl = {"workload": wl["workload"], "n_blocks": n, "bytes_per_gpu": bytes_step,
              "dispatch": dispatch}
    if wl["kind"] in ("sst_trailers", "sst_verify"):
        res_wl["algorithmic_bytes"] = ("sum(len) read + 5 B trailer written per block"
                                       if wl["kind"] == "sst_trailers"
                                       else "sum(len + 5) read + 1 B flag written per block")
    elif wl["kind"] == "log_write":
        res_wl["algorithmic_bytes"] = "sum(7 + len) per record: header length/type and payload read, CRC written"
    elif wl["kind"] == "log_verify":
        res_wl["algorithmic_bytes"] = "sum(7 + len) read + 1 B status written per record"
    elif wl["kind"] == "parity":
        res_wl["algorithmic_bytes"] = "8 fragments read + the parity written"
    return {
        "config": cfg,
        "value": round(ctx.world * bytes_step * args.steps / dt_max / 2**30, 2),
        "unit": "GiB/s",
        "ms_per_step": round(dt_max / args.steps * 1e3, 4),
        "workload": res_wl,
        "settle": {"settle_ms": round(settle_ms, 1), "settle_launches": settle_launches},
        "roofline": roof,
        "verified_sample": verified,
    }


KERNEL_SOURCES = ("crc32c_kernels.hpp", "crc32c_internal.hpp", "crc32c_device.hip")


def kernel_src_sha16() -> str:
    """Hash of the product kernels' sources: a PMC pass taken on other sources
    (even for a kernel of the same name) does not describe this run."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "novalsm_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def traffic_of(cfg, dispatch: dict) -> dict:
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    pass (tools/pmc.sh -> profiles/pmc_config<N>.json); PMC counters cannot be
    read from inside the timed run.  Used only when that pass profiled the
    kernel this run dispatches, built from the same kernel sources
    (src_sha16); otherwise traffic is null and traffic_source says why."""
    path = os.path.join("profiles", f"pmc_config{cfg}.json")
    try:
        with open(os.path.join(ROOT, path)) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return {"traffic": None, "traffic_source": f"no PMC pass ({path})"}
    k = pmc.get("kernel")
    if k and k != dispatch.get("kernel"):
        return {"traffic": None, "traffic_source": f"{path} profiled {k}, not this dispatch"}
    sha = kernel_src_sha16()
    if pmc.get("src_sha16") != sha:
        return {"traffic": None,
                "traffic_source": f"{path} was taken on kernel sources {pmc.get('src_sha16')}, "
                                  f"not this tree's {sha}"}
    src = f"{path} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, separate pass, kernel sources {sha}"
    if pmc.get("commit"):
        src += f", tree {pmc['commit']}"
    return {"traffic": pmc.get("hbm_bytes_per_launch"), "traffic_source": src + ")"}


def host_config_measure(args, ctx: Ctx, steps: int, warmup: int) -> dict:
    """Config 5: 4 GiB of pinned 16 KiB blocks streamed H2D -> CRC -> D2H
    (nova_crc32c_stream_host), its rate against the same-run pinned H2D copy
    ceiling, every block's CRC checked against the device-resident path."""
    import torch
    from novalsm_amd import crc32c as C
    wl = workload(5)
    hbm_preflight(5, wl, ctx)
    L, n = wl["block_bytes"], wl["n_blocks"]
    host = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    tmp = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    C.fill_splitmix64(tmp, 5, first_word=ctx.rank * (n * L // 8))
    host.copy_(tmp.cpu())
    want = C.batch_strided(tmp, L, L, n).cpu()
    ceiling = h2d_ceiling(torch, host, tmp, 4096 * L)
    del tmp
    torch.cuda.empty_cache()
    out = None
    for _ in range(max(1, warmup)):
        out = C.stream_host(host, L, L, n)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = C.stream_host(host, L, L, n)
    ctx.barrier()
    dt = max(ctx.all_gather_f64(time.perf_counter() - t0))
    verified = bool(np.array_equal(np.asarray(out).view(np.uint32), want.numpy().view(np.uint32)))
    gbs = n * L * steps / dt / 1e9
    return {"value": round(ctx.world * n * L * steps / dt / 2**30, 3), "unit": "GiB/s",
            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "workload": {"workload": wl["workload"], "n_blocks": n, "block_bytes": L,
                         "bytes_per_gpu": n * L, "op": "nova_crc32c_stream_host",
                         "chunk_blocks": 4096, "streams": 3},
            "roofline": {"bound": "pcie_h2d", "achieved": round(gbs, 2), "peak": ceiling["achieved"],
                         "unit": "GB/s", "frac": round(gbs / ceiling["achieved"], 4),
                         "ceiling": ceiling, "pcie_gen5_x16_spec_GBps": 63.0,
                         "traffic": None, "traffic_source": "host-link bound: no HBM PMC pass"},
            "verified_sample": verified}


def run_host_config(args, ctx: Ctx) -> int:
    r = host_config_measure(args, ctx, args.steps, args.warmup)
    value, dt = r["value"], r["ms_per_step"] * args.steps / 1e3
    wl = workload(5)
    L, n = wl["block_bytes"], wl["n_blocks"]
    if ctx.rank == 0:
        print(json.dumps({"metric": "GiB/s pinned-host streamed CRC32C (H2D->CRC->D2H), 16 KiB",
                          "value": round(value, 3), "unit": "GiB/s", "n_gpus": ctx.world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / args.steps * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "u8", "data": "synthetic (splitmix64)",
                          "config": {"workload": wl["workload"], "n_blocks": n,
                                     "block_bytes": L}, "roofline": r["roofline"],
                          "verified_sample": r["verified_sample"]}), flush=True)
    return 0 if r["verified_sample"] else 3


def compact_secondary(s: dict) -> dict:
    """A secondary's numbers without its descriptive objects: config, rate,
    roofline (achieved, frac, kernel time, PMC traffic / algorithmic bytes),
    ceiling fractions, the check."""
    if s.get("config") == ENGINE_WORKLOAD:
        keep = ("op", "threads", "GBps", "frac", "p50_us", "p99_us", "max_us", "launches", "fallbacks",
                "exits_yield", "verified")
        return {"config": s["config"], "value": s["value"], "unit": s["unit"],
                "lone_p50_us": s.get("lone", {}).get("p50_us"),
                "runs": [{k: x[k] for k in keep} for x in s["runs"]], "verified": s["verified_sample"]}
    r = s.get("roofline", {})
    out = {"config": s.get("config"), "value": s.get("value"), "unit": s.get("unit")}
    for k in ("bound", "achieved", "frac", "kernel_ms_avg", "frac_of_ceiling"):
        if k in r:
            out[k] = r[k]
    wl = s.get("workload", {})
    algo = wl.get("bytes_per_gpu")
    if r.get("traffic") and algo:
        out["traffic_over_algorithmic"] = round(r["traffic"] / algo, 3)
    if r.get("ceiling"):
        out["ceiling"] = r["ceiling"].get("achieved")
    disp = wl.get("dispatch") or {}
    if disp.get("kernel"):
        out["kernel"] = disp["kernel"]
    out["verified"] = s.get("verified_sample")
    return out


def harness_check(args, world: int, rank: int) -> int:
    """--harness-check: the launcher and collective plumbing on CPU (gloo), no
    GPU and no measurement.  Each rank checksums a small buffer with the
    product's host Extend and reports; rank 0 prints the world size gloo saw."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    from novalsm_amd import crc32c as C
    data = bytes(range(256)) * 16
    crc = C.Value(data)
    import torch
    t = torch.tensor([float(rank)], dtype=torch.float64)
    ranks = [rank]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        parts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0"))]))
        ranks = sorted(int(x[0]) for x in parts)
        local = sorted(int(x[1]) for x in parts)
    else:
        local = [0]
    if rank == 0:
        print(json.dumps({"harness_check": True, "n_gpus": world, "backend": "gloo",
                          "max_rank": int(t.item()), "ranks": ranks, "local_ranks": local,
                          "crc": f"0x{crc:08x}"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="2", choices=["2", "3", "4", "5", *SST_WORKLOADS, *OPS_WORKLOADS,
                                                      ENGINE_WORKLOAD])
    ap.add_argument("--secondary", default="auto",
                    help="configs measured after the primary one in the same run (comma list, "
                         "'none'; auto, when the primary is 2: 3, 4, the SSTable, log and parity "
                         "workloads, and 5 -- pinned host, one GPU only)")
    ap.add_argument("--settle-ms", type=float, default=400.0,
                    help="time-based settle of back-to-back launches before the warmup")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per unit override (tuning)")
    ap.add_argument("--seg", type=int, default=0, help="segment bytes override (tuning)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--verify", type=int, default=1, help="sample-verify vs the oracle")
    ap.add_argument("--harness-check", action="store_true",
                    help="CPU-only check of the rank launcher (gloo), no measurement")
    ap.add_argument("--engine-secs", type=float, default=1.0, help="sst_engine window per point")
    ap.add_argument("--detail-out", default="",
                    help="also write the full result (every secondary's workload, dispatch, "
                         "ceilings) to this JSON file; stdout carries the compact line")
    args = ap.parse_args()
    args.config = int(args.config) if args.config.isdigit() else args.config

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.harness_check:
        return harness_check(args, world, rank)

    import torch
    import torch.distributed as dist
    from novalsm_amd import crc32c as C

    # under torch.distributed.run (WORLD_SIZE set, any world size): one rank
    # per GPU, RCCL for the barriers and the max-over-ranks time
    dist_on = "WORLD_SIZE" in os.environ
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()  # the world RCCL reports
        rank = dist.get_rank()
    dev = torch.device("cuda", local if dist_on else 0)
    torch.cuda.set_device(dev)
    C.load()
    if args.lanes or args.seg:
        C.set_tuning(args.lanes, args.seg)
    if C.load().nova_device_init() != 0:
        raise SystemExit("nova_device_init failed")
    ctx = Ctx(world, rank, dev, dist, dist_on)

    if args.config == ENGINE_WORKLOAD:
        r = engine_measure(args, ctx)
        if rank == 0:
            print(json.dumps(r, separators=(",", ":")), flush=True)
        if dist_on:
            dist.barrier()
            dist.destroy_process_group()
        return 0 if r["verified_sample"] else 3

    if args.config == 5:
        rc = run_host_config(args, ctx)
        if dist_on:
            dist.barrier()
            dist.destroy_process_group()
        return rc

    prim = run_device_config(args.config, args, ctx)
    if args.secondary == "auto":
        sec_cfgs = [3, 4, *SST_WORKLOADS, *OPS_WORKLOADS, 5, ENGINE_WORKLOAD] if args.config == 2 else []
    elif args.secondary in ("", "none"):
        sec_cfgs = []
    else:
        sec_cfgs = [int(x) if x.isdigit() else x for x in args.secondary.split(",")]
        sec_cfgs = [c for c in sec_cfgs if c != args.config]
    secondary = []
    for c in sec_cfgs:
        if c == 5:
            # the host link is per GPU and 4 GiB of pinned memory per rank is
            # the node's, not the GPU's: measured at N = 1 only
            if world == 1:
                r = host_config_measure(args, ctx, max(3, args.steps // 20), max(1, args.warmup // 20))
                secondary.append({"metric": "GiB/s pinned-host streamed CRC32C (H2D->CRC->D2H), 16 KiB; "
                                            "% of the same-run H2D copy ceiling", "config": 5, **r})
            continue
        if c == ENGINE_WORKLOAD:
            # many host threads of ONE process on one GPU: measured at N = 1 only
            if world == 1:
                secondary.append(engine_measure(args, ctx))
            continue
        r = run_device_config(c, args, ctx)
        secondary.append({"metric": METRIC, **r})

    rc = 0
    if prim["verified_sample"] is False or any(s["verified_sample"] is False for s in secondary):
        rc = 3
        if rank == 0:
            print(json.dumps({"error": "GPU CRC mismatch vs oracle"}), file=sys.stderr)
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": prim["value"],
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": prim["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 generated on device)",
            "config": {**prim["workload"],
                       "parallelism": f"shard{world}" if world > 1 else "single"},
            "settle": prim["settle"],
            "roofline": prim["roofline"],
            "verified_sample": prim["verified_sample"],
            "secondary": secondary,
        }
        if not args.no_cpu_baseline and world == 1:
            # rank 0 at N=1 only: the CPU sample is the same at every N
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if args.detail_out:
            with open(args.detail_out, "w") as f:
                json.dump(res, f, indent=1)
        # the driver keeps the last ~8 KB of stdout: one compact line that holds
        # every secondary's rate, roofline and check (the full objects: --detail-out)
        res["secondary"] = [compact_secondary(x) for x in secondary]
        print(json.dumps(res, separators=(",", ":")), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
