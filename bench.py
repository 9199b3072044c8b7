#!/usr/bin/env python3
"""Device-resident batched CRC32C throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

One step = one pass of the hot path (a nova_crc32c_batch* call through the
C-ABI) over one batch of synthetic SSTable blocks already resident in HBM.
Default workload at every N: BASELINE config 2 per rank (1M x 4 KiB uniform
blocks = 4 GiB per GPU, splitmix64 data generated on the device), weak scaling:
rank r checksums its own shard, no data-path collective; RCCL only for the
barrier and the max-over-ranks time.  --config 3: 1M mixed {4,16,64} KiB +
U[1,64] B unaligned blocks (variable-length kernel).  --config 4: 1M x 16 KiB
per rank (8M x 16 KiB over 8 GPUs).  --config 5: host-resident (pinned) 16 KiB
blocks streamed H2D -> CRC -> D2H; reported separately, never as
the device-resident value.

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes per
launch (sum of block lengths) / average launch time measured
with HIP events on the launch stream inside the timed region.
Defaults W=50, K=200: back-to-back launches show a power-management transient
(launches ~4-25 run up to 30% slower, then settle; tools/launches.py), so
the timed steps start after it.
`cpu_baseline` = the reference util/crc32c.cc (oracle/_ref, compiled from the
reference sources) or the oracle restatement, timed on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
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


def workload(cfg: int):
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


def cpu_baseline(threads: int, seconds: float = 4.0):
    """Reference util/crc32c.cc (oracle/_ref) if built, else the oracle restatement,
    on BASELINE config 1: 1024 x 4 KiB splitmix64(seed 1) blocks, repeated."""
    import ctypes
    from novalsm_amd.synth import splitmix64_bytes
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    n, L = 1024, 4096
    buf = splitmix64_bytes(1, n * L)
    out = np.empty(n, dtype=np.uint32)
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        fn = lib.ref_batch_strided_mt
        kind = "reference"
    else:
        from tests.oracle_lib import load_oracle
        lib = load_oracle().lib
        fn = lib.oracle_batch_strided_mt
        kind = "port"
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int]

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

    one, r1 = rate(1)
    allc, r2 = rate(threads)
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
            "single_core": round(one, 3), "cpu": model,
            "sample": f"BASELINE config 1: 1024 x 4 KiB splitmix64(seed 1) blocks, "
                      f"{r2} reps on {threads} threads (+{r1} reps on 1 thread), g++ -O2"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--lanes", type=int, default=0, help="lanes per unit override (tuning)")
    ap.add_argument("--seg", type=int, default=0, help="segment bytes override (tuning)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--verify", type=int, default=1, help="sample-verify vs the oracle")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from novalsm_amd import crc32c as C

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    C.load()
    if args.lanes or args.seg:
        C.set_tuning(args.lanes, args.seg)
    if C.load().nova_device_init() != 0:
        raise SystemExit("nova_device_init failed")

    wl = workload(args.config)
    stream = torch.cuda.current_stream()
    n = wl["n_blocks"]
    seed = args.config

    if wl["kind"] == "host":
        L = wl["block_bytes"]
        host = torch.empty(n * L, dtype=torch.uint8).pin_memory()
        tmp = torch.empty(n * L, dtype=torch.uint8, device=dev)
        C.fill_splitmix64(tmp, seed, first_word=rank * (n * L // 8))
        host.copy_(tmp.cpu())
        del tmp
        for _ in range(max(1, args.warmup)):
            C.stream_host(host, L, L, n)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = C.stream_host(host, L, L, n)
        dt = time.perf_counter() - t0
        bytes_step = n * L
        value = bytes_step * args.steps / dt / 2**30
        if rank == 0:
            print(json.dumps({"metric": "GiB/s pinned-host streamed CRC32C (H2D->CRC->D2H), 16 KiB",
                              "value": round(value, 3), "unit": "GiB/s", "n_gpus": 1,
                              "steps": args.steps, "warmup": args.warmup,
                              "ms_per_step": round(dt / args.steps * 1e3, 3),
                              "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                              "dtype": "u8", "data": "synthetic (splitmix64)",
                              "config": {"workload": wl["workload"], "n_blocks": n,
                                         "block_bytes": L}}))
        return 0

    # ---- device-resident batch -------------------------------------------
    if wl["kind"] == "strided":
        L = wl["block_bytes"]
        total = n * L
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        C.fill_splitmix64(buf, seed, first_word=rank * (total // 8))
        out = torch.empty(n, dtype=torch.int32, device=dev)

        def step():
            C.batch_strided(buf, L, L, n, out=out, stream=stream)
        lens_np = None
        offs_np = None
        bytes_step = total
    else:
        offs_np, lens_np, total = config3_layout(n, seed)
        buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        C.fill_splitmix64(buf, seed, first_word=rank * (total // 8))
        offs = torch.from_numpy(offs_np.view(np.int64)).to(dev)
        lens = torch.from_numpy(lens_np.view(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)

        # config 3 is LevelDB's block_size sweep (mean ~28 KiB): the caller
        # knows its block_size and passes the scheduling hint (results are
        # identical without it; include/nova_crc32c.h)
        hint = C.HINT_LARGE_BLOCKS

        def step():
            C.batch(buf, offs, lens, flags=hint, out=out, stream=stream)
        bytes_step = int(lens_np.astype(np.uint64).sum())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3

    # ---- sample verification against the CPU oracle (outside the timed region)
    verified = None
    if args.verify:
        from tests.oracle_lib import load_oracle
        orc = load_oracle()
        got = out.cpu().numpy().view(np.uint32)
        idx = np.linspace(0, n - 1, 257).astype(np.int64)
        ok = True
        for i in idx:
            if wl["kind"] == "strided":
                o, l = int(i) * L, L
            else:
                o, l = int(offs_np[i]), int(lens_np[i])
            blk = buf[o:o + l].cpu().numpy().tobytes()
            ok &= orc.value(blk) == int(got[i])
        if world > 1:  # every rank learns whether any shard failed (no rank left in a barrier)
            f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item())
        verified = bool(ok)
        if not ok:
            print(json.dumps({"error": "GPU CRC mismatch vs oracle", "rank": rank}), file=sys.stderr)
            if world > 1:
                dist.destroy_process_group()
            return 3

    value = world * bytes_step * args.steps / dt / 2**30
    achieved = bytes_step / avg_launch_s / 1e9
    if wl["kind"] == "strided":
        dispatch = C.describe(n, L, L, variable=False)
    else:
        dispatch = C.describe(n, 0, 0, variable=True, large=True)
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 generated on device)",
            "config": {"workload": wl["workload"], "n_blocks": n, "bytes_per_gpu": bytes_step,
                       "parallelism": f"shard{world}" if world > 1 else "single",
                       "dispatch": dispatch},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel_ms_avg": round(avg_launch_s * 1e3, 4),
                         "kernel_ms_min": round(min(kernel_ms), 4),
                         "kernel_ms_median": round(sorted(kernel_ms)[len(kernel_ms) // 2], 4)},
            "verified_sample": verified,
        }
        if not args.no_cpu_baseline and world == 1:
            # rank 0 at N=1 only: the CPU sample is the same at every N
            th = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            res["cpu_baseline"] = cpu_baseline(th, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
