#!/usr/bin/env python3
"""Concurrent per-SSTable callers.

Drives tools/bin/concurrent_sst (tools/concurrent_sst.cpp: native threads, one
HIP stream and one device-resident SSTable image per thread, synchronous
nova_sstable_verify_blocks / nova_sstable_write_trailers calls) over a matrix
of thread counts and table sizes, one child process per point, and prints its
JSON lines.  --paths direct,engine,queue: each caller launching on its own
stream, or every call through nova_sst_queue_* on the persistent engine
 or on the round-3 coalescing queue.  --hwq runs each point with GPU_MAX_HW_QUEUES set (the HIP
runtime's hardware queues per process; 4 is the default on the box).

  python tools/concurrent_sst.py --build            # here, on the CPU
  python tools/concurrent_sst.py --threads 1,8,16   # on the GPU box
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "bin", "concurrent_sst")
SRC = os.path.join(ROOT, "tools", "concurrent_sst.cpp")


def build() -> None:
    sys.path.insert(0, ROOT)
    from novalsm_amd import build as nb
    nb.build()
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run([nb.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-I", os.path.join(ROOT, "include"), "-o", BIN, SRC,
                    "-L", nb.LIB_DIR, "-lnova_crc32c",
                    "-Wl,-rpath,$ORIGIN/../../novalsm_amd/lib", "-lpthread"], check=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--ops", default="verify,trailers")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--blocks", default="1024,4096", help="blocks per table (4 KiB blocks)")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--paths", default="direct,engine",
                    help="direct: nova_sstable_* on each caller's stream; engine / queue: "
                         "nova_sst_queue_* on the persistent engine / the coalescing queue")
    ap.add_argument("--hwq", default="", help="comma list of GPU_MAX_HW_QUEUES values (<= 32)")
    args = ap.parse_args()
    if args.build:
        build()
        return 0
    if not os.path.exists(BIN):
        print("tools/bin/concurrent_sst is not built (python tools/concurrent_sst.py --build)")
        return 2
    hwqs = [int(x) for x in args.hwq.split(",")] if args.hwq else [None]
    for hwq in hwqs:
        env = dict(os.environ)
        if hwq is not None:
            assert 1 <= hwq <= 32
            env["GPU_MAX_HW_QUEUES"] = str(hwq)
        for op in args.ops.split(","):
            for n in [int(x) for x in args.blocks.split(",")]:
                for t, path in [(int(x), p) for p in args.paths.split(",") for x in args.threads.split(",")]:
                    r = subprocess.run([BIN, op, str(t), str(n), str(args.seconds), path], env=env,
                                       capture_output=True, text=True, timeout=120)
                    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                    if r.returncode != 0 or not line:
                        print(r.stdout, r.stderr, file=sys.stderr)
                        return r.returncode or 1
                    row = json.loads(line[-1])
                    for extra in line[:-1]:  # engine_trace: the spans
                        row.update(json.loads(extra))
                    row["hw_queues"] = hwq if hwq is not None else env.get("GPU_MAX_HW_QUEUES", "default")
                    print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
