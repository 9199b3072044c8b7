#!/usr/bin/env python3
"""Concurrent per-SSTable callers.

Runs the native caller harness (novalsm_amd/callers.py ->
libnova_sst_callers.so: T native threads, one HIP stream and one
device-resident SSTable image of 4096+U[0,255] B blocks per thread, each call
waited on) over a matrix of thread counts and table sizes, one child process
per point, and prints its JSON lines.  --paths direct,engine,queue: each
caller launching on its own stream, or every call through nova_sst_queue_* on
the persistent engine or the round-3 coalescing queue.  --plain-gap-us adds a
thread of plain calls (verify, log verify, batch) beside the callers.
--hwq runs each point with GPU_MAX_HW_QUEUES set (<= 32).

  python tools/concurrent_sst.py --threads 1,8,16   # on the GPU box
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, %r)
from novalsm_amd import callers
print(json.dumps(callers.run(%r, %d, %d, %f, %r, warm_s=%f)), flush=True)
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="verify,trailers")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--blocks", default="1024,4096", help="blocks per table (4 KiB blocks)")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--warm", type=float, default=0.3)
    ap.add_argument("--paths", default="direct,engine")
    ap.add_argument("--hwq", default="", help="comma list of GPU_MAX_HW_QUEUES values (<= 32)")
    args = ap.parse_args()
    hwqs = [int(x) for x in args.hwq.split(",")] if args.hwq else [None]
    for hwq in hwqs:
        env = dict(os.environ)
        if hwq is not None:
            assert 1 <= hwq <= 32
            env["GPU_MAX_HW_QUEUES"] = str(hwq)
        for op in args.ops.split(","):
            for n in [int(x) for x in args.blocks.split(",")]:
                for t, path in [(int(x), p) for p in args.paths.split(",") for x in args.threads.split(",")]:
                    code = CHILD % (ROOT, op, t, n, args.seconds, path, args.warm)
                    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                       timeout=180)
                    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                    if r.returncode != 0 or not line:
                        print(r.stdout, r.stderr, file=sys.stderr)
                        return r.returncode or 1
                    row = json.loads(line[-1])
                    row["hw_queues"] = hwq if hwq is not None else env.get("GPU_MAX_HW_QUEUES", "default")
                    print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
