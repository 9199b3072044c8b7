#!/usr/bin/env python3
"""Engine throughput lost to yields.

8 native threads call nova_sst_queue_verify_blocks on their own 4096-block
tables while a 9th thread makes plain calls (SSTable verify, log verify, CRC
batch; every result checked against expectations taken from the oracle) with
a pause of --gaps microseconds between calls.  Each plain call makes the
resident engine yield (exit, relaunch behind it); the rows show what that
costs the engine callers and what the plain calls wait.

  python tools/mixed_callers.py [--gaps 0,200,1000,5000] [--op verify]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", default="0,200,1000,5000")
    ap.add_argument("--op", default="verify")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=1.0)
    args = ap.parse_args()
    import torch
    from novalsm_amd import callers
    from novalsm_amd import crc32c as C
    from tests.oracle_lib import load_oracle
    from tests.test_gpu_engine import _plain_inputs
    C.load()
    assert C.load().nova_device_init() == 0
    plain, keep = _plain_inputs(torch, load_oracle())
    for g in [float(x) for x in args.gaps.split(",")]:
        plain.gap_us = g
        r = callers.run(args.op, args.threads, 4096, args.seconds, "engine", warm_s=0.3, seed=5, plain=plain)
        e = r["engine"]
        print(json.dumps({"plain_gap_us": g, "engine_GBps": r["aggregate_GBps"], "p50_us": r["p50_us"],
                          "p99_us": r["p99_us"], "max_us": r["max_us"], "launches": e["launches"],
                          "exits_yield": e["exits_yield"], "fallbacks": e["fallbacks"],
                          "plain": r["plain"], "verified": r["verified"]}), flush=True)
    del keep
    return 0


if __name__ == "__main__":
    sys.exit(main())
