#!/usr/bin/env python3
"""Per-launch durations of back-to-back config-2 launches (HIP events), three
trials separated by 0.5 s idle.  Shows the power-management transient that
sets bench.py's default warmup: launches ~4-25 of a burst run up to 30%
slower before settling (profiles/r01_launch_transient.log)."""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--block", type=int, default=4096)
    args = ap.parse_args()
    import torch
    from novalsm_amd import crc32c as C
    assert C.load().nova_device_init() == 0
    n, L = (4 << 30) // args.block, args.block
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    C.fill_splitmix64(buf, 2)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for trial in range(args.trials):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.launches)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            C.batch_strided(buf, L, L, n, out=out)
            b.record()
        torch.cuda.synchronize()
        us = [a.elapsed_time(b) * 1e3 for a, b in ev]
        print(f"trial {trial} us:", " ".join(f"{u:.0f}" for u in us), flush=True)
        time.sleep(0.5)


if __name__ == "__main__":
    main()
