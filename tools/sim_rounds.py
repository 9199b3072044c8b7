#!/usr/bin/env python3
"""Offline replay of the rounds kernel's schedule (no GPU): for a batch layout,
count the steps the waves execute and the rounds they run under a given lane
group width G, swaths per step, sort window and round width, and report the
useful fraction of the loaded step capacity (CRC input bytes / bytes of steps
executed by all groups); replay_continuous models round 3's continuous rounds
(rounds of a chunk back to back, swath by swath).  Used to pick the log-record schedule.

  python tools/sim_rounds.py --workload log --records 200000
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def layout(workload: str, n: int):
    from novalsm_amd.synth import splitmix64_words, log_layout
    if workload == "log":
        r = splitmix64_words(6, 0, n)
        plens = ((r % np.uint64(4096)) + np.uint64(1)).astype(np.int64)
        offs, lens, _, _, _ = log_layout(plens)
        u0 = offs.astype(np.int64) + 6
        u1 = u0 + 1 + lens.astype(np.int64)
    else:  # sst4k: 4096+U[0,255] B blocks, 5-B trailers; verify covers n+1
        r = splitmix64_words(5, 0, n)
        lens = (4096 + (r % np.uint64(256))).astype(np.int64)
        offs = np.zeros(n, np.int64)
        offs[1:] = np.cumsum(lens[:-1] + 5)
        u0 = offs
        u1 = offs + lens + 1
    return u0, u1


def steps_of(u0, u1, G, sw):
    """Steps per record on the group's line grid: lines (16G B) from the one
    holding u0 & ~15 to the one holding E-1 (E = u1 & ~15), in steps of sw."""
    line = 16 * G
    E = u1 & ~15
    first = (u0 & ~15) // line
    last = (E + line - 1) // line
    lines = np.maximum(last - first, 1)
    return (lines + sw - 1) // sw


def replay(u0, u1, G, sw, window, chunk=None):
    n = len(u0)
    S = steps_of(u0, u1, G, sw)
    groups = 64 // G
    steps = 0
    rounds = 0
    for c0 in range(0, n, window):
        s = np.sort(S[c0:c0 + window])[::-1]
        pad = (-len(s)) % groups
        s = np.concatenate([s, np.zeros(pad, s.dtype)]).reshape(-1, groups)
        m = s.max(axis=1)
        steps += int(m.sum())
        rounds += int((m > 0).sum())
    useful = int((u1 - u0).sum())
    cap = steps * groups * sw * 16 * G
    return {"G": G, "swaths_per_step": sw, "window": window, "wave_steps": steps,
            "rounds": rounds, "useful_frac": round(useful / cap, 4),
            "bytes_per_round": round(useful / max(rounds, 1), 1),
            "steps_per_round": round(steps / max(rounds, 1), 2)}


def replay_continuous(u0, u1, G, window, chunk):
    """Continuous rounds (round 3): a round runs max(m, 4) lines (m = its
    longest region in lines); rounds of one chunk follow each other swath by
    swath, a chunk's last round pads its step to the 4-swath boundary."""
    S = steps_of(u0, u1, G, 1)
    groups = 64 // G
    swaths = 0
    for c0 in range(0, len(u0), window):
        s = np.sort(S[c0:c0 + window])[::-1]
        for k0 in range(0, len(s), chunk):
            c = s[k0:k0 + chunk]
            pad = (-len(c)) % groups
            c = np.concatenate([c, np.zeros(pad, c.dtype)]).reshape(-1, groups)
            m = c.max(axis=1)
            m = m[m > 0]
            lines = int(np.maximum(m, 4).sum())
            swaths += (lines + 3) // 4 * 4
    useful = int((u1 - u0).sum())
    return {"G": G, "continuous": True, "window": window, "chunk": chunk,
            "useful_frac": round(useful / (swaths * groups * 16 * G), 4)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="log")
    ap.add_argument("--records", type=int, default=200000)
    args = ap.parse_args()
    u0, u1 = layout(args.workload, args.records)
    for G, sw in ((8, 4), (8, 2), (16, 2), (16, 4), (4, 4)):
        for window in (64, 128, 256, 512, 4096):
            print(replay(u0, u1, G, sw, window))
    chunk = 64 if args.workload == "log" else 32
    for window in (chunk, 512):
        print(replay_continuous(u0, u1, 8, window, chunk))
    return 0


if __name__ == "__main__":
    sys.exit(main())
