#!/usr/bin/env python3
"""Does work on other streams wait behind the resident engine?  

HIP maps streams onto GPU_MAX_HW_QUEUES shared hardware queues whose packets
run in order; a persistent kernel on one of them blocks every stream mapped to
the same queue until it exits.  For each engine queue mode
(NOVA_SST_ENGINE_QUEUE 0/1/2, optionally NOVA_SST_ENGINE_SLICE_US), a child
process keeps the engine busy with two native caller threads for 2 s while
the main thread runs a small torch op on each of 16 fresh streams and on the
null stream, timing each; a latency near the window means that stream waited
for the engine.

  python tools/queue_probe.py [--modes 0,1,2,0:1000]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, threading, time
sys.path.insert(0, %r)
import torch
from novalsm_amd import crc32c as C, callers
C.load(); assert C.load().nova_device_init() == 0
res = {}
def bg():
    res["bg"] = callers.run("verify", 2, 4096, 2.0, "engine", warm_s=0.2)
t = threading.Thread(target=bg); t.start()
time.sleep(0.6)
x = torch.empty(1 << 20, device="cuda")
lat = []
for k in range(16):
    s = torch.cuda.Stream()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        x.zero_()
    s.synchronize()
    lat.append(round((time.perf_counter() - t0) * 1e3, 3))
t0 = time.perf_counter()
v = float(x.sum().item())
null_ms = round((time.perf_counter() - t0) * 1e3, 3)
t.join()
bg = res["bg"]
print(json.dumps({"stream_ms": lat, "null_stream_ms": null_ms, "engine_GBps": bg["aggregate_GBps"],
                  "p50_us": bg["p50_us"], "max_us": bg["max_us"], "verified": bg["verified"],
                  "engine": bg["engine"]}), flush=True)
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1,2,0:1000")
    args = ap.parse_args()
    for m in args.modes.split(","):
        q, _, sl = m.partition(":")
        env = dict(os.environ, NOVA_SST_ENGINE_QUEUE=q, NOVA_SST_ENGINE_SLICE_US=sl or "0")
        r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True,
                           timeout=120)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode or not line:
            print(json.dumps({"mode": m, "rc": r.returncode, "err": r.stderr[-1500:]}), flush=True)
            continue
        row = json.loads(line[-1])
        row["mode"] = {"queue": int(q), "slice_us": int(sl or 0)}
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
