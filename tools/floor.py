#!/usr/bin/env python3
"""Fixed per-launch cost: HIP-event time of one-block and tiny launches of each
entry point next to a trivial torch kernel."""
import sys, statistics, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np, torch
from novalsm_amd import crc32c as C
assert C.load().nova_device_init() == 0
s = torch.cuda.current_stream()
x = torch.zeros(16, device="cuda")
buf = torch.zeros(1 << 24, dtype=torch.uint8, device="cuda")
C.fill_splitmix64(buf, 1)
def ev(fn, R=200):
    out = []
    for i in range(R + 20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); fn(); b.record(s); b.synchronize()
        if i >= 20: out.append(a.elapsed_time(b) * 1e3)
    return round(statistics.median(out), 1)
o1 = torch.zeros(1, dtype=torch.int64, device="cuda"); l1 = torch.full((1,), 16, dtype=torch.int32, device="cuda")
res = {"torch_add": ev(lambda: x.add_(1)),
       "empty_events": ev(lambda: None),
       "strided_1x16B": ev(lambda: C.batch_strided(buf, 16, 16, 1)),
       "strided_1x4KiB": ev(lambda: C.batch_strided(buf, 4096, 4096, 1)),
       "strided_16x4KiB": ev(lambda: C.batch_strided(buf, 4096, 4096, 16)),
       "batch_1x16B": ev(lambda: C.batch(buf, o1, l1)),
       "verify_1x16B": ev(lambda: C.verify_blocks(buf, o1, l1)),
}
for G in (8, 16):
    C.set_tuning(G, 0)
    res[f"batch_1x16B_G{G}"] = ev(lambda: C.batch(buf, o1, l1))
C.set_tuning(0, 0)
print(res)
