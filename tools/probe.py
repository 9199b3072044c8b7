#!/usr/bin/env python3
"""Run one workload/variant N times (for rocprofv3 --pmc passes).

    python tools/probe.py <workload> <variant> [iters]
workload: cfg2 | cfg3 | sst4k | log (tools/sweep_flat.py); variant as there."""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main() -> int:
    import torch
    from novalsm_amd import crc32c as C
    from sweep_flat import make_workload, set_variant
    wl, var = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    assert C.load().nova_device_init() == 0
    fn, _, keep = make_workload(wl, torch.cuda.current_stream())
    set_variant(C, var)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    del keep
    return 0


if __name__ == "__main__":
    sys.exit(main())
