#!/usr/bin/env python3
"""Per-wave timeline of the streaming kernel (diagnostic build path, variant 4):
where does a launch lose time -- late starts, early finishers, per-XCD skew?"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from novalsm_amd import crc32c as C
    L = C.enable_diagnostics()
    L.nova_diag_set_variant.argtypes = [ctypes.c_int]
    L.nova_diag_set_stamps.argtypes = [ctypes.c_void_p]
    L.nova_diag_set_static_pct.argtypes = [ctypes.c_int]
    assert L.nova_device_init() == 0
    res = {}
    for Lb, g, var, pct in [(4096, 8, 4, 0), (4096, 8, 4, 8), (4096, 8, 12, 0),
                            (16384, 16, 4, 0), (16384, 16, 12, 0)]:
        L.nova_diag_set_static_pct(pct)
        n = 1 << 20
        buf = torch.empty(n * Lb, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 2)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(3 * 256 * 16, dtype=torch.int64, device="cuda")
        L.nova_diag_set_stamps(st.data_ptr())
        C.set_tuning(g, 0)
        L.nova_diag_set_variant(var)
        for _ in range(3):
            C.batch_strided(buf, Lb, Lb, n, out=out)
        torch.cuda.synchronize()
        a = st.cpu().numpy().reshape(-1, 3)
        a = a[a[:, 0] != 0]  # rows of the waves the launch had (8 or 16 per workgroup)
        L.nova_diag_set_variant(0)
        C.set_tuning(0, 0)
        t0 = a[:, 0].min()
        b = (a[:, 0] - t0) / 100.0  # us
        e = (a[:, 1] - t0) / 100.0
        span = e.max()
        r = {
            "block_bytes": Lb, "lanes": g, "var": var, "steal_limit": pct, "span_us": float(span),
            "begin_us_pct": [float(x) for x in np.percentile(b, [0, 50, 90, 99, 100])],
            "end_us_pct": [float(x) for x in np.percentile(e, [0, 1, 10, 50, 90, 100])],
            "busy_frac": float(((e - b).sum()) / (len(e) * span)),
            "per_xcd_end_mean": [float(e[a[:, 2] == x].mean()) for x in range(8)],
            "per_xcd_waves": [int((a[:, 2] == x).sum()) for x in range(8)],
            "GBps_if_span": n * Lb / span / 1e3,
        }
        print(json.dumps(r), flush=True)
        res[f"{Lb}_{g}_{pct}"] = r
        assert torch.equal(out, C.batch_strided(buf, Lb, Lb, n)), "stamp build changed results"
        del buf
        torch.cuda.empty_cache()
    with open(os.path.join(ROOT, "gpurun_out", "stamps.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
