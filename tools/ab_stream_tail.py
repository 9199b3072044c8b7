#!/usr/bin/env python3
"""Same-box A/B of the stream kernel's tail rounds (diagnostics knob
nova_diag_set_stream_tail): config 2 (1M x 4 KiB) and config 4's shard
(1M x 16 KiB), after a 400 ms settle, alternating settings over several
rounds of 50 timed launches (HIP events on the launch stream); prints the
median kernel time and % of the 8 TB/s HBM peak per setting."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch
    from novalsm_amd import crc32c as C
    stream = torch.cuda.current_stream()
    settings = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "-1,0,1,4").split(",")]
    for L in (4096, 16384):
        n = 1 << 20
        buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(buf, 2)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        ref = C.batch_strided(buf, L, L, n).clone()
        res = {k: [] for k in settings}
        with C.diagnostics() as D:
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.4:
                C.batch_strided(buf, L, L, n, out=out, stream=stream)
                torch.cuda.synchronize()
            for _ in range(4):
                for k in settings:
                    D.nova_diag_set_stream_tail(k)
                    for _ in range(5):
                        C.batch_strided(buf, L, L, n, out=out, stream=stream)
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(50)]
                    for a, b in ev:
                        a.record(stream)
                        C.batch_strided(buf, L, L, n, out=out, stream=stream)
                        b.record(stream)
                    torch.cuda.synchronize()
                    res[k] += [a.elapsed_time(b) for a, b in ev]
                    assert torch.equal(out, ref), k
            D.nova_diag_set_stream_tail(0)
        for k in settings:
            ms = statistics.median(res[k])
            print(json.dumps({"block_bytes": L, "tail_rounds": k, "ms_median": round(ms, 4),
                              "frac": round(n * L / (ms * 1e-3) / 8e12, 4)}), flush=True)
        del buf
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
