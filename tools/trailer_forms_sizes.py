#!/usr/bin/env python3
"""Trailer writer by batch size: the product's two-pass form (CRC pass, then
whole-piece rewrite) against the one-pass form (trailer bytes
stored by the CRC kernel; diagnostics knob nova_diag_set_trailer_single_pass(9))
on sst4k images of 4K-1M blocks, stream-synchronous calls timed by HIP events
(the launch path included, as a caller waiting for one table sees it).

    python tools/trailer_forms_sizes.py --sizes 4096,16384,65536,262144,1048576
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
    ap.add_argument("--sizes", default="4096,16384,65536,262144,1048576")
    ap.add_argument("--reps", type=int, default=40)
    args = ap.parse_args()
    import numpy as np
    import torch
    from novalsm_amd import crc32c as C
    from bench import sst4k_layout
    assert C.load().nova_device_init() == 0
    stream = torch.cuda.current_stream()
    for n in [int(x) for x in args.sizes.split(",")]:
        offs_np, lens_np, total = sst4k_layout(n, 5)
        img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        C.fill_splitmix64(img, 9)
        offs = torch.from_numpy(offs_np.view(np.int64)).cuda()
        lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
        algo = int(lens_np.astype(np.uint64).sum()) + 5 * n
        row = {"blocks": n, "bytes": algo}
        ref = None
        for name, knob in (("two_pass", 0), ("one_pass", 9)):
            with C.diagnostics() as D:
                D.nova_diag_set_trailer_single_pass(knob)
                for _ in range(5):
                    C.write_trailers(img, offs, lens, 0, True, stream=stream)
                torch.cuda.synchronize()
                ms = []
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    C.write_trailers(img, offs, lens, 0, True, stream=stream)
                    b.record(stream)
                    b.synchronize()
                    ms.append(a.elapsed_time(b))
                D.nova_diag_set_trailer_single_pass(0)
            ms.sort()
            med = ms[len(ms) // 2]
            row[name + "_us"] = round(med * 1e3, 1)
            row[name + "_frac"] = round(algo / (med / 1e3) / 8e12, 4)
            img_h = img.cpu().numpy()
            ref = img_h if ref is None else ref
            row[name + "_same_image"] = bool(np.array_equal(img_h, ref))
        print(json.dumps(row), flush=True)
        del img, offs, lens
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
