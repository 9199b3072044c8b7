#!/usr/bin/env python3
"""Debug helper: repeat the flat-kernel many-blocks case and report every
mismatching block (index, offset, length, chunk position) per run."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_bytes
    from tests.oracle_lib import load_oracle
    lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    kernel = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    sort = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    orc = load_oracle()
    L = C.enable_diagnostics()
    assert L.nova_device_init() == 0
    C.set_tuning(lanes, 0)
    L.nova_diag_set_chunk_blocks(chunk)
    L.nova_diag_set_variable_kernel(kernel)
    L.nova_diag_set_rounds_sort(sort)
    print(C.describe(1, 0, 0, variable=True), flush=True)
    rng = np.random.default_rng(1000 + lanes * 7 + chunk)
    n = 120000
    lens = rng.choice([0, 1, 2, 3, 4, 5, 17, 100, 600, 1500, 4096, 9000], n,
                      p=[.02, .02, .02, .02, .02, .05, .1, .25, .2, .1, .15, .05]).astype(np.uint32)
    lens += (rng.integers(0, 64, n) * (lens > 5)).astype(np.uint32)
    pos = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 9, n).astype(np.uint64))
    offs = (pos - lens.astype(np.uint64)).astype(np.uint64)
    perm = rng.permutation(n)
    offs, lens = offs[perm], lens[perm]
    host = splitmix64_bytes(lanes + 3, int(pos[-1]) + 64)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    buf = torch.from_numpy(host).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    di = torch.from_numpy(init.view(np.int32)).cuda()
    want = orc.batch(host, offs, lens, init)
    want0 = orc.batch(host, offs, lens, None)
    for r in range(reps):
        out = torch.full((n,), -559038737, dtype=torch.int32, device="cuda")
        C.batch(buf, do, dl, init=di, out=out)
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        print(f"run {r}: {bad.size} bad, {int((got[bad] == 0xDEADBEEF).sum())} unwritten", flush=True)
        for i in bad[:10]:
            # does the wrong value equal the CRC of some other descriptor?
            hits = np.nonzero(want == got[i])[0][:3].tolist()
            print(f"  i={i} off={int(offs[i])} (mod16={int(offs[i]) % 16}) len={int(lens[i])} "
                  f"init={int(init[i]):#x} got={int(got[i]):#x} want={int(want[i]):#x} "
                  f"noinit={int(want0[i]):#x} same_as={hits}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
