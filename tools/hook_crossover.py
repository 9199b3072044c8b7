#!/usr/bin/env python3
"""Where the port hook should hand Extend() to the GPU (NOVA_HOOK_MIN_BYTES).

nova_port_accelerated_crc32c (port::AcceleratedCRC32C, port/port_stdcxx.h:
179-189) gets every Extend() once NovaLSM adopts it (util/crc32c.cc:487-491).
For a buffer in pageable host memory it either runs the host Extend
(crc32c_host.cpp) or copies the buffer to the GPU, checksums it there and
folds the sub-block CRCs on the host.  This tool times both on the same
buffers, one thread, per size, and prints the crossover:

  host    nova_diag_host_extend_loop (the product's host Extend, native loop)
  device  nova_port_accelerated_crc32c in a child process started with
          NOVA_HOOK_MIN_BYTES=1 (every call goes to the device; the hook reads
          the variable once)

One JSON line per size and a final {"crossover_bytes": ...}.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SIZES = [64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20]


def child(sizes):
    """Device side: every call through the hook on the GPU (env set by the parent)."""
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_bytes
    lib = C.load()
    assert lib.nova_device_init() == 0
    import ctypes
    buf = splitmix64_bytes(13, max(sizes))
    p = ctypes.cast(buf.ctypes.data, ctypes.c_char_p)  # the address, no copy
    for size in sizes:
        want = C.Extend(0, buf[:size].tobytes())
        got = lib.nova_port_accelerated_crc32c(0, p, size)  # warm: staging, stream, tables
        assert got == want, (size, hex(got), hex(want))
        reps, dt = 1, 0.0
        while True:
            t0 = time.perf_counter()
            for _ in range(reps):
                lib.nova_port_accelerated_crc32c(0, p, size)
            dt = time.perf_counter() - t0
            if dt >= 0.2 or reps >= 1 << 14:
                break
            reps *= 2
        st = C.port_stats()
        print(json.dumps({"size": size, "device_us": dt / reps * 1e6, "device_calls": st["device"],
                          "fallbacks": st["fallback"]}), flush=True)


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(SIZES)
        return 0
    from novalsm_amd import crc32c as C
    from novalsm_amd.synth import splitmix64_bytes
    fn = C.load_diag().nova_diag_host_extend_loop
    buf = splitmix64_bytes(13, max(SIZES))
    host_us = {}
    for size in SIZES:
        reps = 1
        while True:
            t0 = time.perf_counter()
            fn(buf.ctypes.data, size, reps)
            dt = time.perf_counter() - t0
            if dt >= 0.2:
                break
            reps *= 2
        host_us[size] = dt / reps * 1e6
    env = dict(os.environ, NOVA_HOOK_MIN_BYTES="1")
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                         capture_output=True, text=True, check=True).stdout
    dev_us = {}
    for line in out.splitlines():
        if line.startswith("{"):
            r = json.loads(line)
            dev_us[r["size"]] = r["device_us"]
            assert r["fallbacks"] == 0, r
    cross = None
    for size in SIZES:
        h, d = host_us[size], dev_us[size]
        print(json.dumps({"size": size, "host_us": round(h, 2), "device_us": round(d, 2),
                          "host_GiBps": round(size / h / 1e-6 / 2**30, 2),
                          "device_GiBps": round(size / d / 1e-6 / 2**30, 2),
                          "faster": "device" if d < h else "host"}), flush=True)
        if cross is None and d < h:
            cross = size
    print(json.dumps({"crossover_bytes": cross,
                      "note": "smallest size measured at which the device path beats the host Extend"}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
