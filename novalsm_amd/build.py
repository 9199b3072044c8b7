"""Build the in-tree native libraries for gfx950.

Sources: novalsm_amd/csrc/{crc32c_device.hip, crc32c_stream.cpp, crc32c_host.cpp}
(+ crc32c_kernels.hpp, crc32c_internal.hpp) and, for the diagnostics library
only, crc32c_diag.hip.
Outputs (git-ignored, travel to the GPU box):
  novalsm_amd/lib/libnova_crc32c.so       the product: production kernels only
  novalsm_amd/lib/libnova_crc32c_diag.so  the SAME product objects plus
      crc32c_diag.o: timing ablations (some compute WRONG CRCs on purpose), the
      flat kernel, the sort pre-pass, the log-stream experiment, read-ceiling
      probes and the nova_diag_* knobs -- for tools/ and the tuning-variant
      tests, never for callers
hipcc cross-compiles gfx950 code objects without a GPU; the objects compile in
parallel.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libnova_crc32c.so")
DIAG_LIB = os.path.join(LIB_DIR, "libnova_crc32c_diag.so")
# native caller threads for the per-SSTable paths (bench.py, tools, tests);
# links the product library
CALLERS_LIB = os.path.join(LIB_DIR, "libnova_sst_callers.so")
CALLERS_SOURCE = "sst_callers.cpp"
ARCH = os.environ.get("NOVA_OFFLOAD_ARCH", "gfx950")

SOURCES = ["crc32c_device.hip", "crc32c_stream.cpp", "crc32c_host.cpp", "crc32c_queue.hip",
           "crc32c_engine.hip"]
DIAG_SOURCE = "crc32c_diag.hip"
HEADERS = ["gf2_crc32c.hpp", "crc32c_kernels.hpp", "crc32c_internal.hpp",
           os.path.join("..", "..", "include", "nova_crc32c.h"),
           os.path.join("..", "..", "include", "nova_crc32c.hpp")]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale(lib: str) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    extra = [DIAG_SOURCE] if lib == DIAG_LIB else []
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS + extra] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile_cmd(cc: str, src: str, obj: str, defines: list[str], extra: list[str] | None):
    cmd = [cc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
           "-I", os.path.join(ROOT, "include")] + defines + [
           "-c", os.path.join(CSRC, src), "-o", obj]
    if src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"] if "stream" in src else ["-x", "c++"]
    return cmd + (extra or [])


def build(force: bool = False, verbose: bool = False, extra: list[str] | None = None,
          diag: bool = True) -> str:
    """Build the product library (and, with diag=True, the diagnostics one)."""
    want = [LIB] + ([DIAG_LIB] if diag else [])
    if not force and not any(_stale(x) for x in want):
        if not os.path.exists(CALLERS_LIB) or \
                os.path.getmtime(os.path.join(CSRC, CALLERS_SOURCE)) > os.path.getmtime(CALLERS_LIB):
            build_callers()
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    cc = hipcc()
    jobs = {}  # obj -> cmd
    shared = []
    for src in SOURCES[1:]:
        obj = os.path.join(LIB_DIR, os.path.splitext(src)[0] + ".o")
        jobs[obj] = _compile_cmd(cc, src, obj, [], extra)
        shared.append(obj)
    dev_obj = os.path.join(LIB_DIR, "crc32c_device.o")
    jobs[dev_obj] = _compile_cmd(cc, SOURCES[0], dev_obj, [], extra)
    diag_obj = os.path.join(LIB_DIR, "crc32c_diag.o")
    if diag:
        jobs[diag_obj] = _compile_cmd(cc, DIAG_SOURCE, diag_obj, [], extra)
    # objects stay in lib/ (git- and gpurun-ignored): one whose source and the
    # shared headers are older than it is not compiled again
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [__file__]
    def fresh(obj: str, src: str) -> bool:
        if force or not os.path.exists(obj):
            return False
        t = os.path.getmtime(obj)
        return all(os.path.getmtime(d) <= t for d in hdrs + [os.path.join(CSRC, src)] if os.path.exists(d))
    srcs = {os.path.join(LIB_DIR, os.path.splitext(s)[0] + ".o"): s for s in SOURCES + [DIAG_SOURCE]}
    jobs = {o: c for o, c in jobs.items() if not fresh(o, srcs[o])}
    procs = []
    for obj, cmd in jobs.items():
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    links = [(LIB, [dev_obj] + shared)] + ([(DIAG_LIB, [dev_obj, diag_obj] + shared)] if diag else [])
    for lib, objs in links:
        tmp = lib + ".tmp"
        subprocess.run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
                       ["-lpthread"], check=True)
        os.replace(tmp, lib)
    build_callers(cc)
    return LIB


def build_callers(cc: str | None = None) -> str:
    """libnova_sst_callers.so (sst_callers.cpp) against the product library."""
    cc = cc or hipcc()
    tmp = CALLERS_LIB + ".tmp"
    subprocess.run([cc, "-x", "hip", f"--offload-arch={ARCH}", "-O2", "-fPIC", "-std=c++17", "-Wall", "-shared",
                    "-I", os.path.join(ROOT, "include"), os.path.join(CSRC, CALLERS_SOURCE), "-o", tmp,
                    "-L", LIB_DIR, "-lnova_crc32c", "-Wl,-rpath,$ORIGIN", "-lpthread"], check=True)
    os.replace(tmp, CALLERS_LIB)
    return CALLERS_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
