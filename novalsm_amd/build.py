"""Build the in-tree native library libnova_crc32c.so for gfx950.

Sources: novalsm_amd/csrc/{crc32c_device.hip, crc32c_stream.cpp, crc32c_host.cpp}.
Output:  novalsm_amd/lib/libnova_crc32c.so (git-ignored, travels to the GPU box).
hipcc cross-compiles gfx950 code objects without a GPU.
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
ARCH = os.environ.get("NOVA_OFFLOAD_ARCH", "gfx950")

SOURCES = ["crc32c_device.hip", "crc32c_stream.cpp", "crc32c_host.cpp"]
HEADERS = ["gf2_crc32c.hpp", os.path.join("..", "..", "include", "nova_crc32c.h"),
           os.path.join("..", "..", "include", "nova_crc32c.hpp")]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, extra: list[str] | None = None) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    objs = []
    cc = hipcc()
    for src in SOURCES:
        obj = os.path.join(LIB_DIR, os.path.splitext(src)[0] + ".o")
        cmd = [cc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-I", os.path.join(ROOT, "include"), "-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"] if "stream" in src else ["-x", "c++"]
        cmd += extra or []
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = LIB + ".tmp"
    subprocess.run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
                   ["-lpthread"], check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
