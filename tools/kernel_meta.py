#!/usr/bin/env python3
"""Kernel resource metadata of a built library, without a GPU: VGPRs, spills
and private (scratch) memory per kernel, read from the gfx950 code objects
embedded in the .so (objcopy the .hip_fatbin section, clang-offload-bundler
--unbundle each bundle, llvm-readelf --notes).

  python tools/kernel_meta.py [novalsm_amd/lib/libnova_crc32c.so] [--all]

A kernel with private_segment_fixed_size > 0 keeps an array in scratch memory
(round 3: a whole-uint4 select in the rounds kernel's head masking did, and
every launch ran 2.4x slower); tests/test_host_api.py checks that no product
kernel does.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
BUNDLER = os.path.join(ROCM, "llvm", "bin", "clang-offload-bundler")
READELF = os.path.join(ROCM, "llvm", "bin", "llvm-readelf")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def tools_present() -> bool:
    return all(os.path.exists(p) for p in (BUNDLER, READELF)) and shutil.which("objcopy") is not None


def kernels(lib: str) -> dict:
    """{kernel symbol: {"vgpr": n, "vgpr_spill": n, "sgpr_spill": n, "private": bytes}}"""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, s in enumerate(starts):  # one bundle per translation unit with device code
            e = starts[k + 1] if k + 1 < len(starts) else len(data)
            b = os.path.join(d, f"b{k}.bin")
            open(b, "wb").write(data[s:e])
            co = os.path.join(d, f"b{k}.co")
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={b}", f"--targets={TARGET}",
                                f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
            cur = {}
            for line in notes.splitlines():
                m = re.match(r"^\s+\.(name|private_segment_fixed_size|vgpr_count|vgpr_spill_count|"
                             r"sgpr_spill_count):\s+(\S+)", line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2)
                if key == "name":
                    cur["name"] = val
                else:
                    cur[key] = int(val)
                if "name" in cur and "vgpr_spill_count" in cur and "private_segment_fixed_size" in cur:
                    out[cur["name"]] = {"vgpr": cur.get("vgpr_count", -1),
                                        "vgpr_spill": cur["vgpr_spill_count"],
                                        "sgpr_spill": cur.get("sgpr_spill_count", 0),
                                        "private": cur["private_segment_fixed_size"]}
                    cur = {}
    return out


def main() -> int:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(root, "novalsm_amd", "lib", "libnova_crc32c.so")
    ks = kernels(lib)
    bad = {k: v for k, v in ks.items() if v["private"] or v["vgpr_spill"]}
    for k, v in sorted(ks.items()):
        if "--all" in sys.argv or k in bad:
            print(v, k)
    print(f"{len(ks)} kernels, {len(bad)} with scratch or VGPR spills")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
