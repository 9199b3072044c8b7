#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for the CRC kernel -> profiles/pmc_config<N>.json.

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read
(128-B requests tallied at 64 B), so hbm_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE
is exact for 16-B streaming stores (ours are 4-B: reported uncorrected)."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_label(name: str) -> str:
    """'void (anonymous namespace)::crc32c_units_kernel<16, 0, 0>(...)' ->
    'crc32c_units_kernel<16, 0>' (the form nova_crc32c_describe reports)."""
    m = re.search(r"(crc32c_\w+_kernel)<([^>]*)>", name)
    if not m:
        return name
    args = [a.strip() for a in m.group(2).split(",")][:2]
    return f"{m.group(1)}<{', '.join(args)}>"


KERNELS = collections.Counter()


def per_dispatch(ctr, cfg):
    vals = []
    for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc{cfg}", ctr, "**", "*counter_collection.csv"),
                          recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "crc32c" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    vals.append(float(row["Counter_Value"]))
                    KERNELS[kernel_label(row["Kernel_Name"])] += 1
    return vals


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
    fetch = per_dispatch("FETCH_SIZE", cfg)
    write = per_dispatch("WRITE_SIZE", cfg)
    if not fetch:
        print("no FETCH_SIZE rows found")
        sys.exit(1)
    f_med = sorted(fetch)[len(fetch) // 2]
    w_med = sorted(write)[len(write) // 2] if write else None
    algo = {"2": 1 << 32, "3": 30060563723, "4": 1 << 34}.get(cfg)  # config 3: bench.config3_layout sum
    res = {
        "config": int(cfg),
        "dispatches": len(fetch),
        "FETCH_SIZE_kB_median": f_med,
        "WRITE_SIZE_kB_median": w_med,
        "hbm_read_bytes_per_launch": 2 * f_med * 1024,
        "hbm_write_bytes_per_launch": None if w_med is None else w_med * 1024,
        "hbm_bytes_per_launch": 2 * f_med * 1024 + (0 if w_med is None else w_med * 1024),
        "algorithmic_bytes_per_launch": algo,
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM section)",
        "kernel": KERNELS.most_common(1)[0][0] if KERNELS else None,
        "commit": os.environ.get("PMC_COMMIT"),
    }
    if algo:
        res["read_over_algorithmic"] = res["hbm_read_bytes_per_launch"] / algo
    out = os.path.join(ROOT, os.environ.get("PMC_OUT_DIR", "profiles"), f"pmc_config{cfg}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
