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


# the kernels of one step of each workload (the first is the one whose
# dispatches count the steps) -- bench.py's dispatches
STEP_KERNELS = {
    "2": ["crc32c_stream_kernel<8, 0>"],
    "3": ["crc32c_units_kernel<16, 0>"],
    "4": ["crc32c_stream_kernel<16, 0>"],
    "sst4k_trailers": ["crc32c_rounds_kernel<8, 0>", "trailer_layout_kernel", "trailer_rmw_kernel"],
    "sst4k_verify": ["crc32c_rounds_kernel<8, 2>"],
    "log4k_write": ["crc32c_rounds_kernel<8, 3>"],
    "log4k_verify": ["crc32c_rounds_kernel<8, 4>", "log_sort_kernel", "log_unperm_kernel"],
    "log512_write": ["crc32c_rounds_kernel<2, 3>"],
    "log512_verify": ["crc32c_rounds_kernel<2, 4>"],
    "parity": ["xor_parity_kernel<8, 1>"],
}
SQ_COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
               "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
               "SQ_INSTS_VMEM_WR", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
               "SQ_INSTS_SMEM", "SQ_ACTIVE_INST_VALU"]


def label(name: str) -> str:
    m = re.search(r"xor_parity_kernel<([^>]*)>", name)
    if m:  # bench.py's dispatch names it with its template arguments
        return f"xor_parity_kernel<{m.group(1)}>"
    m = re.search(r"(trailer_\w+_kernel|log_\w+_kernel)", name)
    return m.group(1) if m and "crc32c_" not in name else kernel_label(name)


def per_kernel(ctr, cfg):
    vals = collections.defaultdict(list)
    for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc{cfg}", "**", "*counter_collection.csv"),
                          recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == ctr:
                    vals[label(row.get("Kernel_Name", ""))].append(float(row["Counter_Value"]))
    return vals


def step_bytes(vals, kernels):
    """Median per step: the main kernel's median plus the others' medians."""
    tot = 0.0
    for k in kernels:
        v = sorted(vals.get(k, []))
        if v:
            tot += v[len(v) // 2]
    return tot


def algorithmic(cfg):
    sys.path.insert(0, ROOT)
    import bench
    import numpy as np
    n = 1 << 20
    if cfg == "2":
        return 1 << 32
    if cfg == "4":
        return 1 << 34
    if cfg == "3":
        return int(bench.config3_layout(n, 3)[1].astype(np.uint64).sum())
    if cfg in ("sst4k_trailers", "sst4k_verify"):
        s = int(bench.sst4k_layout(n, 5)[1].astype(np.uint64).sum())
        return s + 5 * n if cfg == "sst4k_trailers" else s + 6 * n
    # the others: the bytes the bench line of the same pass reports
    path = os.path.join(ROOT, "gpurun_out", f"pmc{cfg}", "FETCH_SIZE.log")
    if os.path.exists(path):
        for line in reversed(open(path).read().splitlines()):
            if line.startswith("{"):
                return int(json.loads(line)["config"]["bytes_per_gpu"])
    return None


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
    kernels = STEP_KERNELS[cfg]
    fetch = per_kernel("FETCH_SIZE", cfg)
    write = per_kernel("WRITE_SIZE", cfg)
    if not fetch.get(kernels[0]):
        print(f"no FETCH_SIZE rows for {kernels[0]}; kernels seen: {sorted(fetch)}")
        sys.exit(1)
    f_kb = step_bytes(fetch, kernels)
    w_kb = step_bytes(write, kernels) if write else None
    sys.path.insert(0, ROOT)
    import bench
    algo = algorithmic(cfg)
    res = {
        "config": cfg,
        "kernels": kernels,
        "dispatches": len(fetch[kernels[0]]),
        "FETCH_SIZE_kB_per_step": f_kb,
        "WRITE_SIZE_kB_per_step": w_kb,
        "hbm_read_bytes_per_launch": 2 * f_kb * 1024,
        "hbm_write_bytes_per_launch": None if w_kb is None else w_kb * 1024,
        "hbm_bytes_per_launch": 2 * f_kb * 1024 + (0 if w_kb is None else w_kb * 1024),
        "algorithmic_bytes_per_launch": algo,
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM section); "
                      "WRITE_SIZE uncorrected",
        "kernel": kernels[0],
        "src_sha16": bench.kernel_src_sha16(),
        "commit": os.environ.get("PMC_COMMIT"),
    }
    if algo:
        res["read_over_algorithmic"] = res["hbm_read_bytes_per_launch"] / algo
    sq = {}
    for ctr in SQ_COUNTERS:  # the main kernel's median per dispatch
        v = sorted(per_kernel(ctr, cfg).get(kernels[0], []))
        if v:
            sq[ctr] = v[len(v) // 2]
    if sq:
        res["sq"] = sq
        kib = (algo or 0) / 1024.0
        if kib and "SQ_INSTS_VALU" in sq:
            res["valu_per_kib"] = sq["SQ_INSTS_VALU"] / kib
        if kib and "SQ_INSTS_LDS" in sq:
            res["lds_per_kib"] = sq["SQ_INSTS_LDS"] / kib
        if kib and "SQ_INSTS_SALU" in sq:
            res["salu_per_kib"] = sq["SQ_INSTS_SALU"] / kib
        if sq.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in sq:
            res["wait_over_wave_cycles"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
        if sq.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in sq:
            res["lds_conflict_over_active"] = sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]
    out = os.path.join(ROOT, os.environ.get("PMC_OUT_DIR", "profiles"), f"pmc_config{cfg}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
