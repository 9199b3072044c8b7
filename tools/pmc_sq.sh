#!/bin/bash
# SQ issue/wait counters for one workload/variant (two --pmc passes, each its
# own run, no tracing next to --pmc).  Usage: bash tools/pmc_sq.sh <wl> <variant> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=$1; VAR=$2; TAG=$3
mkdir -p gpurun_out/sq_$TAG
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sq_$TAG/p1 -o pmc -- python3 tools/probe.py $WL $VAR 6 > gpurun_out/sq_$TAG/p1.log 2>&1 || { echo "pass1 failed rc=$?"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sq_$TAG/p2 -o pmc -- python3 tools/probe.py $WL $VAR 6 > gpurun_out/sq_$TAG/p2.log 2>&1 || { echo "pass2 failed rc=$?"; exit 1; }
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for path in glob.glob(f"gpurun_out/sq_{tag}/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if "crc32c" in row.get("Kernel_Name", ""):
                acc[(row["Kernel_Name"][:40], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    v.sort()
    print(f"{tag:10s} {k:40s} {c:24s} {v[len(v)//2]:.4g}  (n={len(v)})")
PY
