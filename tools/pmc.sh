#!/bin/bash
# HBM traffic of the CRC kernel from PMC counters, in separate passes (no
# sys/runtime tracing next to --pmc).  Usage: bash tools/pmc.sh [config]
# (config: 2, 3, 4, sst4k_trailers, sst4k_verify -- bench.py's workloads)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-2}
mkdir -p gpurun_out/pmc$CFG
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc$CFG/$ctr -o pmc \
    -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --secondary none --settle-ms 0 \
    > gpurun_out/pmc$CFG/$ctr.log 2>&1 || { echo "pmc $ctr failed rc=$?"; exit 1; }
done
python3 tools/pmc_summary.py $CFG
