#!/bin/bash
# HBM traffic of a bench.py workload from PMC counters, one counter per pass
# (no sys/runtime tracing next to --pmc); with SQ=1 also two SQ issue/wait
# passes (8 SQ counters each).  Usage: [SQ=1] bash tools/pmc.sh [config]
# (config: any bench.py --config: 2, 3, 4, sst4k_*, log*_write/verify, parity)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-2}
mkdir -p gpurun_out/pmc$CFG
run() {  # run <dir> <counters...>
  local dir=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc$CFG/$dir -o pmc \
    -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --secondary none --settle-ms 0 \
    > gpurun_out/pmc$CFG/$dir.log 2>&1 || { echo "pmc $dir failed rc=$?"; exit 1; }
}
run FETCH_SIZE FETCH_SIZE
run WRITE_SIZE WRITE_SIZE
if [ "${SQ:-0}" = 1 ]; then
  run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
  run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU
fi
python3 tools/pmc_summary.py $CFG
