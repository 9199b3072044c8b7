#!/bin/bash
# Log-stream kernel profile: kernel trace (pre-pass / main / gated fallback
# split) and SQ counters for the 4 GiB log workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${VAR:-logstream:0:0:0:0}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lsprof -o run -- python3 tools/probe.py log $VAR 8 > gpurun_out/lsprof.log 2>&1 || { echo "trace rc=$?"; exit 1; }
cat gpurun_out/lsprof/run_kernel_stats.csv | cut -c1-160
timeout -k 10 200 bash tools/pmc_sq.sh log $VAR ls > gpurun_out/lssq.log 2>&1 || { echo "sq rc=$?"; tail gpurun_out/lssq.log; exit 1; }
grep logstream gpurun_out/lssq.log || cat gpurun_out/lssq.log
