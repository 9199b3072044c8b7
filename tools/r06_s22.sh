#!/bin/bash
# Round 6, session 22: the log sort pre-pass with a wave-parallel prefix at 64
# threads per window: the log GPU tests, then log4k verify (and write, log512
# as controls) in one bench line, and rocprof of the log4k verify line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "log" > gpurun_out/s22_logtests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/s22_logtests.log; exit 1; }
tail -1 gpurun_out/s22_logtests.log
timeout -k 10 300 python bench.py --config log4k_verify --secondary log4k_write,log512_verify --no-cpu-baseline > gpurun_out/s22_bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/s22_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s22_prof -o run -- python3 bench.py --config log4k_verify --secondary none --no-cpu-baseline > gpurun_out/s22_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
