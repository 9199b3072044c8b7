#!/bin/bash
# SQ counters of the rounds kernel on the final tree: log write, log verify,
# SSTable-like verify (tools/pmc_sq.sh, two passes each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in log log_vf sst4k_vf; do
  bash tools/pmc_sq.sh $wl auto $wl > gpurun_out/sq_$wl.txt 2>&1 || { echo "sq $wl failed"; cat gpurun_out/sq_$wl.txt | tail -5; exit 1; }
done
cat gpurun_out/sq_*.txt
