#!/bin/bash
# SQ counters of the rounds kernel on log write, log verify and SSTable verify.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in log log_vf sst4k_vf; do
  bash tools/pmc_sq.sh $wl auto:0:0:0:0 $wl > gpurun_out/sq_$wl.log 2>&1 || { cat gpurun_out/sq_$wl.log; exit 1; }
done
cat gpurun_out/sq_log.log gpurun_out/sq_log_vf.log gpurun_out/sq_sst4k_vf.log
