#!/bin/bash
# Rounds kernel: loads-in-flight sensitivity -- waves per workgroup 6/8/10/12
# (launch bound 12) on the SSTable-like verify image (chunks of 32) and the log
# images (chunks of 64), tools/sweep_flat.py variants rounds:8:X:W:0 (sorted).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/sweep_flat.py --workloads sst4k_vf \
  --variants rounds:8:131:6:0,rounds:8:131:8:0,rounds:8:131:10:0,rounds:8:131:12:0 \
  --rounds 3 --iters 15 > gpurun_out/waves_sst.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep_flat.py --workloads log_vf,log \
  --variants rounds:8:259:6:0,rounds:8:259:8:0,rounds:8:259:10:0,rounds:8:259:12:0 \
  --rounds 3 --iters 15 > gpurun_out/waves_log.log 2>&1 || exit 1
grep -h '^{' gpurun_out/waves_sst.log gpurun_out/waves_log.log
