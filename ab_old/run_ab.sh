#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out ab_new
export TMPDIR=/tmp
cp novalsm_amd/lib/libnova_crc32c.so novalsm_amd/lib/libnova_crc32c_diag.so ab_new/
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for leg in new old new old; do
  cp ab_$leg/libnova_crc32c.so ab_$leg/libnova_crc32c_diag.so novalsm_amd/lib/
  echo "== $leg"
  timeout -k 10 300 python -u tools/bench_ops.py --ops log_write,log_verify,trailers,verify --images sst4k > gpurun_out/ops_$leg.log 2>&1 || exit 3
  grep '"op"' gpurun_out/ops_$leg.log | sed "s/^/$leg /" >> gpurun_out/ab_ops.log
done
cp ab_new/libnova_crc32c.so ab_new/libnova_crc32c_diag.so novalsm_amd/lib/
exit 0
