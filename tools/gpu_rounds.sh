#!/bin/bash
# After a rounds-kernel change: GPU parity suite, then the variable-length
# workloads (sweep_flat: auto dispatch) and the composite ops (bench_ops).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sweep_flat.py --workloads ${WL:-log,sst4k,cfg3,c2var} --variants auto --rounds 3 --iters 10 > gpurun_out/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/sweep.log
timeout -k 10 400 python -u tools/bench_ops.py --ops trailers,verify,log_write,log_verify > gpurun_out/bench_ops.log 2>&1
echo "ops rc=$?"; grep -v amdgpu.ids gpurun_out/bench_ops.log | cut -c1-400
