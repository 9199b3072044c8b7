#!/bin/bash
# GPU tests after the burst-threshold change, parity variants, queue slots 2/4,
# burst vs rounds around the new threshold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
#timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
#tail -2 gpurun_out/pytest_gpu.log
echo "== parity sweep"
timeout -k 10 300 python -u tools/bench_ops.py --ops parity --images sst4k --no-ablations --parity-sweep 0x812,0xff81,0xff82,0x881,0xff41,0xff11,0xff12,0x1081,0x2081 > gpurun_out/parity_sweep.log 2>&1 || { tail -5 gpurun_out/parity_sweep.log; exit 1; }
echo "== burst threshold"
timeout -k 10 200 python -u tools/latency_burst.py --lanes 64,-1 --sizes 6144,10240,12288,14336 --reps 100 > gpurun_out/latency_burst_thr.log 2>&1 || exit 1
echo "== queue slots"
for sl in 2 4; do
  NOVA_SST_QUEUE_SLOTS=$sl timeout -k 10 300 python -u tools/concurrent_sst.py --seconds 0.5 --paths queue --threads 4,8,16 > gpurun_out/concurrent_q$sl.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/concurrent_sst.py --seconds 0.5 --paths direct --threads 4,8,16 > gpurun_out/concurrent_direct.log 2>&1 || exit 1
exit 0
