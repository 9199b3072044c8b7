#!/bin/bash
# Coalescing-queue checks and measurements, then the parity ceiling: queue
# tests -> one 4-thread queue point -> the concurrency sweep (direct vs queue,
# 1 and 2 slots) -> XOR parity vs copy ceilings -> parity PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "sst_queue" > gpurun_out/pt_queue.log 2>&1 || { tail -30 gpurun_out/pt_queue.log; exit 1; }
tail -3 gpurun_out/pt_queue.log
timeout -k 10 60 tools/bin/concurrent_sst verify 4 1024 0.5 queue || exit 1
echo "== burst mid sizes"
timeout -k 10 200 python -u tools/latency_burst.py --lanes 64,16,-1 --sizes 4096,8192,16384,32768,65536 --reps 100 > gpurun_out/latency_burst_mid.log 2>&1 || exit 1
echo "== concurrent"
timeout -k 10 400 python -u tools/concurrent_sst.py --seconds 0.5 > gpurun_out/concurrent_sst2.log 2>&1 || { tail -3 gpurun_out/concurrent_sst2.log; exit 1; }
NOVA_SST_QUEUE_SLOTS=1 timeout -k 10 200 python -u tools/concurrent_sst.py --seconds 0.5 --paths queue > gpurun_out/concurrent_sst_slots1.log 2>&1 || exit 1
echo "== parity ceiling"
timeout -k 10 300 python -u tools/ceiling.py --only parity > gpurun_out/parity_ceiling.log 2>&1 || { tail -5 gpurun_out/parity_ceiling.log; exit 1; }
tail -1 gpurun_out/parity_ceiling.log
BEST=$(python3 -c "import json; print(json.load(open('gpurun_out/parity_ceiling.json'))['summary']['best']['k0']['name'])")
echo "== pmc parity ($BEST)"
bash tools/pmc_parity.sh "$BEST" > gpurun_out/pmc_parity.log 2>&1 || { tail -5 gpurun_out/pmc_parity.log; exit 1; }
exit 0
