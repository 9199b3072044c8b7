#!/bin/bash
# Parity at U = 8 / 16 on the one-pass grid against the copy ceilings (U <= 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "xor_parity" > gpurun_out/pt_f.log 2>&1 || { tail -30 gpurun_out/pt_f.log; exit 1; }
tail -1 gpurun_out/pt_f.log
timeout -k 10 300 python -u tools/ceiling.py --only parity > gpurun_out/parity_ceiling.log 2>&1 || exit 1
tail -1 gpurun_out/parity_ceiling.log
timeout -k 10 300 python -u tools/bench_ops.py --ops parity --images sst4k --no-ablations --parity-sweep 0x8,0x10,0x4,0x2,0x28,0x48,0x1008,0x1010 > gpurun_out/parity_sweep3.log 2>&1 || exit 1
BEST=$(python3 -c "import json; print(json.load(open('gpurun_out/parity_ceiling.json'))['summary']['best']['k0']['name'])")
bash tools/pmc_parity.sh "$BEST" > gpurun_out/pmc_parity.log 2>&1 || { tail -5 gpurun_out/pmc_parity.log; exit 1; }
exit 0
