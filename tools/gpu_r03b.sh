#!/bin/bash
# Round-3 measurement call: GPU tests + lane_xor/wave_max A/B (ab_libs.sh),
# concurrent per-SSTable callers (direct vs coalescing queue), XOR parity vs
# its copy ceilings, parity PMC passes.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh || exit 1
echo "== concurrent"
timeout -k 10 400 python -u tools/concurrent_sst.py --seconds 0.5 > gpurun_out/concurrent_sst2.log 2>&1 || exit 1
NOVA_SST_QUEUE_SLOTS=1 timeout -k 10 200 python -u tools/concurrent_sst.py --seconds 0.5 --paths queue --blocks 4096 > gpurun_out/concurrent_sst_slots1.log 2>&1 || exit 1
echo "== parity ceiling"
timeout -k 10 300 python -u tools/ceiling.py --only parity > gpurun_out/parity_ceiling.log 2>&1 || exit 1
tail -1 gpurun_out/parity_ceiling.log
BEST=$(python3 -c "import json; print(json.load(open('gpurun_out/parity_ceiling.json'))['summary']['best']['k0']['name'])")
echo "== pmc parity ($BEST)"
bash tools/pmc_parity.sh "$BEST" > gpurun_out/pmc_parity.log 2>&1 || { tail -5 gpurun_out/pmc_parity.log; exit 1; }
exit 0
