#!/bin/bash
# Same-box composite bounds: trailer writer (product, CRC-pass-only ablation,
# isolated scatter of 1M trailers after an image read), XOR parity (product
# vs copy ceilings, extended variant sweep), parity/queue tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "parity or queue or dispatch_thresholds or memory_growth" > gpurun_out/pt_e.log 2>&1 || { tail -30 gpurun_out/pt_e.log; exit 1; }
tail -1 gpurun_out/pt_e.log
echo "== trailer bound"
timeout -k 10 300 python -u tools/bench_ops.py --ops trailers,verify --images sst4k > gpurun_out/tb_ops1.log 2>&1 || exit 1
timeout -k 10 120 tools/bin/exp_scatter > gpurun_out/tb_scatter.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_ops.py --ops trailers,verify --images sst4k > gpurun_out/tb_ops2.log 2>&1 || exit 1
echo "== parity"
timeout -k 10 300 python -u tools/ceiling.py --only parity > gpurun_out/parity_ceiling.log 2>&1 || exit 1
tail -1 gpurun_out/parity_ceiling.log
timeout -k 10 300 python -u tools/bench_ops.py --ops parity --images sst4k --no-ablations --parity-sweep 0x12,0x11,0x14,0x18,0x22,0x24,0x42,0x44,0x81,0x82,0x812 > gpurun_out/parity_sweep2.log 2>&1 || exit 1
exit 0
