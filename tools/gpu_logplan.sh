#!/bin/bash
# Full GPU test suite, then the product's log plan (no knobs: the "op" lines)
# over record-size distributions, seed_payloadmax.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-8_512 6_768 6_1024 6_1536 6_2048 6_4096 6_8192 6_16384}; do
  set -- ${cfg/_/ }
  echo "== seed $1 pmax $2" >> gpurun_out/logplan.log
  timeout -k 10 240 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-seed $1 \
    --log-payload-max $2 >> gpurun_out/logplan.log 2>&1 || exit 3
done
exit 0
