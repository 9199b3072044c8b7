#!/bin/bash
# Round 4: the page-granularity registration test, log write's composite bound
# on both log images, and the parity line (copy ceiling at 1-8 chunks per lane).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "pageable" > gpurun_out/r04a_tests.log 2>&1 || { tail -n 30 gpurun_out/r04a_tests.log; exit 1; }
tail -n 4 gpurun_out/r04a_tests.log
for pm in 4096 512; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write --log-payload-max $pm --log-bound \
    > gpurun_out/r04a_logbound_$pm.log 2>&1 || { tail -n 20 gpurun_out/r04a_logbound_$pm.log; exit 3; }
  grep -E '"op"|sweep' gpurun_out/r04a_logbound_$pm.log
done
timeout -k 10 300 python -u bench.py --config parity --steps 50 --warmup 10 --no-cpu-baseline --secondary none \
  > gpurun_out/r04a_parity.log 2>&1 || { tail -n 20 gpurun_out/r04a_parity.log; exit 3; }
tail -n 1 gpurun_out/r04a_parity.log
