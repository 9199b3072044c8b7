#!/bin/bash
# Log verify sort windows across record-size distributions:
# the sorted-window GPU tests, then per (seed, payload max) the product's
# adaptive window (the "op" line) and fixed windows from the diagnostics knob.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "log_sorted_windows or log_96mib" \
  --timeout 200 --timeout-method thread > gpurun_out/logwin_tests.log 2>&1 || { tail -n 30 gpurun_out/logwin_tests.log; exit 1; }
tail -n 1 gpurun_out/logwin_tests.log
for cfg in ${CFGS:-6_4096 7_4096 6_16384 6_8192 6_1024 8_512}; do  # seed_payloadmax
  set -- ${cfg/_/ }
  echo "== seed $1 pmax $2" >> gpurun_out/logwin.log
  timeout -k 10 240 python -u tools/bench_ops.py --ops ${OPS:-log_verify} --no-ablations --log-seed $1 --log-payload-max $2 \
    --sort-sweep "${WINS:-2:64,2:128,2:256,2:512,2:1024}" ${EXTRA:-} >> gpurun_out/logwin.log 2>&1 || exit 3
done
exit 0
