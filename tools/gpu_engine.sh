#!/bin/bash
# Persistent SSTable engine on one box: its GPU tests, then
# the concurrent-caller matrix (tools/concurrent_sst.py) for the direct calls
# and the engine.  Stops at the first failing step.
#   STEPS=tests,conc  CONC_ARGS="--threads 1,8,16 --blocks 4096"
#   TESTS_K="engine or sst_queue or adjacent"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 14
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,conc}
TESTS_K=${TESTS_K:-"engine or sst_queue or adjacent"}
[[ $STEPS == *tests* ]] && step engine_tests 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 120 --timeout-method thread -k "$TESTS_K"
[[ $STEPS == *conc* ]] && step engine_conc 400 python -u tools/concurrent_sst.py ${CONC_ARGS:---threads 1,8,16 --blocks 4096 --paths engine}
exit 0
