#!/bin/bash
# Persistent SSTable engine on one box: its GPU tests, then
# the concurrent-caller matrix (tools/concurrent_sst.py) for the direct calls
# and the engine.  Stops at the first failing step.
#   STEPS=tests,conc,cbsweep  CONC_ARGS="--threads 1,8,16 --blocks 4096"
#   SWEEP_ENV=NOVA_SST_ENGINE_CB SWEEP_VALS="4 8 16" SWEEP_ARGS=...: one engine knob swept
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 12
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,conc}
TESTS_K=${TESTS_K:-"engine or sst_queue or adjacent"}
[[ $STEPS == *tests* ]] && step engine_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$TESTS_K"
[[ $STEPS == *conc* ]] && step engine_conc 600 python -u tools/concurrent_sst.py ${CONC_ARGS:---threads 1,4,8,16 --blocks 4096 --paths direct,engine}
if [[ $STEPS == *cbsweep* ]]; then
  for v in ${SWEEP_VALS:-4 8 16}; do
    env "${SWEEP_ENV:-NOVA_SST_ENGINE_CB}=$v" timeout -k 10 300 python -u tools/concurrent_sst.py \
      ${SWEEP_ARGS:---threads 1 --blocks 1024,4096 --paths engine_trace --ops verify} > "gpurun_out/sweep_$v.log" 2>&1 \
      || { echo "STOP after sweep $v"; exit 1; }
    echo "== sweep ${SWEEP_ENV:-NOVA_SST_ENGINE_CB}=$v"; grep '^{' "gpurun_out/sweep_$v.log"
  done
fi
exit 0
