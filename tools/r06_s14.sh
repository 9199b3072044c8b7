#!/bin/bash
# Round 6, session 14: the engine at 12 waves per CU (two-pass build, kEK12 = 9
# swaths per pass, 157 VGPRs) against the 8-wave one-pass build (kEK = 18,
# 211 VGPRs): engine GPU tests at 12 waves, then verify / trailers on
# 4096-block tables at 1, 8 and 16 callers, NOVA_SST_ENGINE_WAVES alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l)
        print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['verified'])
    elif 'passed' in l or 'failed' in l or 'Error' in l:
        print(l.rstrip())"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
# configurations "waves:ek" (ek 0: the build's default pass size)
W=${WAVES:-"8:0 12:0 12:6"}
if [ "${TESTS:-1}" = 1 ]; then
  step s14_tests_w12k6 300 env NOVA_SST_ENGINE_WAVES=12 NOVA_SST_ENGINE_EK=6 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
fi
for rep in 1 2; do
  for cfg in $W; do
    w=${cfg%%:*}; k=${cfg##*:}
    step s14_w${w}k${k}_$rep 200 env NOVA_SST_ENGINE_WAVES=$w NOVA_SST_ENGINE_EK=$k python -u tools/concurrent_sst.py --ops verify,trailers --threads 1,8,16 --blocks 4096 --paths engine --seconds 1.0
  done
done
exit 0
