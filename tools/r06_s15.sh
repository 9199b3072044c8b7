#!/bin/bash
# Round 6, session 15: the next ticket's claim issued under the chunk's last
# loads (NOVA_SST_ENGINE_EARLY_CLAIM=1, default) against the claim after the
# chunk's count (0, round 5), at 12 waves (and the 8-wave build): engine GPU
# tests, then verify / trailers on 4096-block tables at 1, 8 and 16 callers.
# (No gain measured: the switch and the early claim were removed after this
# run, profiles/r06_engine_waves.log.)
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
# configurations "waves:early_claim"
W=${WAVES:-"12:1 12:0 8:1"}
if [ "${TESTS:-1}" = 1 ]; then
  step s15_tests 300 env python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
fi
for rep in 1 2; do
  for cfg in $W; do
    w=${cfg%%:*}; k=${cfg##*:}
    step s15_w${w}e${k}_$rep 200 env NOVA_SST_ENGINE_WAVES=$w NOVA_SST_ENGINE_EARLY_CLAIM=$k python -u tools/concurrent_sst.py --ops verify,trailers --threads 1,8,16 --blocks 4096 --paths engine --seconds 1.0
  done
done
exit 0
