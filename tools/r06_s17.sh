#!/bin/bash
# Round 6, session 17: the retuned adaptive chunk size (0; 4 per ~21.8K blocks
# in flight at 12 waves) against fixed 4 / 8 / 12 / 16, engine at 12 waves,
# verify / trailers on 4096-block tables at 1, 8, 12 and 16 callers, every result
# checked, alternated over two repetitions.
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
        print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['verified'])"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  for cb in ${CBS:-0 4 8 12 16}; do
    step s17_cb${cb}_$rep 200 env NOVA_SST_ENGINE_CB=$cb python -u tools/concurrent_sst.py --ops verify,trailers --threads 1,8,12,16 --blocks 4096 --paths engine --seconds 1.0
  done
done
exit 0
