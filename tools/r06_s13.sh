#!/bin/bash
# Round 6, session 13: blocks per engine chunk at 8 and 16 callers (verify and
# trailers, 4096-block tables, every result checked), NOVA_SST_ENGINE_CB
# alternated with the default (0: 8 at 8 callers, 16 at 16).  Needs the chunk
# cap (kEngMaxCb) raised above 16: the sweep ran with it at 64 (not kept).
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
  for cb in 0 24 32 48 64; do
    step s13_cb${cb}_$rep 200 env NOVA_SST_ENGINE_CB=$cb python -u tools/concurrent_sst.py --ops verify,trailers --threads 8,16 --blocks 4096 --paths engine --seconds 1.0
  done
done
exit 0
