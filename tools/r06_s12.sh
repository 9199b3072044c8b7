#!/bin/bash
# Round 6, session 12: where the engine's time goes at 1 / 8 / 16 callers
# (per-request spans from the engine's trace, NOVA_CALLERS_TRACE=1), verify on
# 4096-block tables, every result checked; then the same without the trace.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | cut -c1-240 | tail -n 6
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step s12_engine_trace 300 env NOVA_CALLERS_TRACE=1 python -u tools/concurrent_sst.py --ops verify --threads 1,8,16 --blocks 4096 --paths engine --seconds 1.0
step s12_engine_notrace 300 python -u tools/concurrent_sst.py --ops verify --threads 1,8,16 --blocks 4096 --paths engine,direct --seconds 1.0
exit 0
