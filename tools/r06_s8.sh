#!/bin/bash
# Round 6, session 8: waves per workgroup of the rounds kernel on the log
# composites (does G=2 log512 want fewer waves, as the lane-stream probe's
# 2-lane shape did?).  Each step has its own limit; stops at the first failure.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | grep '"sweep"\|"op"' | tail -n 12
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step s8_log512_waves 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --waves-sweep 6,8,10
step s8_log4k_waves 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --waves-sweep 8,10
exit 0
