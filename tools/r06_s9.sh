#!/bin/bash
# Round 6, session 9: the rounds kernel's step work, timed by ablation (head
# masking, round-end group fold, WRONG results, no
# mismatch atomics) with the decode-stage ablations, log512 and log4k.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | grep '"sweep"\|"op"' | cut -c1-150 | tail -n 16
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step s9_log512_abl 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --decode-ablations
step s9_log4k_abl 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --decode-ablations
exit 0
