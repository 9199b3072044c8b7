#!/bin/bash
# Round 6, session 2: the log paths' decode-stage loads (timing ablations:
# no tail line / no header / neither; tools/bench_ops.py --decode-ablations) at
# U[1,512] and U[1,4096] B payloads, and one lane per short record (diagnostics
# tuning, sorted windows).  Each step has its own time limit; stops at the
# first failure.
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
  grep '"op"\|"sweep"' "gpurun_out/$name.log" | cut -c1-200 | tail -n 12
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  step s2_dec512_$rep 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --decode-ablations --log-payload-max 512
  step s2_dec4k_$rep 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --decode-ablations
done
step s2_g1_512 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --lanes 1 --sort-sweep 2:0,2:-1024,2:-256
exit 0
