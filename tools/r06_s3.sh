#!/bin/bash
# Round 6, session 3: short log records (payloads U[1,512] B) at 2 and 4 lanes
# in sorted windows of 128-1024 records (log_sort_kernel, results by
# position), file-order chunk claims vs the XCD-contiguous order (ablation
# 11), every entry's results checked (tools/bench_ops.py --sort-sweep).
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
  grep '"op"\|"sweep"' "gpurun_out/$name.log" | cut -c1-230 | tail -n 20
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
SW=${SW:-2:0,2:-128,2:-256,2:-512,2:-1024,2:-256:0:11,2:-1024:0:11}
for rep in 1 2; do
  step s3_sorted512_g2_$rep 500 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --sort-sweep "$SW"
done
step s3_sorted512_g4 500 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --lanes 4 --sort-sweep "$SW"
exit 0
