#!/bin/bash
# Round 6, session 10: log write / verify at the same mean span (263.5 B) and
# record count, narrower payload spreads -- the rounds pad less (replay useful
# share 0.644 / 0.755 / 0.839 / 0.892), so the rate shows what fewer padded
# steps are worth (128-record chunks would give U[1,512] ~0.761).
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | grep '"op"' | cut -c1-200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  for mm in 1:512 128:384 200:312 256:256; do
    step s10_spread_${mm/:/_}_$rep 300 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations \
      --log-payload-min ${mm%:*} --log-payload-max ${mm#*:}
  done
done
exit 0
