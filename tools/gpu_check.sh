#!/bin/bash
# One gpurun call: smoke -> GPU parity tests -> bench -> rocprof kernel trace.
# Every GPU step has its own time limit; the script stops at the first step that
# faults, aborts, segfaults or times out (exit >= 2 other than pytest's 1).
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
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && step pytest_gpu 900 python -m pytest tests -m gpu -q -x
[[ $STEPS == *bench* ]] && step bench 600 python bench.py
[[ $STEPS == *prof* ]] && step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
[[ $STEPS == *cfgs* ]] && for c in 3 4 5; do step bench_config$c 600 python bench.py --config $c --no-cpu-baseline; done
[[ $STEPS == *pmc* ]] && step pmc2 900 bash tools/pmc.sh 2
exit 0
