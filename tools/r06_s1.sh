#!/bin/bash
# Round 6, session 1 (one gpurun call): the GPU suite on this tree, then the
# log experiments -- log4k verify's sort key / window (timing + FETCH_SIZE per
# variant, tools/log_sort_ab.py) and one lane per short log record
# (tools/bench_ops.py --lanes 1 vs 2).  Every step has its own time limit; the
# script stops at the first failure.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
VARS=${VARS:-2:0:0,2:128:0,2:64:0,2:0:1,2:0:2,2:0:3,0}
STEPS=${STEPS:-pytest,sort,g1,pmc}
[[ $STEPS == *pytest* ]] && step s1_pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
[[ $STEPS == *sort* ]] && step s1_log_sort_ab 400 python -u tools/log_sort_ab.py --variants "$VARS" --rounds 2
if [[ $STEPS == *g1* ]]; then
  # one lane per record: file order, and sorted windows (negative: log write sorts too)
  for rep in 1 2; do
    for g in 2 1; do
      SW=""; [ $g = 1 ] && SW="--sort-sweep 2:-1024,2:-256,2:256,2:512"
      step s1_log512_g${g}_$rep 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 --lanes $g $SW
      grep '"op"\|"sweep"' gpurun_out/s1_log512_g${g}_$rep.log | sed "s/^/G=$g /" >> gpurun_out/s1_log512_lanes.log
    done
  done
fi
if [[ $STEPS == *pmc* ]]; then
  rm -rf gpurun_out/s1_pmc_sort
  step s1_pmc_sort 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s1_pmc_sort -o pmc \
    -- python3 tools/log_sort_ab.py --variants "$VARS" --rounds 1 --steps 10 --warmup 2
  step s1_pmc_split 60 python3 tools/log_sort_ab.py --split gpurun_out/s1_pmc_sort --variants "$VARS" --steps 10 --warmup 2
fi
exit 0
