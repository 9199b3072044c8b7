#!/bin/bash
# End-of-round measurement on one box: smoke, the whole GPU suite, the driver's
# bench line, rocprof kernel stats of the same command, PMC traffic passes for
# every workload of the line (PMC_CFGS; SQ=1 adds the SQ issue/wait passes;
# summarised on the host afterwards: python tools/pmc_summary.py <cfg>), the
# composite ops.  Stops at the first
# failing step.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 3
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof,pmc,ops}
[[ $STEPS == *smoke* ]] && step final_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && step final_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *bench* ]] && step final_bench 600 python bench.py --detail-out gpurun_out/bench_detail.json
# (the sst_engine secondary is left out: under kernel tracing the persistent
# engine's callers stalled the run past the box's 3-minute silence limit)
[[ $STEPS == *prof* ]] && step final_rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --no-cpu-baseline --secondary 3,4,sst4k_trailers,sst4k_verify,log4k_write,log4k_verify,log512_write,log512_verify,parity,5
if [[ $STEPS == *pmc* ]]; then
  for cfg in ${PMC_CFGS:-2 3 4 sst4k_trailers sst4k_verify log4k_write log4k_verify log512_write log512_verify parity}; do
    rm -rf gpurun_out/pmc$cfg
    step final_pmc_$cfg 400 bash tools/pmc.sh $cfg
  done
fi
[[ $STEPS == *ops* ]] && step final_ops 600 python -u tools/bench_ops.py --images sst4k
exit 0
