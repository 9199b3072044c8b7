#!/bin/bash
# One gpurun call after a kernel change: smoke -> GPU parity tests -> benches
# (config 2 default, config 3) -> composite ops -> variable-length sweep ->
# rocprof kernel stats of the default bench.  Every GPU step has its own time
# limit; the script stops at the first step that faults, aborts, segfaults or
# times out (exit >= 2 other than pytest's 1).  STEPS selects the steps.
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
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,cfg3,ops,sweep,prof}
VARIANTS=${VARIANTS:-auto,units:16:32768:12:0,rounds:8:131:12:0,rounds:8:259:12:0}
WORKLOADS=${WORKLOADS:-cfg3,sst4k,log}
[[ $STEPS == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *bench* ]] && step bench 600 python bench.py
[[ $STEPS == *trun* ]] && step bench_torchrun 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port=29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
[[ $STEPS == *cfg3* ]] && step bench_config3 600 python bench.py --config 3 --no-cpu-baseline
[[ $STEPS == *cfg4* ]] && step bench_config4 600 python bench.py --config 4 --no-cpu-baseline
[[ $STEPS == *ops* ]] && step bench_ops 600 python -u tools/bench_ops.py ${OPS_ARGS:-}
[[ $STEPS == *sweep* ]] && step sweep 600 python -u tools/sweep_flat.py --workloads "$WORKLOADS" --variants "$VARIANTS"
[[ $STEPS == *cross* ]] && step hook_crossover 600 python -u tools/hook_crossover.py
[[ $STEPS == *prof* ]] && step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
exit 0
