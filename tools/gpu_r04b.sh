#!/bin/bash
# Round 4: lanes per record (2/4/8/16) on the short-record log images after the
# bucketed chunk sort (tools/bench_ops.py --lanes-sweep), payloads U[1,512] and U[1,1024].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pm in 512 1024; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max $pm \
    --lanes-sweep > gpurun_out/r04b_lanes_$pm.log 2>&1 || { tail -n 20 gpurun_out/r04b_lanes_$pm.log; exit 3; }
  echo "== pmax $pm"; grep -E '"op"|sweep' gpurun_out/r04b_lanes_$pm.log | cut -c1-160
done
