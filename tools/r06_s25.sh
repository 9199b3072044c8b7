#!/bin/bash
# Round 6, session 25: engine tails at 8 and 16 callers with the 12-wave build,
# 20 ms time slices (default) against none (NOVA_SST_ENGINE_SLICE_US=0),
# verify on 4096-block tables, every result checked, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for sl in default 0; do
    if [ $sl = default ]; then envs=""; else envs="NOVA_SST_ENGINE_SLICE_US=$sl"; fi
    timeout -k 10 150 env $envs python -u tools/concurrent_sst.py --ops verify --threads 8,16 --blocks 4096 --paths engine --seconds 1.0 > gpurun_out/s25_sl${sl}_$rep.log 2>&1 || { echo "rc=$?"; exit 1; }
    echo "== s25_slice_${sl}_$rep"
    grep '^{' gpurun_out/s25_sl${sl}_$rep.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['p999_us'], d['max_us'], round(d['max_us'] / d['p50_us'], 1), d['engine']['launches'], d['verified'])"
  done
done
