#!/bin/bash
# Round 6, session 23: blocks per engine chunk for a lone caller (and two):
# NOVA_SST_ENGINE_CB 1-4 against the default (4 below 20K blocks in flight),
# verify on 4096-block tables, every result checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for cb in 0 1 2 3; do
    timeout -k 10 120 env NOVA_SST_ENGINE_CB=$cb python -u tools/concurrent_sst.py --ops verify --threads 1,2 --blocks 4096 --paths engine --seconds 1.0 > gpurun_out/s23_cb${cb}_$rep.log 2>&1 || { echo "cb $cb rc=$?"; exit 1; }
    echo "== s23_cb${cb}_$rep"
    grep '^{' gpurun_out/s23_cb${cb}_$rep.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['verified'])"
  done
done
