#!/bin/bash
# Mid-size SSTable-block batches (16K-256K blocks: a few SSTables, a compaction
# slab): rounds-kernel chunk size and lane-group width against the default
# plan, kernel time by HIP events (tools/latency.py --variants; diagnostics
# build).  Variant "rounds:G:X:0:0" with X = 4 * chunk + 3 (sorted chunks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SIZES=${SIZES:-16384,32768,65536,131072,262144}
VARS=${VARS:-auto,rounds:8:19:0:0,rounds:8:35:0:0,rounds:8:67:0:0,rounds:8:131:0:0,rounds:16:19:0:0,rounds:16:35:0:0,rounds:16:67:0:0}
timeout -k 10 500 python -u tools/latency.py --sizes "$SIZES" --variants "$VARS" > gpurun_out/midsize.log 2>&1
rc=$?
tail -n 8 gpurun_out/midsize.log
exit $rc
