#!/bin/bash
# Round 6, session 5: log4k verify's result placement -- by position + the
# un-permute pass (product, sort mode 2) vs in place (4), and windows without
# the in-chunk sort (3 / 5), alternated three times (tools/log_sort_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-2:0:0,4:0:0,3:0:0,5:0:0}
timeout -k 10 400 python -u tools/log_sort_ab.py --variants "$V" --rounds 3 > gpurun_out/s5_log4k_place.log 2>&1 || { tail -5 gpurun_out/s5_log4k_place.log; exit 1; }
grep '"variant"' gpurun_out/s5_log4k_place.log
