#!/bin/bash
# Log-record kernels side by side on the 4 GiB log image (tools/sweep_flat.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-auto,rounds:8:3:0:0,logstream:0:0:0:0,logstream:0:0:0:64}
timeout -k 10 300 python -u tools/sweep_flat.py --workloads log --variants "$V" --rounds 3 --iters 10 > gpurun_out/ls_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/ls_sweep.log
