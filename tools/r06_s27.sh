#!/bin/bash
# Round 6, session 27: yield storms routed to the plain path (declined, not
# failed): the engine and queue GPU tests, then tools/mixed_callers.py (8
# engine callers beside a plain thread at 0 / 200 / 1000 / 5000 us gaps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "engine or sst_queue or adjacent" > gpurun_out/s27_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/s27_tests.log; exit 1; }
tail -1 gpurun_out/s27_tests.log
timeout -k 10 300 python -u tools/mixed_callers.py > gpurun_out/s27_mixed.log 2>&1 || { echo "mixed rc=$?"; tail -5 gpurun_out/s27_mixed.log; exit 1; }
echo done
