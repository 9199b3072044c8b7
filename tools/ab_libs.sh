#!/bin/bash
# Same-box A/B of two builds of the libraries (one gpurun call): the working
# tree's novalsm_amd/lib ("new") against a previous build copied into ab_old/
# ("old", e.g. built from the parent commit), alternating new/old/new/old.
# Runs the GPU tests on "new" first; each leg times the composite ops of
# tools/bench_ops.py (OPS, default log_write,log_verify,trailers,verify on the
# SSTable-like image) and appends them to gpurun_out/ab_ops.log; with LAT=1 each
# leg also runs tools/latency_burst.py (burst-kernel launch times, default lanes)
# into gpurun_out/ab_lat.log; with LOG512=1 the log ops also on a U[1,512] B
# payload image; with LATR=1 tools/latency.py's mid-size batches
# (rounds kernel, default plan) into gpurun_out/ab_latr.log.  Every step has
# its own time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OPS=${OPS:-log_write,log_verify,trailers,verify}
mkdir -p gpurun_out ab_new
export TMPDIR=/tmp
[ -f ab_old/libnova_crc32c.so ] || { echo "ab_old/ holds no build"; exit 1; }
cp novalsm_amd/lib/libnova_crc32c.so novalsm_amd/lib/libnova_crc32c_diag.so ab_new/
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for leg in new old new old; do
  cp ab_$leg/libnova_crc32c.so ab_$leg/libnova_crc32c_diag.so novalsm_amd/lib/
  echo "== $leg"
  timeout -k 10 300 python -u tools/bench_ops.py --ops "$OPS" --images sst4k > gpurun_out/ops_$leg.log 2>&1 || exit 3
  grep '"op"' gpurun_out/ops_$leg.log | sed "s/^/$leg /" >> gpurun_out/ab_ops.log
  if [ "${LOG512:-0}" = 1 ]; then  # the short-record log image (payloads U[1,512] B)
    timeout -k 10 300 python -u tools/bench_ops.py --ops log_write,log_verify --no-ablations --log-payload-max 512 \
      > gpurun_out/ops512_$leg.log 2>&1 || exit 3
    grep '"op"' gpurun_out/ops512_$leg.log | sed "s/^/$leg 512 /" >> gpurun_out/ab_ops.log
  fi
  if [ "${LATR:-0}" = 1 ]; then  # mid-size batches, default dispatch (rounds kernel), events
    timeout -k 10 200 python -u tools/latency.py --sizes 16384,32768,65536,262144 --variants auto > gpurun_out/latr_$leg.log 2>&1 || exit 3
    grep '^{' gpurun_out/latr_$leg.log | sed "s/^/$leg /" >> gpurun_out/ab_latr.log
  fi
  if [ "${LAT:-0}" = 1 ]; then
    timeout -k 10 200 python -u tools/latency_burst.py --lanes 64,16 --sizes 16,256,1024,4096 > gpurun_out/lat_$leg.log 2>&1 || exit 3
    grep '^{' gpurun_out/lat_$leg.log | sed "s/^/$leg /" >> gpurun_out/ab_lat.log
  fi
done
cp ab_new/libnova_crc32c.so ab_new/libnova_crc32c_diag.so novalsm_amd/lib/
exit 0
