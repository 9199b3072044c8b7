#!/bin/bash
# Round 6, session 4: what the lines two short log records share cost.  Log
# verify at U[1,512] B payloads on the writer's packed layout and on layouts
# with every record at a multiple of 64 / 128 bytes (no 128-B line shared),
# unsorted (the product's 2 lanes) and in sorted windows of 256 / 1024 records
# (diagnostics), timing and FETCH_SIZE per variant (tools/log_sort_ab.py).
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
  grep '"variant"\|"image"' "gpurun_out/$name.log" | cut -c1-200 | tail -n 12
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
V=2:0:0,2:256:0,2:1024:0
for al in 0 128 64; do
  step s4_t_a$al 400 python -u tools/log_sort_ab.py --payload-max 512 --align $al --variants "$V" --rounds 2 --info gpurun_out/s4_info_a$al.json
  rm -rf gpurun_out/s4_pmc_a$al
  step s4_pmc_a$al 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s4_pmc_a$al -o pmc \
    -- python3 tools/log_sort_ab.py --payload-max 512 --align $al --variants "$V" --rounds 1 --steps 10 --warmup 2 --info gpurun_out/s4_info_a$al.json
  step s4_split_a$al 60 python3 tools/log_sort_ab.py --split gpurun_out/s4_pmc_a$al --variants "$V" --steps 10 --warmup 2 --info gpurun_out/s4_info_a$al.json
done
exit 0
