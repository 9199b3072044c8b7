#!/bin/bash
# Round-2 diagnosis of the two slowest composites:
#   1. log records on the rounds kernel: lanes per record x chunk size;
#   2. SQ counters for the log write path (post line-grid tree);
#   3. FETCH_SIZE / WRITE_SIZE for the trailer writer vs plain store vs verify on
#      the SSTable-like image, each counter in its own --pmc pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
V=""
for g in 2 4 8 16; do
  for c in 0 16 32 64; do V="$V,rounds:$g:$((c * 4 + 3)):0:0"; done
done
V=${V#,}
timeout -k 10 400 python3 -u tools/sweep_flat.py --workloads log --variants "$V" --rounds 2 --iters 10 \
  > gpurun_out/exp/log_sweep.log 2>&1 || { echo "log sweep failed rc=$?"; exit 1; }
timeout -k 10 200 bash tools/pmc_sq.sh log auto log_r02 > gpurun_out/exp/sq_log.log 2>&1 || { echo "sq failed rc=$?"; exit 1; }
for wl in sst4k sst4k_tw sst4k_vf; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/exp/pmc_$wl/$ctr -o pmc \
      -- python3 tools/probe.py $wl auto 6 > gpurun_out/exp/pmc_${wl}_$ctr.log 2>&1 || { echo "pmc $wl $ctr failed rc=$?"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for wl in ("sst4k", "sst4k_tw", "sst4k_vf"):
    acc = collections.defaultdict(list)
    for path in glob.glob(f"gpurun_out/exp/pmc_{wl}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                if "crc32c" in k or "trailer" in k:
                    acc[(k[:44], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        v.sort()
        print(f"{wl:9s} {k:44s} {c:12s} median {v[len(v)//2]:.5g} (n={len(v)})")
PY
