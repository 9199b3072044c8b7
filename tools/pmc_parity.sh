#!/bin/bash
# HBM traffic of the XOR parity kernel and of its 8-read + 1-write copy
# ceiling (tools/ceiling.py --only parity --one NAME), one rocprofv3 --pmc pass
# per counter and per variant.  Usage: bash tools/pmc_parity.sh [CEILING_NAME]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
BEST=${1:-k0_u2_l1_s1_g0}
for v in product "$BEST"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmcpar/$v/$ctr
    mkdir -p $d
    timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $d -o pmc \
      -- python3 tools/ceiling.py --only parity --one $v > $d.log 2>&1 || { echo "pmc $v $ctr failed rc=$?"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, json, collections
res = {}
for path in glob.glob("gpurun_out/pmcpar/*/*/**/*counter_collection.csv", recursive=True):
    v, ctr = path.split("/")[2:4]
    vals = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row.get("Counter_Name") == ctr:
            vals[row["Kernel_Name"][:60]].append(float(row["Counter_Value"]))
    for k, xs in vals.items():
        if "parity" in k or "copy_ceiling" in k:
            xs.sort()
            med = xs[len(xs) // 2]
            # gfx950: FETCH_SIZE counts 128-B streaming reads at 64 B (MI355X_MICROARCH.md)
            res.setdefault(v, {})[ctr] = {"kernel": k, "launches": len(xs), "median_kib": med,
                                         "hbm_bytes": med * 1024 * (2 if ctr == "FETCH_SIZE" else 1)}
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/pmc_parity.json", "w"), indent=1)
PY
