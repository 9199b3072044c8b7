set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for pm in 512 4096; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --var-ab 2 --steps 30 --warmup 20 > gpurun_out/cab_log$pm.log 2>&1 || { tail -20 gpurun_out/cab_log$pm.log; exit 1; }
  grep -h '"variant"\|"op"' gpurun_out/cab_log$pm.log | cut -c1-160
done
timeout -k 10 400 python -u tools/bench_ops.py --ops verify --images sst4k --no-ablations --var-ab 2 --steps 30 --warmup 20 > gpurun_out/cab_verify.log 2>&1 || { tail -20 gpurun_out/cab_verify.log; exit 1; }
grep -h '"variant"\|"op"' gpurun_out/cab_verify.log | cut -c1-160
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmccab_$c
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmccab_$c -o pmc -- python3 tools/bench_ops.py --ops log_write,log_verify --log-payload-max 512 --no-ablations --var-ab 2 --steps 4 --warmup 2 > gpurun_out/pmccab_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmccab_$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, re
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = collections.defaultdict(list)
    for p in glob.glob(f"gpurun_out/pmccab_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") == c:
                n = r.get("Kernel_Name", "")
                m = re.search(r"(\w+_kernel<[^>]*>)", n)
                vals[m.group(1) if m else n[:60]].append(float(r["Counter_Value"]))
    for k, v in sorted(vals.items()):
        v = sorted(v)
        print(c, k, "n", len(v), "median_kB", v[len(v) // 2])
PY
