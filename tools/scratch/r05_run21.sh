set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests21.log 2>&1 || { tail -30 gpurun_out/engine_tests21.log; exit 1; }
tail -1 gpurun_out/engine_tests21.log
for rep in 1 2; do
for ps in 1 0; do
  NOVA_SST_ENGINE_PRESLEEP=$ps timeout -k 10 300 python -u tools/concurrent_sst.py --threads 8,16 --blocks 1024,4096 --paths engine --seconds 1 > gpurun_out/ps21_${ps}_$rep.log 2>&1 || exit 1
done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/ps21_*.log')):
  for l in open(f):
    if not l.startswith('{'): continue
    d=json.loads(l)
    print(f[-9:-4], d['op'], d['threads'], d['blocks_per_table'], d['aggregate_GBps'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'p999', d['p999_us'], 'max', d['max_us'], 'thr', d['cpu_throttled_periods'])
"
