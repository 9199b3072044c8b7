set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests13.log 2>&1 || { tail -30 gpurun_out/engine_tests12.log; exit 1; }
tail -1 gpurun_out/engine_tests13.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --seconds 1 > gpurun_out/conc13_$rep.log 2>&1 || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/conc13_*.log')):
  for l in open(f):
    if not l.startswith('{'): continue
    d=json.loads(l)
    print(d['op'], d['threads'], d['aggregate_GBps'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'max', d['max_us'], 'sleepw', d['engine']['sleep_waits'])
    for s in d['slowest_detail'][:3]: print('   ', json.dumps(s))
"
