set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['p999_us'], d['max_us'], d['slowest_us_at_s'][:3], 'L', e['launches'], 'lmax', e['launch_us_max'], 'sleepw',e['sleep_waits'],'spin',e['max_spinners'],'thr',d['cpu_throttled_periods'], d['verified'])
" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests6.log 2>&1 || { tail -30 gpurun_out/engine_tests6.log; exit 1; }
tail -1 gpurun_out/engine_tests6.log
for sl in 5000 0; do
  NOVA_SST_ENGINE_SLICE_US=$sl timeout -k 10 300 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --seconds 2 > gpurun_out/conc6_s$sl.log 2>&1 || exit 1
  echo "== slice $sl"; summ gpurun_out/conc6_s$sl.log
done
