set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['slowest_us_at_s'][:3], 'L',e['launches'],'slice',e['exits_slice'],'yield',e['exits_yield'],'lmax',e['launch_us_max'],'lslow',e['launch_slow'],'gap',e['poll_gap_us_max'], json.dumps({k:(v['max_us'],v['p50_us']) for k,v in (d['plain'] or {}).items()}), d['verified'])
  if d.get('trace'): print('  trace', json.dumps(d['trace']))
" "$1"; }
for k in 1 2; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -m gpu -v -s --timeout 120 --timeout-method thread -k "mixed" > gpurun_out/mixed_$k.log 2>&1
  echo "== mixed $k rc=$?"; summ gpurun_out/mixed_$k.log
done
for sl in 0 2000 5000 10000; do
  NOVA_SST_ENGINE_SLICE_US=$sl timeout -k 10 200 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --ops verify > gpurun_out/conc_s$sl.log 2>&1 || { echo conc failed; tail -5 gpurun_out/conc_s$sl.log; exit 1; }
  echo "== slice $sl"; summ gpurun_out/conc_s$sl.log
done
NOVA_CALLERS_TRACE=1 timeout -k 10 200 python -u tools/concurrent_sst.py --threads 1,8 --blocks 4096 --paths engine --ops verify > gpurun_out/conc_trace.log 2>&1 || exit 1
echo "== trace"; summ gpurun_out/conc_trace.log
