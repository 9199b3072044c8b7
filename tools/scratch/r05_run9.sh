set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'max', d['max_us'], 'L', e['launches'], 'ring_dev', e.get('ring_device'), d['verified'])
" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests9.log 2>&1 || { tail -30 gpurun_out/engine_tests9.log; exit 1; }
tail -1 gpurun_out/engine_tests9.log
for rep in 1 2; do
for ring in device host; do
  NOVA_SST_ENGINE_RING=$ring timeout -k 10 300 python -u tools/concurrent_sst.py --threads 1,8,16 --blocks 4096 --paths engine --seconds 1 > gpurun_out/conc9_${ring}_$rep.log 2>&1 || exit 1
  echo "== ring $ring rep $rep"; summ gpurun_out/conc9_${ring}_$rep.log
done
done
