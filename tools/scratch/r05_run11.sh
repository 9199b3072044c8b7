set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'max', d['max_us'], 'L', e['launches'], d['verified'])
" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests11.log 2>&1 || { tail -30 gpurun_out/engine_tests11.log; exit 1; }
tail -1 gpurun_out/engine_tests11.log
for rep in 1 2; do
for pp in 1 0; do
  NOVA_SST_ENGINE_PAGE_POLL=$pp timeout -k 10 300 python -u tools/concurrent_sst.py --threads 1,8,16 --blocks 4096 --paths engine --seconds 1 > gpurun_out/conc11_pp${pp}_$rep.log 2>&1 || exit 1
  echo "== page_poll $pp rep $rep"; summ gpurun_out/conc11_pp${pp}_$rep.log
done
done
NOVA_CALLERS_TRACE=1 timeout -k 10 300 python -u tools/concurrent_sst.py --ops verify --threads 1,8 --blocks 4096 --paths engine --seconds 1 > gpurun_out/trace11.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/trace11.log'):
  if not l.startswith('{'): continue
  d=json.loads(l); print(d['threads'], d['aggregate_GBps'], d['p50_us'], json.dumps(d['trace']))
"
