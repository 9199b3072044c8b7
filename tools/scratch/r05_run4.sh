set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['slowest_us_at_s'][:2], 'L',e['launches'],'slice',e['exits_slice'],'yield',e['exits_yield'],'sleepw',e['sleep_waits'],'spin',e['max_spinners'],'thr',d['cpu_throttled_periods'], json.dumps({k:(v['max_us'],v['p50_us']) for k,v in (d['plain'] or {}).items()}), d['verified'])
" "$1"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "engine or sst_queue or adjacent" > gpurun_out/engine_tests.log 2>&1 || { tail -30 gpurun_out/engine_tests.log; exit 1; }
tail -1 gpurun_out/engine_tests.log
timeout -k 10 300 python -u tools/concurrent_sst.py --threads 1,8,16 --blocks 4096 --paths engine > gpurun_out/conc_default.log 2>&1 || { tail -5 gpurun_out/conc_default.log; exit 1; }
echo "== default"; summ gpurun_out/conc_default.log
NOVA_SST_ENGINE_SPINNERS=64 timeout -k 10 300 python -u tools/concurrent_sst.py --threads 16 --blocks 4096 --paths engine > gpurun_out/conc_spin64.log 2>&1 || exit 1
echo "== all spin"; summ gpurun_out/conc_spin64.log
timeout -k 10 300 python -u tools/concurrent_sst.py --threads 8,16 --blocks 1024 --paths engine --ops verify > gpurun_out/conc_1k.log 2>&1 || exit 1
echo "== 1024-block tables"; summ gpurun_out/conc_1k.log
for pipe in 1 0; do
  NOVA_STREAM_HOST_PIPE=$pipe timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/cfg5_pipe$pipe.log 2>&1 || { tail -5 gpurun_out/cfg5_pipe$pipe.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cfg5_pipe$pipe.log').read().strip().splitlines()[-1]); r=d['roofline']
print('cfg5 pipe=$pipe', d['value'], 'GiB/s frac', r['frac'], 'ceiling', r['ceiling']['forms'], d['verified_sample'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "log" > gpurun_out/log_tests.log 2>&1 || { tail -30 gpurun_out/log_tests.log; exit 1; }
tail -1 gpurun_out/log_tests.log
timeout -k 10 300 python -u bench.py --config log512_verify --secondary log512_write,log4k_verify,log4k_write --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/logbench.log 2>&1 || { tail -5 gpurun_out/logbench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/logbench.log').read().strip().splitlines()[-1])
print('log512_verify', d['roofline']['frac'])
for s in d['secondary']: print(s['config'], s.get('frac'), s.get('kernel'))"
