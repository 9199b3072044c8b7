set -u
timeout -k 10 60 python -u tools/stall_probe.py --seconds 3 > gpurun_out/stall_probe.log 2>&1; echo "== stall probe"; tail -1 gpurun_out/stall_probe.log
mkdir -p gpurun_out
for q in 1 0; do
  NOVA_SST_ENGINE_QUEUE=$q timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -m gpu -v -s --timeout 120 --timeout-method thread -k "mixed" > gpurun_out/mixed_q$q.log 2>&1
  echo "== mixed queue=$q rc=$?"
  grep -o '{"op".*' gpurun_out/mixed_q$q.log | python3 -c "
import json,sys
for l in sys.stdin:
  d=json.loads(l.split('\n')[0]); print(json.dumps({k:d[k] for k in ['op','aggregate_GBps','p50_us','p99_us','max_us','slowest_us_at_s']}), json.dumps({k:(v['max_us'],v['p50_us']) for k,v in d['plain'].items()}), d['engine']['launches'], d['engine']['exits_slice'], d['engine']['launch_us_max'], d['engine']['launch_slow'])"
done
for sl in 0 2000; do
  NOVA_SST_ENGINE_SLICE_US=$sl timeout -k 10 200 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --ops verify,trailers > gpurun_out/conc_slice_$sl.log 2>&1 || { echo conc failed; tail -5 gpurun_out/conc_slice_$sl.log; exit 1; }
  echo "== slice $sl"; python3 -c "
import json
for l in open('gpurun_out/conc_slice_$sl.log'):
  if l.startswith('{'):
    d=json.loads(l); print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['max_us'], d['slowest_us_at_s'][:3], d['engine']['launches'], d['engine']['launch_us_max'], d['engine']['launch_slow'], d['verified'])"
done
