bash tools/gpu_engine.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "log" > gpurun_out/log_tests.log 2>&1 || { tail -30 gpurun_out/log_tests.log; exit 1; }
tail -2 gpurun_out/log_tests.log
for sl in 0 1000 5000; do
  NOVA_SST_ENGINE_SLICE_US=$sl timeout -k 10 200 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --ops verify > gpurun_out/conc_slice_$sl.log 2>&1 || exit 1
  echo "== slice $sl"; cut -c1-300 gpurun_out/conc_slice_$sl.log
done
timeout -k 10 300 python -u bench.py --config log512_verify --secondary log512_write,log4k_verify,log4k_write --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/logbench.log 2>&1 || { tail -5 gpurun_out/logbench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/logbench.log').read().strip().splitlines()[-1])
print('primary', d['config']['workload'][:30], d['roofline']['frac'])
for s in d['secondary']: print(s['config'], s.get('frac'), s.get('kernel'))"
for pipe in 1 0 1; do
  NOVA_STREAM_HOST_PIPE=$pipe timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/cfg5_pipe$pipe.log 2>&1 || { tail -5 gpurun_out/cfg5_pipe$pipe.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cfg5_pipe$pipe.log').read().strip().splitlines()[-1]); r=d['roofline']
print('cfg5 pipe=$pipe', d['value'], 'GiB/s frac', r['frac'], 'ceiling', r['ceiling']['forms'], d['verified_sample'])"
done
