set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "log" --timeout 300 --timeout-method thread > gpurun_out/logtests15.log 2>&1 || { tail -30 gpurun_out/logtests15.log; exit 1; }
tail -1 gpurun_out/logtests15.log
for pm in 512 1024 2048; do
  timeout -k 10 300 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --steps 30 --warmup 20 > gpurun_out/ops15_$pm.log 2>&1 || { tail -20 gpurun_out/ops15_$pm.log; exit 1; }
  grep -h '"op"' gpurun_out/ops15_$pm.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print($pm, d['op'], d['ms_per_launch'], d['roofline']['frac'], d.get('verified_sample'))"
done
