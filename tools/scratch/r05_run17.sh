set -u
mkdir -p gpurun_out
for pm in 256 512 1024 4096; do
  timeout -k 10 300 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --var-ab 16384 --steps 30 --warmup 20 > gpurun_out/fe17_$pm.log 2>&1 || { tail -20 gpurun_out/fe17_$pm.log; exit 1; }
  echo "== $pm"; grep -h '"variant"\|"op"' gpurun_out/fe17_$pm.log | cut -c1-150
done
timeout -k 10 300 python -u tools/bench_ops.py --ops verify --images sst4k --no-ablations --var-ab 16384 --steps 30 --warmup 20 > gpurun_out/fe17_verify.log 2>&1 || { tail -20 gpurun_out/fe17_verify.log; exit 1; }
grep -h '"variant"\|"op"' gpurun_out/fe17_verify.log | cut -c1-150
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "log or verify or trailer" --timeout 300 --timeout-method thread > gpurun_out/tests17.log 2>&1 || { tail -30 gpurun_out/tests17.log; exit 1; }
tail -1 gpurun_out/tests17.log
