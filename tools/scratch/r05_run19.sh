set -u
mkdir -p gpurun_out
for pm in 512 4096; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --var-ab 2,32768,65536 --steps 30 --warmup 20 > gpurun_out/pol19_$pm.log 2>&1 || { tail -20 gpurun_out/pol19_$pm.log; exit 1; }
  echo "== $pm"; grep -h '"variant"' gpurun_out/pol19_$pm.log | cut -c1-120
done
timeout -k 10 400 python -u tools/bench_ops.py --ops verify --images sst4k --no-ablations --var-ab 2,32768,65536 --steps 30 --warmup 20 > gpurun_out/pol19_verify.log 2>&1 || { tail -20 gpurun_out/pol19_verify.log; exit 1; }
grep -h '"variant"' gpurun_out/pol19_verify.log | cut -c1-120
