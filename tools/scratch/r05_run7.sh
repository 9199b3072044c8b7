set -u
mkdir -p gpurun_out
for pm in 512 4096; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --w16 --steps 30 --warmup 20 > gpurun_out/w16_log$pm.log 2>&1 || { tail -20 gpurun_out/w16_log$pm.log; exit 1; }
  grep -h '"waves"\|"op"' gpurun_out/w16_log$pm.log | cut -c1-200
done
timeout -k 10 400 python -u tools/bench_ops.py --ops verify --images sst4k --no-ablations --w16 --steps 30 --warmup 20 > gpurun_out/w16_verify.log 2>&1 || { tail -20 gpurun_out/w16_verify.log; exit 1; }
grep -h '"waves"\|"op"' gpurun_out/w16_verify.log | cut -c1-200
