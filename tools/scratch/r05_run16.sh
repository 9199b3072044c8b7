set -u
mkdir -p gpurun_out
for g in 2 4; do
  timeout -k 10 300 python -u tools/bench_ops.py --lanes $g --ops log_write,log_verify --log-payload-max 512 --no-ablations --chunk-sweep 16,32,48,64 --steps 30 --warmup 20 > gpurun_out/chunk16_g$g.log 2>&1 || { tail -20 gpurun_out/chunk16_g$g.log; exit 1; }
  echo "== G $g"; grep -h '"chunk"\|"op"' gpurun_out/chunk16_g$g.log | cut -c1-150
done
