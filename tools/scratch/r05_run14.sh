set -u
mkdir -p gpurun_out
for pm in ${PMS:-512 1024}; do
  timeout -k 10 400 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max $pm --no-ablations --lanes-sweep --steps 30 --warmup 20 > gpurun_out/lanes14_$pm.log 2>&1 || { tail -20 gpurun_out/lanes14_$pm.log; exit 1; }
  echo "== pmax $pm"; grep -h '"lanes"\|"op"' gpurun_out/lanes14_$pm.log | cut -c1-150
done
