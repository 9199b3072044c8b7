set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_ops.py --ops log_write,log_verify --log-payload-max 512 --sort-sweep 0,2 --steps 30 --warmup 20 > gpurun_out/abl20.log 2>&1 || { tail -20 gpurun_out/abl20.log; exit 1; }
grep -h '"sweep"\|"op"' gpurun_out/abl20.log | cut -c1-160
