set -u
mkdir -p gpurun_out
NOVA_CALLERS_TRACE=1 timeout -k 10 300 python -u tools/concurrent_sst.py --ops verify --threads 1,8 --blocks 4096 --paths engine --seconds 1 > gpurun_out/trace10.log 2>&1 || { tail -5 gpurun_out/trace10.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/trace10.log'):
  if not l.startswith('{'): continue
  d=json.loads(l); print(d['threads'], d['aggregate_GBps'], d['p50_us'], json.dumps(d['trace']))
"
