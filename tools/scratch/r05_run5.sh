set -u
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
  i=l.find('{\"op\"')
  if i<0: continue
  d=json.loads(l[i:].split('\n')[0]); e=d['engine']
  print(d['op'], d['threads'], d['aggregate_GBps'], d['p50_us'], d['p99_us'], d['p999_us'], d['max_us'], d['slowest_us_at_s'][:3], 'sleepw',e['sleep_waits'],'spin',e['max_spinners'],'thr',d['cpu_throttled_periods'], 'gap', e['poll_gap_us_max'], d['verified'])
" "$1"; }
for sp in 4 8 12; do
  NOVA_SST_ENGINE_SPINNERS=$sp timeout -k 10 300 python -u tools/concurrent_sst.py --threads 16 --blocks 4096 --paths engine --seconds 2 > gpurun_out/conc_sp$sp.log 2>&1 || exit 1
  echo "== spinners $sp"; summ gpurun_out/conc_sp$sp.log
done
