set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "lane_xor or sst_queue or concurrent" > gpurun_out/pt_q.log 2>&1 || { tail -40 gpurun_out/pt_q.log; exit 1; }
tail -8 gpurun_out/pt_q.log
bash tools/ab_libs.sh || exit 1
timeout -k 10 400 python -u tools/concurrent_sst.py --seconds 0.5 > gpurun_out/concurrent_sst2.log 2>&1 || exit 1
NOVA_SST_QUEUE_SLOTS=1 timeout -k 10 200 python -u tools/concurrent_sst.py --seconds 0.5 --paths queue --blocks 4096 > gpurun_out/concurrent_sst_slots1.log 2>&1
