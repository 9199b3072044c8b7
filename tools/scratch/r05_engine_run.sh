bash tools/gpu_engine.sh || exit 1
for sl in 0 1000 5000; do
  NOVA_SST_ENGINE_SLICE_US=$sl timeout -k 10 200 python -u tools/concurrent_sst.py --threads 8,16 --blocks 4096 --paths engine --ops verify > gpurun_out/conc_slice_$sl.log 2>&1 || exit 1
  echo "== slice $sl"; cut -c1-400 gpurun_out/conc_slice_$sl.log
done
