mkdir -p gpurun_out && rm -f gpurun_out/cmp.log
timeout -k 10 300 python -m pytest tests/test_gpu_scan.py -m gpu -x -q > gpurun_out/tcmp.log 2>&1 || exit 1
for r in 1 2; do
for L in libdpscan.so libdpscan_head.so libdpscan_v_steal.so libdpscan_v_coordpub.so libdpscan_v_coordpub_nopf.so libdpscan_v_nopf.so libdpscan_v_noprio.so libdpscan_v_coordpub_nopf_noprio.so; do
  DPSCAN_LIB=dataplug_amd/lib/$L timeout -k 10 120 python tools/probe_perf.py --no-stream --reps 8 | tail -1 >> gpurun_out/cmp.log || exit 1
done; done
tail -1 gpurun_out/tcmp.log
