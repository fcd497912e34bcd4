set -o pipefail
O=gpurun_out/ab19; mkdir -p $O
L=dataplug_amd/lib
DPSCAN_LIB=$L/libdpscan_v_sp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > $O/tests_sp.log 2>&1 || exit 1
for i in 1 2; do
 for v in base d14 sp; do
  DPSCAN_LIB=$L/libdpscan_v_$v.so timeout -k 10 200 python tools/probe_perf.py --no-stream --reps 10 >> $O/probe.log 2>&1 || exit 1
 done
done
