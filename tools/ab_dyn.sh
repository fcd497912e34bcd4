set -o pipefail
O=gpurun_out/ab23; mkdir -p $O
L=dataplug_amd/lib
for i in 1 2 3; do
 for v in base f1; do
  DPSCAN_LIB=$L/libdpscan_v_$v.so timeout -k 10 200 python tools/probe_perf.py --no-stream --reps 10 >> $O/probe.log 2>&1 || exit 1
 done
done
