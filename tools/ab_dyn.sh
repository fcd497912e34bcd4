set -o pipefail
O=gpurun_out/ab4; mkdir -p $O
L=dataplug_amd/lib
for i in 1 2; do
 for v in head c41 c81 c43 c42b; do
  f=$L/libdpscan_v_$v.so
  DPSCAN_LIB=$f timeout -k 10 200 python tools/probe_perf.py --no-stream --reps 10 >> $O/probe.log 2>&1 || exit 1
 done
done
