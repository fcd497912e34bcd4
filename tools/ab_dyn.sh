set -o pipefail
O=gpurun_out/ab17; mkdir -p $O
L=dataplug_amd/lib
for i in 1 2; do
 for v in pre fix2 ad5 ad3; do
  DPSCAN_LIB=$L/libdpscan_v_$v.so timeout -k 10 300 python tools/probe_delim_modes.py --gib 8 >> $O/$v.log 2>&1 || exit 1
 done
done
