set -o pipefail
O=gpurun_out/ab7; mkdir -p $O
L=dataplug_amd/lib
for v in pdata pa; do
DPSCAN_LIB=$L/libdpscan_v_$v.so timeout -k 10 120 python tools/timeline.py --out $O/tl_$v.npz > $O/tl_$v.log 2>&1 || exit 1
done
