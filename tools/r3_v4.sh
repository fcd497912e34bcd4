set -o pipefail
bash tools/r3_variants.sh r3_v4 base dyn onepass || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in prof profdyn; do
DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_$v.so timeout -k 10 120 python tools/place_timeline.py > gpurun_out/r3_v4/pl_$v.json 2>&1; cat gpurun_out/r3_v4/pl_$v.json
done
