set -o pipefail
bash tools/r3_variants.sh r3_v2 base sync syncprio onepass || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_prof.so timeout -k 10 120 python tools/map_timeline.py > gpurun_out/r3_v2/tl_prof.json 2>&1; cat gpurun_out/r3_v2/tl_prof.json
DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_profsync.so timeout -k 10 120 python tools/map_timeline.py > gpurun_out/r3_v2/tl_profsync.json 2>&1; cat gpurun_out/r3_v2/tl_profsync.json
