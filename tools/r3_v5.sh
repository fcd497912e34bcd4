set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r3_v5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_v5/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3_v5/gpu_tests.log; [ $rc = 0 ] || exit 1
bash tools/r3_variants.sh r3_v5 base static soft1 soft2 onepass || exit 1
DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_prof.so timeout -k 10 120 python tools/place_timeline.py > gpurun_out/r3_v5/pl_prof.json 2>&1; cat gpurun_out/r3_v5/pl_prof.json
