set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_v6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -15 $O/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 && cat $O/size_sweep.log &&
DP_DELIM_TWOPASS_MAX=0 timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.5,1,2,4,8 > $O/size_sweep_delim1.log 2>&1 && cat $O/size_sweep_delim1.log
