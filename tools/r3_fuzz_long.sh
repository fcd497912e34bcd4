# Round 3: longer randomized campaigns of the final tree (newline launches up to 48 MiB: all two-kernel now)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_fuzz_long}; mkdir -p $O
timeout -k 10 330 python -u tools/fuzz_gpu.py --mode kernel --seconds 300 --seed 71 --out $O/fuzz_s71.json > $O/fuzz_s71.log 2>&1 || { tail -20 $O/fuzz_s71.log; exit 1; }
tail -n 1 $O/fuzz_s71.log | cut -c1-400
timeout -k 10 260 python -u tools/fuzz_gpu.py --mode object --seconds 230 --seed 72 --out $O/fuzz_obj_s72.json > $O/fuzz_obj_s72.log 2>&1 || { tail -20 $O/fuzz_obj_s72.log; exit 1; }
tail -n 1 $O/fuzz_obj_s72.log | cut -c1-400
