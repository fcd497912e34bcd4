# Round 3: randomized campaigns of the final tree (one group per map claim; newline launches up to 48 MiB: two-kernel)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_fuzz_long}; mkdir -p $O
timeout -k 10 330 python -u tools/fuzz_gpu.py --mode kernel --seconds 300 --seed 81 --out $O/fuzz_s81.json > $O/fuzz_s81.log 2>&1 || { tail -20 $O/fuzz_s81.log; exit 1; }
tail -n 1 $O/fuzz_s81.log | cut -c1-400
timeout -k 10 260 python -u tools/fuzz_gpu.py --mode object --seconds 230 --seed 82 --out $O/fuzz_obj_s82.json > $O/fuzz_obj_s82.log 2>&1 || { tail -20 $O/fuzz_obj_s82.log; exit 1; }
tail -n 1 $O/fuzz_obj_s82.log | cut -c1-400
