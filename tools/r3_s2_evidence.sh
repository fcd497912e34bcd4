# Round 3 evidence of HEAD: the 8-context and allocation logs, both fuzz modes, one- and four-group e2e rates.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_s2_evidence}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step multi-logs
timeout -k 10 200 python -u -m pytest -s -q --timeout 150 --timeout-method thread "tests/test_gpu_multi.py::test_eight_contexts_share_the_scan_stream" "tests/test_gpu_multi.py::test_second_preprocess_allocates_nothing" > $O/multi_logs.log 2>&1 || { tail -20 $O/multi_logs.log; exit 1; }
grep -E "solo scan|alloc counts" $O/multi_logs.log
step fuzz-kernel
timeout -k 10 200 python -u tools/fuzz_gpu.py --mode kernel --seconds 120 --seed 31 --out $O/fuzz_s31.json > $O/fuzz_s31.log 2>&1 || { tail -20 $O/fuzz_s31.log; exit 1; }
tail -1 $O/fuzz_s31.log | cut -c1-600
step fuzz-object
timeout -k 10 200 python -u tools/fuzz_gpu.py --mode object --seconds 120 --seed 32 --out $O/fuzz_obj_s32.json > $O/fuzz_obj_s32.log 2>&1 || { tail -20 $O/fuzz_obj_s32.log; exit 1; }
tail -1 $O/fuzz_obj_s32.log | cut -c1-600
step e2e
timeout -k 10 300 python -u tools/e2e_rate.py --only memory,loopback_http --reps 2 > $O/e2e_1group.log 2>&1 || { tail -20 $O/e2e_1group.log; exit 1; }
timeout -k 10 300 python -u tools/e2e_rate.py --only memory,loopback_http --reps 2 --devices 0,0,0,0 --no-stages > $O/e2e_4groups.log 2>&1 || { tail -20 $O/e2e_4groups.log; exit 1; }
tail -4 $O/e2e_1group.log $O/e2e_4groups.log | cut -c1-300
step done
