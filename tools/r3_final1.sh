# Round 3, default build only: GPU tests, the 8-context and allocation logs, both fuzz modes, the DELIM form
# sweep, multi-group e2e, and the bench lines. Every step has its own time limit; the first failure ends it.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_final1; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step multi-logs
timeout -k 10 200 python -u -m pytest -s -q --timeout 150 --timeout-method thread "tests/test_gpu_multi.py::test_eight_contexts_share_the_scan_stream" "tests/test_gpu_multi.py::test_second_preprocess_allocates_nothing" > $O/multi_logs.log 2>&1 || { tail -20 $O/multi_logs.log; exit 1; }
grep -E "solo scan|alloc counts" $O/multi_logs.log
step fuzz-kernel
timeout -k 10 200 python -u tools/fuzz_gpu.py --mode kernel --seconds 100 --seed 31 --out $O/fuzz_s31.json > $O/fuzz_s31.log 2>&1 || { tail -20 $O/fuzz_s31.log; exit 1; }
tail -1 $O/fuzz_s31.log | cut -c1-400
step fuzz-object
timeout -k 10 200 python -u tools/fuzz_gpu.py --mode object --seconds 100 --seed 32 --out $O/fuzz_obj_s32.json > $O/fuzz_obj_s32.log 2>&1 || { tail -20 $O/fuzz_obj_s32.log; exit 1; }
tail -1 $O/fuzz_obj_s32.log | cut -c1-400
step e2e
timeout -k 10 300 python -u tools/e2e_rate.py --only memory,loopback_http --reps 2 > $O/e2e_1group.log 2>&1 || { tail -20 $O/e2e_1group.log; exit 1; }
timeout -k 10 300 python -u tools/e2e_rate.py --only memory,loopback_http --reps 2 --devices 0,0,0,0 --no-stages > $O/e2e_4groups.log 2>&1 || { tail -20 $O/e2e_4groups.log; exit 1; }
tail -3 $O/e2e_1group.log $O/e2e_4groups.log | cut -c1-300
step bench
timeout -k 10 300 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
cut -c1-300 $O/bench_fasta.json
timeout -k 10 300 python -u bench.py --workload csv --no-cpu-baseline > $O/bench_csv.json 2> $O/bench_csv.err || { tail -20 $O/bench_csv.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload vcf --no-cpu-baseline > $O/bench_vcf.json 2> $O/bench_vcf.err || { tail -20 $O/bench_vcf.err; exit 1; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), r.get('frac_of_mixed_peak'), d['verified_bit_exact'])
" $O/bench_fasta.json $O/bench_csv.json $O/bench_vcf.json
step delim-twokernel-tests
DP_DELIM_TWOPASS_MAX=1099511627776 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "delim or csv or vcf or fastq or line or newline" > $O/gpu_tests_delim2.log 2>&1 || { tail -30 $O/gpu_tests_delim2.log; exit 1; }
tail -2 $O/gpu_tests_delim2.log
step delim-sweep
timeout -k 10 400 python -u tools/delim_sweep.py > $O/delim_sweep.log 2>&1 || { tail -20 $O/delim_sweep.log; exit 1; }
grep fixed_us $O/delim_sweep.log
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
grep fixed_us $O/size_sweep.log
step variants
bash tools/r3_variants.sh r3_final1/var base mw8 || exit 1
step done
