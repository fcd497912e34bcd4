# Placement latency fixes (no private array, look-back loads together), new DELIM placement, 8-wave map A/B.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_probe2; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step delim-twokernel-tests
DP_DELIM_TWOPASS_MAX=1099511627776 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "delim or csv or vcf or fastq or line or newline" > $O/gpu_tests_delim2.log 2>&1 || { tail -30 $O/gpu_tests_delim2.log; exit 1; }
tail -2 $O/gpu_tests_delim2.log
step bench
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
cut -c1-200 $O/bench_fasta.json; grep -o '"kernel_avg_us": [0-9.]*\|"frac": [0-9.]*' $O/bench_fasta.json
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
cat $O/size_sweep.log
step delim-sweep
timeout -k 10 400 python -u tools/delim_sweep.py > $O/delim_sweep.log 2>&1 || { tail -20 $O/delim_sweep.log; exit 1; }
cat $O/delim_sweep.log
step place-timeline
for sz in 67108864 536870912 4294967296; do
  DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_prof2.so timeout -k 10 120 python -u tools/place_timeline.py --size $sz > $O/place_tl_$sz.json 2>&1 || { tail -20 $O/place_tl_$sz.json; exit 1; }
  cat $O/place_tl_$sz.json
done
step variants
bash tools/r3_variants.sh r3_probe2/var base mw8 || exit 1
step done
