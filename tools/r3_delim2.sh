# Round 3: the newline index's two-kernel form with 64-range placement blocks: its GPU tests with every launch
# in that form, then the one-pass vs two-kernel sweep over CSV / VCF / FASTA bytes (same box).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_delim2}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step delim-twokernel-tests
DP_DELIM_TWOPASS_MAX=1099511627776 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "delim or csv or vcf or fastq or line or newline or gz" > $O/gpu_tests_delim2.log 2>&1 || { tail -30 $O/gpu_tests_delim2.log; exit 1; }
tail -1 $O/gpu_tests_delim2.log
step delim-sweep
timeout -k 10 400 python -u tools/delim_sweep.py --sizes-gib 0.0625,0.125,0.25,0.5,1,2,4 > $O/delim_sweep.log 2>&1 || { tail -20 $O/delim_sweep.log; exit 1; }
cat $O/delim_sweep.log | cut -c1-200
step done
