set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r4_line1}; mkdir -p $O
DP_DELIM_FORM=line timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/delim_sweep.py --content csv,vcf,fasta --sizes-gib 0.0625,0.25,0.5,1,2,4 --reps 10 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
cat $O/sweep.log
