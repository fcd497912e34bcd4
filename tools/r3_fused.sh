# Round 3: the fused FASTA form (map + placement in one launch) on the GPU: its parity tests first, then the
# whole GPU suite, a kernel fuzz campaign, bench lines of the three forms and the FASTA size sweep.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_fused}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step fused-tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -v --timeout 120 --timeout-method thread -k "forms or fused or golden or adversarial" > $O/fused_tests.log 2>&1 || { tail -30 $O/fused_tests.log; exit 1; }
tail -2 $O/fused_tests.log
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step fuzz-kernel
timeout -k 10 200 python -u tools/fuzz_gpu.py --mode kernel --seconds 90 --seed 41 --out $O/fuzz_s41.json > $O/fuzz_s41.log 2>&1 || { tail -20 $O/fuzz_s41.log; exit 1; }
tail -n 1 $O/fuzz_s41.log | cut -c1-400
step bench
for f in 2 1 0; do
  DP_FASTA_FORM=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_fasta_form$f.json 2> $O/bench_fasta_form$f.err || { tail -20 $O/bench_fasta_form$f.err; exit 1; }
done
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), d['verified_bit_exact'])
" $O/bench_fasta_form2.json $O/bench_fasta_form1.json $O/bench_fasta_form0.json
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
cat $O/size_sweep.log
step done
