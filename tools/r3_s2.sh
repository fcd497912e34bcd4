# Round 3, session 2 status of HEAD: GPU tests, the three bench lines, the FASTA size sweep, the DELIM form sweep.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_s2}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step bench
timeout -k 10 300 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload csv --no-cpu-baseline > $O/bench_csv.json 2> $O/bench_csv.err || { tail -20 $O/bench_csv.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload vcf --no-cpu-baseline > $O/bench_vcf.json 2> $O/bench_vcf.err || { tail -20 $O/bench_vcf.err; exit 1; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), r.get('frac_of_mixed_ref'), d['verified_bit_exact'], (d.get('cpu_baseline') or {}).get('value'))
" $O/bench_fasta.json $O/bench_csv.json $O/bench_vcf.json
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
cat $O/size_sweep.log
step delim-sweep
timeout -k 10 400 python -u tools/delim_sweep.py > $O/delim_sweep.log 2>&1 || { tail -20 $O/delim_sweep.log; exit 1; }
cat $O/delim_sweep.log
step done
