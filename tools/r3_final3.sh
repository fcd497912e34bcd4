# Round 3 final tree: GPU tests, smoke, the three bench lines (FASTA with its cpu_baseline, every launch verified).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_final3}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench
timeout -k 10 300 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload csv --no-cpu-baseline > $O/bench_csv.json 2> $O/bench_csv.err || { tail -20 $O/bench_csv.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload vcf --no-cpu-baseline > $O/bench_vcf.json 2> $O/bench_vcf.err || { tail -20 $O/bench_vcf.err; exit 1; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), r.get('frac_of_mixed_ref'), d['verified_bit_exact'], (d.get('cpu_baseline') or {}).get('value'), r.get('traffic'))
" $O/bench_fasta.json $O/bench_csv.json $O/bench_vcf.json
step done
