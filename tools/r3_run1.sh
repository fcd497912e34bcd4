# Round 3: one group per claim (DP_MAP_RUN=1) shipped: GPU tests, bench line, size sweep, placement timeline.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_run1}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step bench
timeout -k 10 300 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), d['verified_bit_exact'], (d.get('cpu_baseline') or {}).get('value'))
" $O/bench_fasta.json
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.125,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
grep -E 'fixed_us|"size_gib": (0.5|1.0|4.0),' $O/size_sweep.log | cut -c1-200
step timeline
DPSCAN_LIB=dataplug_amd/lib/libdpscan_v_prof2.so timeout -k 10 120 python -u tools/place_timeline.py > $O/tl.json 2>&1 || { tail -5 $O/tl.json; exit 1; }
cut -c1-300 $O/tl.json
step done
