# Round 3 end-of-session evidence of HEAD: GPU tests, fuzz campaigns, the three bench lines (FASTA with its
# cpu_baseline), the FASTA rocprofv3 trace + PMC passes and summary, the CSV PMC passes, the size sweep.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_final2}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step fuzz
timeout -k 10 150 python -u tools/fuzz_gpu.py --mode kernel --seconds 80 --seed 51 --out $O/fuzz_s51.json > $O/fuzz_s51.log 2>&1 || { tail -20 $O/fuzz_s51.log; exit 1; }
tail -n 1 $O/fuzz_s51.log | cut -c1-300
timeout -k 10 150 python -u tools/fuzz_gpu.py --mode object --seconds 80 --seed 52 --out $O/fuzz_obj_s52.json > $O/fuzz_obj_s52.log 2>&1 || { tail -20 $O/fuzz_obj_s52.log; exit 1; }
tail -n 1 $O/fuzz_obj_s52.log | cut -c1-300
step bench
timeout -k 10 300 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload csv --no-cpu-baseline > $O/bench_csv.json 2> $O/bench_csv.err || { tail -20 $O/bench_csv.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload vcf --no-cpu-baseline > $O/bench_vcf.json 2> $O/bench_vcf.err || { tail -20 $O/bench_vcf.err; exit 1; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), r.get('frac_of_mixed_ref'), d['verified_bit_exact'], (d.get('cpu_baseline') or {}).get('value'))
" $O/bench_fasta.json $O/bench_csv.json $O/bench_vcf.json
step profile-fasta
bash tools/profile.sh r3f_fasta || { cat gpurun_out/prof_r3f_fasta/status.txt; exit 1; }
cat gpurun_out/prof_r3f_fasta/status.txt
python3 tools/pmc_summary.py gpurun_out/prof_r3f_fasta $O/fasta --kernel "map_kernel<0>,fasta_place_kernel" --alg-bytes 4311612400 --object-bytes 4294967296 > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg' $O/fasta/pmc_summary.json
step profile-csv
bash tools/profile.sh r3f_csv --workload csv --steps 3 --warmup 1 --no-cpu-baseline --no-verify || { cat gpurun_out/prof_r3f_csv/status.txt; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof_r3f_csv $O/csv --kernel "scan_kernel<1, 2>" --alg-bytes 36290686630 --object-bytes 34359738368 --index-dtype u16b > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg' $O/csv/pmc_summary.json
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
grep fixed_us $O/size_sweep.log
step done
