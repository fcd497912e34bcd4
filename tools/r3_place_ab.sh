# Round 3: FASTA placement with four prefetched spill words, and the map kernel's structural ceiling (noscan:
# loads, barriers, claims and stores without the row scan; wrong results) next to the stream kernel, same box.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_place_ab}; mkdir -p $O
L=dataplug_amd/lib
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/scan_tests.log 2>&1 || { tail -30 $O/scan_tests.log; exit 1; }
tail -1 $O/scan_tests.log
step probe
for round in 1 2; do
  for v in base noscan; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    echo -n "$round $v "
    env DPSCAN_LIB=$lib timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 --no-verify > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*' $O/${v}_$round.json
  done
done
step timeline
for sz in 4294967296 536870912; do
  DPSCAN_LIB=$L/libdpscan_v_prof2.so timeout -k 10 120 python -u tools/place_timeline.py --size $sz > $O/tl_$sz.json 2>&1 || { tail -5 $O/tl_$sz.json; exit 1; }
  cat $O/tl_$sz.json
done
step bench
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_fasta.json 2> $O/bench_fasta.err || { tail -20 $O/bench_fasta.err; exit 1; }
python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('frac_of_measured_peak'), d['verified_bit_exact'])
" $O/bench_fasta.json
step done
