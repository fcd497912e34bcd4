set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_v7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 && tail -3 $O/size_sweep.log || exit 1
for w in csv vcf; do for sz in 4 16; do
  timeout -k 10 300 python -u bench.py --workload $w --size $((sz<<30)) --no-cpu-baseline --steps 10 > $O/${w}_${sz}g_two.json 2>/dev/null || exit 1
  DP_DELIM_TWOPASS_MAX=0 timeout -k 10 300 python -u bench.py --workload $w --size $((sz<<30)) --no-cpu-baseline --steps 10 > $O/${w}_${sz}g_one.json 2>/dev/null || exit 1
  python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], r['kernel_avg_us'], r['frac'], r.get('frac_of_mixed_peak'), d['verified_bit_exact'], r['kernel'][:30])
" $O/${w}_${sz}g_two.json $O/${w}_${sz}g_one.json
done; done
