# Round 3: one-pass newline kernel claim runs A/B on the CSV / VCF bench lines (same box, alternated):
# shipped (2 units per claim while dense, 4 while sparse) vs 1 while dense, 1 / 2, and 2 / 2.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_claimdelim_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2; do
  for w in csv vcf; do
    for v in base cd1 cd1s2 cs2; do
      case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
      env DPSCAN_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline --no-verify --no-strong > $O/${w}_${v}_$round.json 2> $O/${w}_${v}_$round.err || { tail -5 $O/${w}_${v}_$round.err; exit 1; }
      python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); r=d['roofline']
print(sys.argv[2], d['value'], r['kernel_avg_us'], r['frac'], r.get('frac_of_mixed_ref'))" $O/${w}_${v}_$round.json "$round $w $v"
    done
  done
done
