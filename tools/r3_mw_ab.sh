# Round 3: FASTA map kernel workgroup size A/B (same box): 16 waves x 1 per CU (shipped) vs 8 x 2 and 4 x 4.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_mw_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2 3; do
  for v in base mw8 mw4; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    echo -n "$round $v "
    env DPSCAN_LIB=$lib timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*\|"bit_exact": [a-z]*' $O/${v}_$round.json | tr '\n' ' '; echo
  done
done
