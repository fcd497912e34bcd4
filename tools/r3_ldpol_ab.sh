# Round 3: input load cache policy A/B (nt shipped vs plain, sc1, sc1 nt), same box, alternated
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_knob_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2 3; do
  for v in base ldplain ldsc1 ldntsc1; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    [ -f $lib ] || { echo "$v: no library"; continue; }
    echo -n "$round $v "
    env DPSCAN_LIB=$lib timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*\|"bit_exact": [a-z]*' $O/${v}_$round.json | tr '\n' ' '; echo
  done
done
