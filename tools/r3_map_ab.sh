# Round 3: FASTA map kernel load depth A/B (same box): the shipped 2 x 8 KiB buffers vs 4 x 4 KiB (three in
# flight while one is scanned), each with and without the row scan (noscan: timing only, wrong results).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_map_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2; do
  for v in base nbuf4 noscan nbuf4noscan; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    echo -n "$round $v "
    nv=""; case $v in *noscan) nv="--no-verify";; esac
    env DPSCAN_LIB=$lib timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 $nv > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*\|"bit_exact": [a-z]*' $O/${v}_$round.json | tr '\n' ' '; echo
  done
done
