# Round 3: FASTA placement blocks in ticket order (shipped) vs blockIdx order (no claim atomic), same box
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_placeticket_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2 3; do
  for v in base blkidx; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    echo -n "$round $v "
    env DPSCAN_LIB=$lib timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*\|"bit_exact": [a-z]*' $O/${v}_$round.json | tr '\n' ' '; echo
  done
done
for v in prof2 prof2blkidx; do
  DPSCAN_LIB=$L/libdpscan_v_$v.so timeout -k 10 120 python -u tools/place_timeline.py > $O/tl_$v.json 2>&1 || { tail -5 $O/tl_$v.json; exit 1; }
  echo $v; python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in ('map_last_wave_end','start','prefix','end')})" $O/tl_$v.json
done
