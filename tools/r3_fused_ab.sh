# Round 3: where the fused FASTA form spends its time.  Same box: the span of the fused build, its A/B
# variants (static first groups, no acquire fence) and the two-kernel form, alternated over rounds; then the
# profiling build's placement timeline for the fused and the two-kernel forms at 4 GiB and 512 MiB.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_fused_ab}; mkdir -p $O
L=dataplug_amd/lib
for round in 1 2; do
  for v in fused twokernel static nofence; do
    case $v in fused) lib=$L/libdpscan.so; e="DP_FASTA_FORM=2";; twokernel) lib=$L/libdpscan.so; e="DP_FASTA_FORM=1";;
      *) lib=$L/libdpscan_v_$v.so; e="DP_FASTA_FORM=2";; esac
    echo -n "$round $v "
    env DPSCAN_LIB=$lib $e timeout -k 10 120 python -u tools/probe_fasta2.py --reps 20 > $O/${v}_$round.json 2>&1 || { tail -5 $O/${v}_$round.json; exit 1; }
    grep -o '"span_us": [0-9.]*' $O/${v}_$round.json
  done
done
for sz in 4294967296 536870912; do
  for f in 2 1; do
    DP_FASTA_FORM=$f DPSCAN_LIB=$L/libdpscan_v_prof2.so timeout -k 10 120 python -u tools/place_timeline.py --size $sz > $O/tl_form${f}_$sz.json 2>&1 || { tail -5 $O/tl_form${f}_$sz.json; exit 1; }
    echo "form $f size $sz"; cat $O/tl_form${f}_$sz.json
  done
done
