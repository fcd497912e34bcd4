#!/bin/bash
# Same-box A/B of FASTA form variants (tools/build_variants.py), kernel-event GB/s over 4 GiB.
mkdir -p gpurun_out && rm -f gpurun_out/spill_ab2.log
for r in 1 2; do for n in "$@"; do
  f=1; L=dataplug_amd/lib/libdpscan_v_$n.so
  [ "$n" = base ] && L=dataplug_amd/lib/libdpscan.so
  [ "$n" = onepass ] && { L=dataplug_amd/lib/libdpscan.so; f=0; }
  DP_FASTA_SPILL=$f DPSCAN_LIB=$L timeout -k 10 120 python tools/probe_perf.py --no-stream --reps 20 --only fasta > gpurun_out/pp.txt 2>&1 || { tail -3 gpurun_out/pp.txt; exit 1; }
  echo "$n $(tail -1 gpurun_out/pp.txt)" >> gpurun_out/spill_ab2.log
done; done
cat gpurun_out/spill_ab2.log
