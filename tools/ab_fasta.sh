#!/bin/bash
# Same-box A/B of FASTA kernel variants (tools/build_variants.py names; "base" = the shipped build):
# kernel-event GB/s over the 4 GiB synthetic object, 3 rounds.  bash tools/ab_fasta.sh base v1 v2 ...
mkdir -p gpurun_out && rm -f gpurun_out/ab_fasta.log
for r in $(seq 1 ${ROUNDS:-3}); do for n in "$@"; do
  L=dataplug_amd/lib/libdpscan_v_$n.so; [ "$n" = base ] && L=dataplug_amd/lib/libdpscan.so
  DPSCAN_LIB=$L timeout -k 10 120 python tools/probe_perf.py --no-stream --reps 20 --only ${ONLY:-fasta} > gpurun_out/pp.txt 2>&1 || { tail -3 gpurun_out/pp.txt; exit 1; }
  echo "$n $(tail -1 gpurun_out/pp.txt)" >> gpurun_out/ab_fasta.log
done; done
cat gpurun_out/ab_fasta.log
