#!/bin/bash
# Same-box comparison of perf-probe variants (built by tools/build_variants.py): run on the GPU box.
#   bash tools/cmp_variants.sh name1 name2 ...      (names of dataplug_amd/lib/libdpscan_v_<name>.so; "base" = default)
mkdir -p gpurun_out && rm -f gpurun_out/cmp.log
for r in 1 2; do
for n in "$@"; do
  L=dataplug_amd/lib/libdpscan_v_$n.so; [ "$n" = base ] && L=dataplug_amd/lib/libdpscan.so
  DPSCAN_LIB=$L timeout -k 10 120 python tools/probe_perf.py --no-stream --reps 8 | tail -1 >> gpurun_out/cmp.log || exit 1
done; done
cat gpurun_out/cmp.log
