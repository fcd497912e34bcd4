#!/bin/bash
# rocprofv3 evidence for one bench leg (on the GPU box):  bash tools/r4_prof.sh <leg> <out dir under profiles/>
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in passes of their own (tools/profile.sh), of the same
# command as the bench leg (one leg per run), summarised per launch by tools/pmc_summary.py.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
LEG=${1:?leg}; DST=${2:?dst}
case $LEG in
  fasta) K="map_kernel<0>,fasta_place_kernel<0>"; ALG=4311612400; OBJ=4294967296; IDX="";;
  csv)   K="${DELIM_KERNEL:-line_kernel<1, 2>}"; ALG=36290686630; OBJ=34359738368; IDX="--index-dtype u16b";;   # CSV-dense: line_kernel
  vcf)   K="${DELIM_KERNEL:-scan_kernel<1, 2>}"; ALG=70446072202; OBJ=68719476254; IDX="--index-dtype u16b";;   # one-pass above 2 GiB
esac
bash tools/profile.sh r4_$LEG --workload $LEG --legs $LEG --steps 5 --warmup 2 --no-cpu-baseline --no-verify || { cat gpurun_out/prof_r4_$LEG/status.txt; tail -20 gpurun_out/prof_r4_$LEG/*.log; exit 1; }
cat gpurun_out/prof_r4_$LEG/status.txt
python3 tools/pmc_summary.py gpurun_out/prof_r4_$LEG $DST --kernel "$K" --alg-bytes $ALG --object-bytes $OBJ $IDX > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg|SQ_WAVES"' $DST/pmc_summary.json
