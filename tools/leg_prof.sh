#!/bin/bash
# rocprofv3 evidence for one bench leg (on the GPU box):  bash tools/leg_prof.sh <leg> <out dir> [tag]
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in passes of their own (tools/profile.sh), of the same
# command as the bench leg (one leg per run), summarised per launch by tools/pmc_summary.py.  The newline legs'
# kernel is the one the auto form picks for their stored form (u8s, out_mode 4: line_kernel<3> at every size);
# INDEX_DTYPE / DELIM_KERNEL / ALG_CSV / ALG_VCF override the form, the kernel name and the algorithmic bytes.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
LEG=${1:?leg}; DST=${2:?dst}; TAG=${3:-$LEG}
case $LEG in
  fasta) K="map_kernel,fasta_place_kernel<0>"; ALG=4311612400; OBJ=4294967296; IDX="";;
  csv)   K="${DELIM_KERNEL:-line_kernel<3>}"; ALG=${ALG_CSV:-35595745107}; OBJ=34359738368; IDX="--index-dtype ${INDEX_DTYPE:-u8s}";;
  vcf)   K="${DELIM_KERNEL:-line_kernel<3>}"; ALG=${ALG_VCF:-70123839442}; OBJ=68719476254; IDX="--index-dtype ${INDEX_DTYPE:-u8s}";;
esac
bash tools/profile.sh $TAG --workload $LEG --legs $LEG --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-e2e $IDX || { cat gpurun_out/prof_$TAG/status.txt; tail -20 gpurun_out/prof_$TAG/*.log; exit 1; }
cat gpurun_out/prof_$TAG/status.txt
python3 tools/pmc_summary.py gpurun_out/prof_$TAG $DST --kernel "$K" --alg-bytes $ALG --object-bytes $OBJ $IDX > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg|SQ_WAVES"' $DST/pmc_summary.json
