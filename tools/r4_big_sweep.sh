# line_kernel vs the one-pass kernel at large launch sizes (same box): CSV / VCF 4-32 GiB
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r4_big}; mkdir -p $O
ROUNDS=1 VARIANTS="${VARIANTS:-base slots6}" LIMIT=400 bash tools/gpu_ab.sh ${1:-r4_big}/ab python -u tools/delim_sweep.py --forms line,onepass --content ${CONTENT:-csv,vcf} --sizes-gib ${SIZES:-4,8,16,32} --reps 5 || exit 1
for f in $O/ab/*.out; do echo "$f: $(grep -o '"content": "[a-z]*", "size_gib": [0-9.]*, "line_us": [0-9.]*\|"onepass_us": [0-9.]*' $f | sed 's/"content": //; s/"size_gib": //; s/"line_us": /line /; s/"onepass_us": /one /' | tr '\n' ' ')"; done
