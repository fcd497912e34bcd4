# line_kernel variants, same box: correctness of the shipped build, then the sweep per variant (alternated)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r4_line_ab}; mkdir -p $O
DP_DELIM_FORM=line timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUNDS=${ROUNDS:-2} VARIANTS="${VARIANTS:-base early0 noplace}" LIMIT=200 bash tools/gpu_ab.sh ${1:-r4_line_ab}/ab python -u tools/delim_sweep.py --forms line,onepass --content ${CONTENT:-csv,fasta} --sizes-gib ${SIZES:-1,4} --reps 10 --no-check || exit 1
for f in $O/ab/*.out; do echo "$f: $(grep -o '"content": "[a-z]*", "size_gib": [0-9.]*, "line_us": [0-9.]*\|"onepass_us": [0-9.]*' $f | tr '\n' ' ')"; done
