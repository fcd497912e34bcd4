set -o pipefail
O=gpurun_out/r3_base
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -3 $O/gpu_tests.log &&
timeout -k 10 240 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err &&
cat $O/bench_fasta.json &&
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.5,1,2,4,8 > $O/size_sweep.log 2>&1 &&
cat $O/size_sweep.log
