#!/bin/bash
# One GPU verification pass: the GPU tests, the default bench, CSV/VCF bench lines, the multi-worker
# rehearsals on one GPU (threads, then two torchrun ranks sharing the device).
set -o pipefail
O=gpurun_out/${1:-run}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -3 $O/gpu_tests.log &&
timeout -k 10 240 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err &&
cat $O/bench_fasta.json &&
timeout -k 10 240 python -u bench.py --workload csv --no-cpu-baseline > $O/bench_csv.json 2> $O/bench_csv.err &&
cat $O/bench_csv.json &&
timeout -k 10 300 python -u bench.py --workload vcf --no-cpu-baseline > $O/bench_vcf.json 2> $O/bench_vcf.err &&
cat $O/bench_vcf.json &&
timeout -k 10 240 python -u bench.py --gpus 4 --devices 0,0,0,0 --no-cpu-baseline --no-strong > $O/bench_t4.json 2> $O/bench_t4.err &&
cat $O/bench_t4.json &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --devices 0,0 --no-cpu-baseline --no-strong > $O/bench_tr2.json 2> $O/bench_tr2.err &&
cat $O/bench_tr2.json
