#!/bin/bash
# Round 3: the two-kernel FASTA index vs the one-pass kernel (DP_FASTA_ONEPASS=1), same box.
set -o pipefail
O=gpurun_out/${1:-r3_ab}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 ; echo "pytest rc=$?" >> $O/gpu_tests.log
tail -3 $O/gpu_tests.log
grep -q "pytest rc=0" $O/gpu_tests.log || exit 1
timeout -k 10 240 python -u bench.py > $O/bench_fasta.json 2> $O/bench_fasta.err && cat $O/bench_fasta.json &&
DP_FASTA_ONEPASS=1 timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/bench_fasta_onepass.json 2> $O/bench_fasta_onepass.err && cat $O/bench_fasta_onepass.json &&
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.5,1,2,4,8 > $O/size_sweep.log 2>&1 && cat $O/size_sweep.log &&
DP_FASTA_ONEPASS=1 timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.5,1,2,4,8 > $O/size_sweep_onepass.log 2>&1 && cat $O/size_sweep_onepass.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-verify > $O/bench_prof.json 2> $O/bench_prof.err && echo prof ok
