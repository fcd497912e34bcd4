#!/bin/bash
# One GPU verification pass (on the GPU box):  bash tools/gpu_round.sh <tag> [quick]
# the GPU tests, smoke, the driver's bench command (FASTA headline + CSV / VCF legs in one line), and the
# multi-worker rehearsal on one GPU (threads).  Every step under its own time limit; the first failure ends it.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-run}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ "${2:-}" != quick ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  step smoke
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
step bench
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }

python3 tools/bench_summary.py $O/bench.json
step done
