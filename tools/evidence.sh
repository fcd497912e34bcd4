#!/bin/bash
# Evidence pass (on the GPU box): size sweep, newline form sweep, rocprofv3 trace + PMC of each bench leg, the bench
# line.   bash tools/evidence.sh <tag> [legs]      -> gpurun_out/<tag>/ (copy into profiles/rNN/)
# (NO_SWEEPS / NO_FORM_SWEEP / NO_BENCH skip those steps)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-ev}; O=gpurun_out/$T; mkdir -p $O
LEGS=${2:-fasta csv vcf}
step() { echo "== $1 $(date +%T)"; }
if [ -z "$NO_SWEEPS" ]; then
  step size_sweep
  timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.125,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -5 $O/size_sweep.log; exit 1; }
  tail -3 $O/size_sweep.log
  if [ -z "$NO_FORM_SWEEP" ]; then
    step form_sweep
    timeout -k 10 900 python -u tools/form_sweep.py --content vcf,csv --sizes-gib 2,4,8,16,32,64 --reps 6 --forms line:4,default:4,one:3,line:3 > $O/form_sweep.log 2>&1 || { tail -5 $O/form_sweep.log; exit 1; }
    python3 tools/sweep_table.py $O/form_sweep.log > $O/form_sweep_table.txt
  fi
fi
for leg in $LEGS; do
  step prof_$leg
  timeout -k 10 500 bash tools/leg_prof.sh $leg $O/$leg ${T}_$leg > $O/prof_$leg.log 2>&1 || { tail -20 $O/prof_$leg.log; exit 1; }
  tail -4 $O/prof_$leg.log
done
if [ -z "$NO_BENCH" ]; then
  step bench
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  python3 tools/bench_summary.py $O/bench.json
fi
step done
