#!/bin/bash
# Round-4 evidence pass (on the GPU box): size sweeps, rocprofv3 trace + PMC of each bench leg, the bench line.
#   bash tools/r4_evidence.sh <tag>      -> gpurun_out/<tag>/ (copy into profiles/r04/)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-r4_ev}; O=gpurun_out/$T; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step size_sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.125,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -5 $O/size_sweep.log; exit 1; }
tail -3 $O/size_sweep.log
step delim_sweep
timeout -k 10 400 python -u tools/delim_sweep.py --forms default,line,onepass,twokernel --content csv,vcf,fasta --sizes-gib 0.0625,0.25,1,2,4 --reps 10 > $O/delim_sweep.log 2>&1 || { tail -5 $O/delim_sweep.log; exit 1; }
grep form $O/delim_sweep.log
for leg in fasta csv vcf; do
  step prof_$leg
  timeout -k 10 500 bash tools/r4_prof.sh $leg $O/$leg > $O/prof_$leg.log 2>&1 || { tail -20 $O/prof_$leg.log; exit 1; }
  tail -4 $O/prof_$leg.log
done
step bench
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 tools/bench_summary.py $O/bench.json
step done
