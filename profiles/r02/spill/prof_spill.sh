#!/bin/bash
# FASTA two-pass form: per-kernel durations (rocprofv3 kernel trace) and a size sweep of both forms.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_spill && rm -rf gpurun_out/prof_spill/*
DP_FASTA_SPILL=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_spill -o run -- python3 tools/probe_perf.py --no-stream --reps 10 --only fasta > gpurun_out/prof_spill/out.txt 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find gpurun_out/prof_spill -name '*.db' | head -1) > gpurun_out/prof_spill/stats.txt
cat gpurun_out/prof_spill/stats.txt
for f in 1 0; do
  DP_FASTA_SPILL=$f timeout -k 10 180 python3 tools/size_sweep.py --sizes-gib 1,2,4,8 --reps 6 > gpurun_out/prof_spill/sweep_$f.txt 2>&1 || exit 1
  echo "spill=$f"; grep -E 'fixed|size' gpurun_out/prof_spill/sweep_$f.txt
done
