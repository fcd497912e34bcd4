set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_v8; mkdir -p $O
bash tools/profile.sh r03_fasta || exit 1
( cd /tmp && export TMPDIR=/tmp && DP_DELIM_TWOPASS_MAX=17179869184 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/csv2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload csv --size 4294967296 --no-cpu-baseline --no-verify --steps 10 ) > $O/csv2.log 2>&1 || exit 1
python3 tools/rocpd_stats.py $(find $O/csv2 -name "*results.db" | head -1) > $O/csv2.stats; head -8 $O/csv2.stats
