# Round 3 final tree: rocprofv3 trace + PMC passes of the FASTA bench command, summarised per launch
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_prof_fasta}; mkdir -p $O
bash tools/profile.sh r3f2_fasta || { cat gpurun_out/prof_r3f2_fasta/status.txt; exit 1; }
cat gpurun_out/prof_r3f2_fasta/status.txt
python3 tools/pmc_summary.py gpurun_out/prof_r3f2_fasta $O/fasta --kernel "map_kernel<0>,fasta_place_kernel" --alg-bytes 4311612400 --object-bytes 4294967296 > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg' $O/fasta/pmc_summary.json
cut -c1-220 $O/fasta/kernel_stats.csv
grep -o '"kernel_avg_us": [0-9.]*' $O/fasta/bench_under_rocprof.log || true
