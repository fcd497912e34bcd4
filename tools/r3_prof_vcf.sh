# Round 3: rocprofv3 trace + PMC passes of the VCF bench line (64 GiB, one-pass newline kernel, uint16 + blocks)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_prof_vcf}; mkdir -p $O
bash tools/profile.sh r3f_vcf --workload vcf --steps 3 --warmup 1 --no-cpu-baseline --no-verify || { cat gpurun_out/prof_r3f_vcf/status.txt; exit 1; }
cat gpurun_out/prof_r3f_vcf/status.txt
python3 tools/pmc_summary.py gpurun_out/prof_r3f_vcf $O/vcf --kernel "scan_kernel<1, 2>" --alg-bytes 70446072202 --object-bytes 68719476254 --index-dtype u16b > /dev/null || exit 1
grep -E '"hbm_traffic_bytes"|traffic_over_alg|SQ_WAVES"' $O/vcf/pmc_summary.json
