# Round 3: newline placement blocks in ticket order (shipped) vs blockIdx order, both forms swept (same box)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_dplace_ab}; mkdir -p $O
for v in base dblkidx; do
  case $v in base) lib=dataplug_amd/lib/libdpscan.so;; *) lib=dataplug_amd/lib/libdpscan_v_$v.so;; esac
  env DPSCAN_LIB=$lib timeout -k 10 300 python -u tools/delim_sweep.py --content csv,vcf --sizes-gib 0.0625,0.25,0.5,1,2 > $O/sweep_$v.log 2>&1 || { tail -5 $O/sweep_$v.log; exit 1; }
  echo "== $v"; grep -v fixed $O/sweep_$v.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['content'], d['size_gib'], d['onepass_us'], d['twokernel_us'])"
done
