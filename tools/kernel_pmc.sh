#!/bin/bash
# SQ counters of every kernel a short command launches (on the GPU box), two passes of 8 SQ counters each plus a
# kernel trace, summarised per kernel by tools/kernel_pmc.py:
#     bash tools/kernel_pmc.sh <tag> <python script args...>
# e.g.  bash tools/kernel_pmc.sh sparse2g tools/size_sweep.py --sizes-gib 2 --reps 5
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:?tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/kpmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  local pmc=$1; shift
  timeout -k 10 240 rocprofv3 $pmc -d "$OUT/$name" -o "$name" --output-format csv -- python3 "$ROOT/$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$OUT/status.txt"; return $rc
}
pass trace "--kernel-trace --stats" "$@" &&
pass sqa "--pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" "$@" &&
pass sqb "--pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA" "$@" &&
python3 "$ROOT/tools/kernel_pmc.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
