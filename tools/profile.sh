#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box):  bash tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats   2) FETCH_SIZE   3) WRITE_SIZE   4) SQ instruction / stall counters
# Counters in their own passes (never combined with sys/runtime traces).  Summaries land in
# gpurun_out/prof_<tag>/ ; copy the ones to keep into profiles/.
set -u
TAG=${1:-run}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${@:-"--steps 10 --warmup 2 --no-cpu-baseline --no-verify"}
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  return $rc
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY
echo "done" >> "$OUT/status.txt"
