#!/bin/bash
# Same-box A/B runner for libdpscan variants (replaces round 3's one-off r3_*.sh scripts; on the GPU box).
#
#   VARIANTS="base v1 v2" ROUNDS=3 bash tools/gpu_ab.sh <tag> <command...>
#
# Variants are tools/build_variants.py names ("base" = the shipped dataplug_amd/lib/libdpscan.so); every round
# runs the command once per variant, alternated, with DPSCAN_LIB pointing at the variant, under its own time
# limit.  Output: gpurun_out/<tag>/<variant>_<round>.out (stdout+stderr) and a summary line per run with the
# numbers the probes print (span_us / value / frac / bit_exact / verified*).  A failing run ends the script.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:?tag}; shift
[ $# -gt 0 ] || { echo "usage: VARIANTS=... bash tools/gpu_ab.sh <tag> <command...>"; exit 2; }
O=gpurun_out/$TAG; mkdir -p $O
L=dataplug_amd/lib
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-base}; do
    case $v in base) lib=$L/libdpscan.so;; *) lib=$L/libdpscan_v_$v.so;; esac
    [ -f $lib ] || { echo "$v: no library (refused by the ISA guard?)"; continue; }
    f=$O/${v}_$round.out
    env DPSCAN_LIB=$lib timeout -k 10 ${LIMIT:-180} "$@" > $f 2>&1 || { echo "$v round $round failed"; tail -8 $f; exit 1; }
    echo "$round $v $(grep -oE '"(span_us|value|frac|kernel_avg_us|bit_exact|verified[a-z_]*)": [0-9.a-z]+' $f | head -8 | tr '\n' ' ')" | tee -a $O/summary.txt
  done
done
