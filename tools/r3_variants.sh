#!/bin/bash
# Same-box A/B of FASTA launch variants under rocprofv3 (per-kernel split): bash tools/r3_variants.sh tag v1 v2 ...
# ("base" = the shipped build; "onepass" = base with DP_FASTA_ONEPASS=1; "countonly" = base, placement stores off)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
for n in "$@"; do
  L=$ROOT/dataplug_amd/lib/libdpscan_v_$n.so; E=""
  case $n in base|onepass|countonly) ;; *) [ -f $L ] || { echo "$n: no library (refused by the ISA guard?)"; exit 1; };; esac
  case $n in base) L=$ROOT/dataplug_amd/lib/libdpscan.so;; onepass) L=$ROOT/dataplug_amd/lib/libdpscan.so; E="DP_FASTA_ONEPASS=1";;
    countonly) L=$ROOT/dataplug_amd/lib/libdpscan.so; E="DP_PROBE_PLACE_COUNT_ONLY=1";; esac
  ( cd /tmp && export TMPDIR=/tmp && env DPSCAN_LIB=$L $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/$n -o run -- python3 $ROOT/tools/probe_fasta2.py ) > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
  grep '"span_us"' $O/$n.log
  python3 tools/rocpd_stats.py $(find $O/$n -name "*results.db" | head -1) > $O/$n.stats; head -6 $O/$n.stats || true
done
