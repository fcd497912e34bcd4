#!/bin/bash
# Instruction-cache counters of the FASTA scan (one rocprofv3 --pmc pass per counter group).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_icache${1:-}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="python3 $ROOT/tools/probe_perf.py --no-stream --only fasta --reps 5"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/p1 -o p1 --output-format csv -- $P > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ -d $OUT/p2 -o p2 --output-format csv -- $P > $OUT/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $OUT/p3 -o p3 --output-format csv -- $P > $OUT/p3.log 2>&1
