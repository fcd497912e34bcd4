#!/bin/bash
# SQ instruction counters per KiB of input for perf-probe variants (run on the GPU box):
#   bash tools/pmc_variants.sh <workload: fasta|delim|nogt> name1 name2 ...   ("base" = default library)
# One rocprofv3 --pmc pass per variant (counters never combined with traces); results in gpurun_out/pmc_<name>/.
W=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  L=$ROOT/dataplug_amd/lib/libdpscan_v_$n.so; [ "$n" = base ] && L=$ROOT/dataplug_amd/lib/libdpscan.so
  DPSCAN_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
      -d $ROOT/gpurun_out/pmc_$n -o pmc --output-format csv -- python3 $ROOT/tools/probe_perf.py --no-stream --reps 5 --only $W \
      > $ROOT/gpurun_out/pmc_$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/pmc_$n" "$n" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "scan_kernel" in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
avg = {c: sum(d.values()) / len(d) for c, d in per.items()}
kib = 4 << 20
print(sys.argv[2], {c: round(v / kib, 2) for c, v in sorted(avg.items())})
PY
done
