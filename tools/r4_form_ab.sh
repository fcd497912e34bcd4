#!/bin/bash
# Newline bench legs (configs[2] 32 GiB CSV, configs[3] 64 GiB VCF) with each newline kernel form, alternated on one
# box:  ROUNDS=2 FORMS="hybrid line one" bash tools/r4_form_ab.sh <tag>
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r4_form}; mkdir -p $O
for round in $(seq 1 ${ROUNDS:-2}); do
  for f in ${FORMS:-hybrid line one}; do
    DP_DELIM_FORM=$f timeout -k 10 300 python3 -u bench.py --workload csv --legs csv,vcf --no-cpu-baseline > $O/${f}_$round.json 2> $O/${f}_$round.err || { tail -20 $O/${f}_$round.err; exit 1; }
    python3 - "$O/${f}_$round.json" "$f" "$round" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
legs = [d] if "roofline" in d and d.get("config", {}).get("workload", "").startswith("'") else []
for k in ("csv", "vcf"):
    if isinstance(d.get(k), dict):
        legs.append(d[k])
print(sys.argv[3], sys.argv[2], " ".join(f"{x['metric'].split(',')[-1].strip()}: {x['roofline']['kernel_avg_us']} us frac {x['roofline']['frac']} ({x['roofline']['kernel'][:24]})" for x in legs if "roofline" in x))
PY
  done
done
