"""One line per leg of a bench.py JSON line: value, span, roofline fractions, verification, cpu baseline."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        d = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
    legs = [("fasta", d)] + [(k, d[k]) for k in ("fasta", "csv", "vcf") if isinstance(d.get(k), dict)]
    for name, x in legs:
        if "error" in x:
            print(f"{path} {name}: ERROR {x['error']}")
            continue
        r = x["roofline"]
        cpu = x.get("cpu_baseline") or {}
        print(f"{path} {name}: value {x['value']} {x['unit']}, {x['ms_per_step']} ms/step, span {r['kernel_avg_us']} us, "
              f"frac {r['frac']}, of read ceiling {r.get('frac_of_measured_peak')}, of mixed ref "
              f"{r.get('frac_of_mixed_ref')}, traffic {r.get('traffic')} ({r.get('traffic_source')}), verified "
              f"{x.get('verified_bit_exact', x.get('verified_every_offset'))}, cpu {cpu.get('value')} on "
              f"{cpu.get('cores')} cores, leg {x.get('leg_s')} s")
    print(f"{path}: wall {d.get('bench_wall_s')} s, peak RSS {d.get('peak_rss_gib')} GiB")
