"""One line per leg of a bench.py JSON line: value, span, roofline fractions, verification, cpu baseline."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        d = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
    # the headline's leg from its own metric / workload (bench.py --workload fasta|csv|vcf), the sub-legs by key
    text = (d.get("metric", "") + " " + str((d.get("config") or {}).get("workload", ""))).lower()
    head = next((k for k in ("fasta", "csv", "vcf") if k in d.get("metric", "").lower()), None) or \
        next((k for k in ("fasta", "csv", "vcf") if k in text), "headline")
    legs = [(head, d)] + [(k, d[k]) for k in ("fasta", "csv", "vcf") if k != head and isinstance(d.get(k), dict)]
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
    e2e, fq = d.get("e2e") or {}, d.get("fastq") or {}
    for kind in ("fasta", "csv"):
        x = e2e.get(kind) or {}
        if x:
            print(f"{path} e2e {kind}: memory {(x.get('memory') or {}).get('value')} GiB/s, loopback http "
                  f"{(x.get('loopback_http') or {}).get('value')} GiB/s, verified "
                  f"{(x.get('memory') or {}).get('verified')}/{(x.get('loopback_http') or {}).get('verified')}")
    if fq:
        print(f"{path} fastq: {fq.get('value')} {fq.get('unit')} inflated, verified {fq.get('verified_every_read_end')}, "
              f"fits_in_driver_run {fq.get('fits_in_driver_run')}")
    print(f"{path}: wall {d.get('bench_wall_s')} s, peak RSS {d.get('peak_rss_gib')} GiB")
