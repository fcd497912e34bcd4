"""One row per (content, size) of a tools/form_sweep.py log: each form's median span and roofline fraction, the
stream kernel's rate, each auto form's pick and how far it is from the best fixed form (of any out_mode)."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "size_gib" not in d:
            continue
        forms = [k[:-3] for k in d if k.endswith("_us") and k != "stream_us" and not k.endswith("_all_us")]
        med = {k: d[k + "_us"]["median"] for k in forms}
        best = min(v for k, v in med.items() if not k.startswith("default"))
        row = f"{d['content']} {d['size_gib']:>5g} GiB  stream {d.get('stream_TBps_median', 0):.2f} TB/s  " + "  ".join(
            f"{k} {med[k]:9.1f} us {d[k + '_frac_median']:.3f}" for k in forms)
        for k in forms:
            if k.startswith("default"):
                row += f"  {k} picked {d.get(k + '_forms')}  {k}/best {med[k] / best:.3f}"
        print(row + ("" if d["equal"] else "  MISMATCH"))
