"""Time-bounded randomized parity campaign on the GPU: the HIP scan kernels (through the C ABI) against the C
oracle (oracle/dpref.c) on random inputs, chunk plans, device misalignments and output forms.

    python tools/fuzz_gpu.py [--seconds 240] [--seed 1] [--mode kernel|object] [--out gpurun_out/fuzz.json]

``--mode object`` runs co.preprocess() end to end instead (see object_mode); ``--mode lines`` the CSV newline index
through co.preprocess() in its stored forms (see lines_mode).

FASTA: token soups and structured records (header lines 1 B - 300 KB, so headers span wave ranges, units and
chunks; '\\r'; '>' inside sequence lines; runs of '>' or '\\n'), object sizes log-uniform in [1 B, 48 MiB],
chunk plans of the reference (preprocess.py:38 floor plan with the tail dropped, including the
chunk_size == num_chunks - 1 quirk of handler.py:37 that sends every chunk to EOF), uint32 or uint64 output.
Every pair and every per-chunk count must equal the oracle's.  DELIM: random delimiter byte, [begin, end),
every_k 1-5, emit_add 0/1, uint64 or uint32 output; when every delimiter is an entry, sometimes the stored forms
(out_mode 4 u8s, 3 u16b) at a random object base, decoded.  Exits non-zero on the first mismatch and keeps the case
in gpurun_out/fuzz_fail.npz.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd.scan import ScanContext  # noqa: E402
from dataplug_amd.scan.objects import BlockedOffsets, ByteOffsets  # noqa: E402
from oracle import cpu_ref, dpref  # noqa: E402


def _save_fail(**case):
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed("gpurun_out/fuzz_fail.npz", **case)


def soup(rng, size):
    p_gt, p_nl, p_cr = rng.uniform(0, 0.3), rng.uniform(0, 0.3), rng.uniform(0, 0.02)
    p = np.array([p_gt, p_nl, p_cr, 1.0 - p_gt - p_nl - p_cr])
    p = np.clip(p, 0, None)
    p /= p.sum()
    cls = rng.choice(4, size=size, p=p)
    out = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)].copy()
    out[cls == 0] = 62
    out[cls == 1] = 10
    out[cls == 2] = 13
    return out


def records(rng, size):
    parts, total = [], 0
    hmax = int(rng.choice([40, 2000, 40000, 300000]))
    wmax = int(rng.choice([1, 60, 5000, 100000]))
    while total < size:
        h = b">" + b"h" * int(rng.integers(0, hmax)) + (b"\r" if rng.random() < 0.1 else b"") + b"\n"
        body_len = int(rng.integers(0, 4 * wmax + 1))
        w = max(1, int(rng.integers(1, wmax + 1)))
        body = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, body_len)].copy()
        if body_len and rng.random() < 0.2:                     # '>' inside sequence lines
            body[rng.integers(0, body_len, max(1, body_len // 500))] = 62
        lines = [body[i:i + w].tobytes() + b"\n" for i in range(0, body_len, w)]
        rec = h + b"".join(lines)
        parts.append(rec)
        total += len(rec)
    return np.frombuffer(b"".join(parts)[:size], np.uint8).copy()


def runs(rng, size):
    out = soup(rng, size)
    for _ in range(int(rng.integers(1, 6))):
        a = int(rng.integers(0, max(1, size)))
        b = min(size, a + int(rng.integers(1, 200000)))
        out[a:b] = rng.choice([62, 10])
    return out


def make_object(rng, max_size=48 << 20):
    size = int(math.exp(rng.uniform(0, math.log(max_size))))
    kind = rng.choice(["soup", "records", "runs"])
    a = {"soup": soup, "records": records, "runs": runs}[kind](rng, size)
    return a, str(kind)


def chunk_size(rng, size):
    if size < 2:
        return max(1, size)
    r = rng.random()
    if r < 0.1 and size <= (64 << 10):                           # the cs == num_chunks - 1 quirk (every chunk
        # reads to EOF: ~num_chunks x the headers, so small objects only)
        cs = int(math.isqrt(size))
        while cs > 1 and size // cs != cs + 1:
            cs -= 1
        if cs >= 1 and size // cs == cs + 1:
            return cs
    if r < 0.6:
        return max(1, math.ceil(size / int(rng.integers(1, 2000))))
    return int(rng.integers(1, size + 1))


def object_mode(args, rng):
    """co.preprocess() end to end through storage: random chunk plans (30 % the canonical 1-4 chunk plans)
    split into 1-9 byte-balanced groups on this GPU (dataplug_devices=[0]*g: the multi-GPU split, chunks cut
    at group boundaries and stitched, 64 KiB halos, header ends past a group's halo resolved from later
    bytes), sometimes a launch byte budget far below a group (passes), sometimes the per-chunk joblib route;
    the stored index against the oracle."""
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats.genomics.fasta import FASTA
    from dataplug_amd.storage import MemoryStore
    stats = {"object_cases": 0, "pairs": 0, "bytes": 0, "groups": {}, "budget_cases": 0, "joblib_cases": 0,
             "cut_cases": 0, "cuts": 0}
    t0 = last = time.time()
    i = 0
    while time.time() - t0 < args.seconds:
        size = int(math.exp(rng.uniform(math.log(64), math.log(getattr(args, "max_size", 12 << 20)))))
        a = records(rng, size) if rng.random() < 0.7 else runs(rng, size)
        cs = chunk_size(rng, size)
        if rng.random() < 0.3:                         # the reference's canonical few-chunk plans (fasta_example.py:23)
            cs = max(1, math.ceil(size / int(rng.integers(1, 5))))
        plan = cpu_ref.chunk_plan(size, cs)
        groups = int(rng.integers(1, 10))
        from dataplug_amd.scan.objects import fasta_split
        ncut = sum(not p.first for p in fasta_split(plan, groups, size)[0]) if plan else 0
        pc = {"dataplug_devices": [0] * groups}
        if rng.random() < 0.15:
            pc.update({"backend": "threading", "n_jobs": int(rng.integers(1, 5))})
            stats["joblib_cases"] += 1
        budget = None
        prev_budget = os.environ.get("DATAPLUG_AMD_MAX_LAUNCH_BYTES")
        if rng.random() < 0.25:
            budget = int(rng.integers(64 << 10, 4 << 20))
            os.environ["DATAPLUG_AMD_MAX_LAUNCH_BYTES"] = str(budget)
            stats["budget_cases"] += 1
        name = f"fz{i}"
        MemoryStore._named.pop(name, None)
        cfg = {"endpoint_url": f"memory://{name}"}
        co = CloudObject.from_s3(FASTA, f"s3://data/k{i}", fetch=False, s3_config=cfg)
        co.storage.create_bucket(Bucket="data")
        co.storage.put_object(Body=a.tobytes(), Bucket="data", Key=f"k{i}")
        co = CloudObject.from_s3(FASTA, f"s3://data/k{i}", s3_config=cfg)
        try:
            co.preprocess(chunk_size=cs, parallel_config=pc)
        finally:                                      # the caller's own setting (if any) back
            if prev_budget is None:
                os.environ.pop("DATAPLUG_AMD_MAX_LAUNCH_BYTES", None)
            else:
                os.environ["DATAPLUG_AMD_MAX_LAUNCH_BYTES"] = prev_budget
        got = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=co.meta_path.key)["Body"].read(),
                            np.uint32)
        exp = dpref.fasta_pairs(a, plan).reshape(-1).astype(np.uint32)
        MemoryStore._named.pop(name, None)
        if not np.array_equal(got, exp):
            _save_fail(data=a, chunk_size=cs, groups=groups,
                                budget=-1 if budget is None else budget)
            print(json.dumps({"FAIL": "object", "size": size, "chunk_size": cs, "groups": groups, "budget": budget,
                              "parallel_config": {k: v for k, v in pc.items() if k != "dataplug_devices"},
                              "got": int(len(got)), "expected": int(len(exp))}), flush=True)
            raise SystemExit(1)
        stats["object_cases"] += 1
        stats["pairs"] += len(exp) // 2
        stats["bytes"] += size
        stats["groups"][groups] = stats["groups"].get(groups, 0) + 1
        if ncut and "backend" not in pc:
            stats["cut_cases"] += 1
            stats["cuts"] += ncut
        i += 1
        if time.time() - last > 20:
            last = time.time()
            print(json.dumps({"t": round(last - t0), **{k: v for k, v in stats.items() if k != "groups"}}), flush=True)
    return stats


def csv_like(rng, size):
    """A CSV body that pandas reads: a 3-column header, then rows of 3 fields of random length (a field up to
    1 B - 200 KB, so rows span 256-byte and 64 KiB boundaries and wave ranges), some rows empty of text."""
    fmax = int(rng.choice([4, 40, 400, 20000, 200000]))
    parts, total = [b"a,b,c\n"], 6
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789 .", np.uint8)
    while total < size:
        fl = rng.integers(0, fmax + 1, 3)
        row = alpha[rng.integers(0, len(alpha), int(fl.sum()))].tobytes()
        row = row[:fl[0]] + b"," + row[fl[0]:fl[0] + fl[1]] + b"," + row[fl[0] + fl[1]:] + b"\n"
        parts.append(row)
        total += len(row)
    a = np.frombuffer(b"".join(parts), np.uint8)[:max(size, 6)].copy()
    return a


def lines_mode(args, rng):
    """The CSV newline index through co.preprocess() in a random stored form (u8s, u16b, u32p, u64, or auto: by the
    object's density), the object split into 1-9 parts on this GPU (dataplug_devices=[0]*g: each part its own launch,
    the tables merged on the host) or, for half the u8s / u16b / auto cases, stored as it is produced in pieces of
    64 KiB - 8 MiB (round 6), read back through LineIndex (preloaded or block by block) against the oracle's newline
    offsets."""
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats import _lines
    from dataplug_amd.formats.generic.csv import CSV
    from dataplug_amd.storage import MemoryStore
    stats = {"line_cases": 0, "lines": 0, "bytes": 0, "forms": {}, "groups": {}, "block_fetch_cases": 0}
    t0 = last = time.time()
    i = 0
    while time.time() - t0 < args.seconds:
        size = int(math.exp(rng.uniform(math.log(64), math.log(getattr(args, "max_size", 24 << 20)))))
        a = csv_like(rng, size)
        fmt = str(rng.choice(["u8s", "u8s", "u16b", "u32p", "u64", "auto", "auto"]))
        groups = int(rng.integers(1, 10))
        # (round 6) half the u8s / u16b / auto cases store the index as it is produced: pieces of 64 KiB - 8 MiB
        streamed = fmt not in ("u32p", "u64") and rng.random() < 0.5
        piece = int(math.exp(rng.uniform(math.log(64 << 10), math.log(8 << 20)))) if streamed else _lines.STREAM_PIECE
        _lines.index_object.__defaults__ = (0, "auto", piece)
        name = f"fl{i}"
        MemoryStore._named.pop(name, None)
        cfg = {"endpoint_url": f"memory://{name}"}
        co = CloudObject.from_s3(CSV, f"s3://data/k{i}.csv", fetch=False, s3_config=cfg)
        co.storage.create_bucket(Bucket="data")
        co.storage.put_object(Body=a.tobytes(), Bucket="data", Key=f"k{i}.csv")
        co = CloudObject.from_s3(CSV, f"s3://data/k{i}.csv", s3_config=cfg)
        co.preprocess(parallel_config={"dataplug_devices": [0] * groups}, extra_args={"index_format": fmt})
        preload = rng.random() < 0.5
        saved = _lines._PRELOAD_BYTES
        if not preload:
            _lines._PRELOAD_BYTES = 1024
            stats["block_fetch_cases"] += 1
        try:
            li = _lines.LineIndex.of(co)
            got = li._fetch(0, li.count) if li.count else np.zeros(0, np.uint64)
        finally:
            _lines._PRELOAD_BYTES = saved
        exp = dpref.delim(a, 0, len(a))[0]
        MemoryStore._named.pop(name, None)
        if fmt == "auto":
            from dataplug_amd.scan.objects import line_index_form
            fmt = line_index_form(co, 0, len(a))
        dtype_ok = getattr(co.attributes, "line_index_dtype", None) == (None if fmt == "u64" else fmt)
        stats["streamed_cases"] = stats.get("streamed_cases", 0) + int(streamed and len(a) > piece)
        if not dtype_ok or not np.array_equal(np.asarray(got, np.uint64), exp):
            _save_fail(data=a, groups=groups)
            print(json.dumps({"FAIL": "lines", "size": int(len(a)), "format": fmt, "groups": groups,
                              "got": int(len(got)), "expected": int(len(exp))}), flush=True)
            raise SystemExit(1)
        stats["line_cases"] += 1
        stats["lines"] += int(len(exp))
        stats["bytes"] += int(len(a))
        stats["forms"][fmt] = stats["forms"].get(fmt, 0) + 1
        stats["groups"][groups] = stats["groups"].get(groups, 0) + 1
        i += 1
        if time.time() - last > 20:
            last = time.time()
            print(json.dumps({"t": round(last - t0), **{k: v for k, v in stats.items() if k not in ("forms", "groups")}}),
                  flush=True)
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mode", choices=["kernel", "object", "lines"], default="kernel")
    ap.add_argument("--out", default="gpurun_out/fuzz.json")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    rng = np.random.default_rng(args.seed)
    if args.mode in ("object", "lines"):
        stats = (object_mode if args.mode == "object" else lines_mode)(args, rng)
        stats.update({"seconds": args.seconds, "seed": args.seed, "ok": True, "mode": args.mode})
        with open(args.out, "w") as f:
            json.dump(stats, f)
        print(json.dumps(stats), flush=True)
        return
    stats = kernel_mode(args, rng)
    stats["seconds"] = round(stats.pop("_t"), 1)
    stats["seed"] = args.seed
    stats["ok"] = True
    with open(args.out, "w") as f:
        json.dump(stats, f)
    print(json.dumps(stats), flush=True)


def kernel_mode(args, rng):
    """The kernels through the C ABI on random objects, chunk plans, misalignments and output forms."""
    ctx = ScanContext(0)
    stats = {"fasta_cases": 0, "fasta_pairs": 0, "quirk_cases": 0, "delim_cases": 0, "delim_offsets": 0,
             "bytes": 0, "kinds": {}, "delim_forms": {}, "stored_cases": 0}
    # the newline launch's kernels, drawn per case (dp_ctx_set_form): the default (line_kernel at these sizes), the
    # auto form's density probe at every size (line_max 0) with its threshold at random (either pick), or a form
    # pinned to line_kernel / the one-pass kernel
    delim_forms = [dict(delim=0, delim_line_max=4 << 30, delim_dense=20000),
                   dict(delim=0, delim_line_max=0, delim_dense=20000),
                   dict(delim=0, delim_line_max=0, delim_dense=0),
                   dict(delim=0, delim_line_max=0, delim_dense=1 << 40),
                   dict(delim=1, delim_line_max=4 << 30, delim_dense=20000),
                   dict(delim=3, delim_line_max=4 << 30, delim_dense=20000)]
    t0 = last = time.time()
    while time.time() - t0 < args.seconds:
        a, kind = make_object(rng, getattr(args, "max_size", 48 << 20))
        size = len(a)
        stats["bytes"] += size
        stats["kinds"][kind] = stats["kinds"].get(kind, 0) + 1
        off = int(rng.integers(0, 16))
        buf = ctx.workspace("fz_in", size + 64)
        if size:
            ctx.h2d(buf.ptr + off, a)
        # FASTA
        cs = chunk_size(rng, size)
        plan = cpu_ref.chunk_plan(size, cs) if size else []
        quirk = bool(plan) and cs == len(plan) - 1
        u64 = bool(rng.random() < 0.3)
        exp = dpref.fasta_pairs(a, plan) if plan else np.zeros((0, 2), np.uint64)
        if plan:
            pairs, pending, cend = ctx.fasta_index(buf.ptr + off, size, 0, size, plan, u64=u64)
            ok = (pending == -1).all() and np.array_equal(pairs.astype(np.uint64).reshape(-1, 2), exp)
            k = 0
            for i, (c0, c1) in enumerate(plan):
                k += len(dpref.fasta_pairs(a, [(c0, c1)]))
                ok = ok and int(cend[i]) == k
            if not ok:
                _save_fail(data=a, plan=np.asarray(plan, np.uint64),
                                    offset=off, u64=u64)
                print(json.dumps({"FAIL": "fasta", "size": size, "kind": kind, "chunk_size": cs, "offset": off,
                                  "u64": u64, "got": int(len(pairs)), "expected": int(len(exp))}), flush=True)
                raise SystemExit(1)
            stats["fasta_cases"] += 1
            stats["fasta_pairs"] += int(len(exp))
            stats["quirk_cases"] += int(quirk)
        # DELIM
        if size:
            b0 = int(rng.integers(0, size + 1))
            b1 = int(rng.integers(b0, size + 1))
            delim = int(rng.choice([10, 62, 13, 65, int(rng.integers(0, 256))]))
            k = int(rng.integers(1, 6))
            add = int(rng.integers(0, 2))
            du64 = bool(rng.random() < 0.7)
            ctx.set_form(**delim_forms[int(rng.integers(0, len(delim_forms)))])
            stored = k == 1 and add == 0 and b1 > b0 and rng.random() < 0.4
            if stored:                                # u8s / u16b at object base `off` (congruent to the address)
                mode = int(rng.choice([3, 4]))
                r = ctx.delim_ranges(buf.ptr + off, size, off, [(b0 + off, b1 + off)], delim=delim, out_mode=mode)
                f0 = b0 + off
                o = ByteOffsets(r[0], r[4], r[3], f0 >> 8, f0 >> 16) if mode == 4 else BlockedOffsets(r[0], r[3], f0 >> 16)
                got, nd = o.to_u64() - np.uint64(off), r[1]
                stats["stored_cases"] += 1
            else:
                got, nd = ctx.delim_index(buf.ptr + off, size, 0, b0, b1, delim, k, add, u64=du64)
            if b1 > b0:
                f = str(ctx.last_delim_form())
                stats["delim_forms"][f] = stats["delim_forms"].get(f, 0) + 1
            want, wnd = dpref.delim(a, b0, b1, delim, k, add)
            if nd != wnd or not np.array_equal(got.astype(np.uint64), want):
                _save_fail(data=a, begin=b0, end=b1, delim=delim, k=k,
                                    add=add, offset=off, u64=du64)
                print(json.dumps({"FAIL": "delim", "size": size, "begin": b0, "end": b1, "delim": delim, "k": k,
                                  "add": add, "offset": off}), flush=True)
                raise SystemExit(1)
            stats["delim_cases"] += 1
            stats["delim_offsets"] += int(len(want))
        if time.time() - last > 20:
            last = time.time()
            print(json.dumps({"t": round(last - t0), **{k: v for k, v in stats.items() if k not in ("kinds", "delim_forms")}}),
                  flush=True)
    stats["_t"] = time.time() - t0
    ctx.close()
    return stats


if __name__ == "__main__":
    main()
