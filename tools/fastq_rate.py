"""FASTQ.gz per-read index rates (BASELINE configs[4], fastqgz_example.py shape), for DESIGN.md §6.

    python tools/fastq_rate.py [--reads N] [--reps R] [--repeat K]

A synthetic FASTQ (100 bp reads) in an in-process store (memory://), as
* "gzip6 zlib": one gzip member (level 6) inflated by zlib on one core (the reference's gztool is serial too);
* "gzip6": the same member inflated in parallel (libdpgz dpgz_par: speculative deflate block starts, marker
  windows, CRC-checked) on the process's CPU share;
* "gzip6 xK": the same member K times (multi-member), a K x larger inflated stream through the same bounded
  pipeline (host memory must not grow);
* "bgzf": BGZF 64 KiB members (level 6), inflated member-parallel on the host thread pool.
For each: `co.preprocess()` of FASTQGZip end to end (one streamed GET, inflate into pinned pieces, H2D, the
newline scan on the GPU with the ordinal carried across pieces, D2H of the read ends, window table + read
index PUTs), the peak host memory the call added (RSS sampled every 5 ms), and the read ends checked
against the reads' own line ends.  Plus the device-resident read-end index of the inflated stream
(dp_delim_index every_k = 4, emit_add = 1) timed with HIP events.
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.cloudobject import CloudObject  # noqa: E402
from dataplug_amd.formats.genomics.fastq import FASTQGZip, load_read_index  # noqa: E402
from dataplug_amd.scan import get_context  # noqa: E402
from dataplug_amd.scan.gzindex import pool_threads  # noqa: E402
from dataplug_amd.storage import MemoryStore  # noqa: E402

GiB = float(1 << 30)


def rss() -> int:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) * 1024
    return 0


class PeakRSS:
    def __init__(self):
        self.peak = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            self.peak = max(self.peak, rss())
            time.sleep(0.005)

    def __enter__(self):
        self.base = rss()
        self.peak = self.base
        self._t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self._t.join()


def run_case(name, blob, raw_len, exp_ends, reps, threads=0):
    key = f"r_{name.replace(' ', '_')}.fastq.gz"
    store = MemoryStore.named("fq")
    store.put("genomics", key, blob)
    co = CloudObject.from_s3(FASTQGZip, f"s3://genomics/{key}", s3_config={"endpoint_url": "memory://fq"})
    extra = {"inflate_threads": threads}
    co.preprocess(force=True, extra_args=extra)             # warm: pandas/pyarrow, context, buffers
    ts, peak = [], 0
    for _ in range(reps):
        with PeakRSS() as pr:
            t0 = time.perf_counter()
            co.preprocess(force=True, extra_args=extra)
            ts.append(time.perf_counter() - t0)
        peak = max(peak, pr.peak - pr.base)
    got = load_read_index(co)
    ok = bool(np.array_equal(got, exp_ends))
    t = min(ts)
    out = {"case": name, "inflate_threads": threads or pool_threads(), "gzip_bytes": len(blob),
           "inflated_bytes": raw_len, "members": co.attributes.gzip_members,
           "bgzf": co.attributes.bgzf, "preprocess_s": round(t, 3),
           "preprocess_inflated_GiB_per_s": round(raw_len / t / GiB, 3),
           "preprocess_gzip_GiB_per_s": round(len(blob) / t / GiB, 3),
           "peak_host_rss_added_MiB": round(peak / 2**20, 1), "verified": ok}
    store.delete("genomics", key)
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=4)
    ap.add_argument("--device-gib", type=int, default=16, help="inflated bytes of the device-resident launch")
    args = ap.parse_args()
    t0 = time.perf_counter()
    raw = synth.fastq(args.reads, seed=5)
    rb = raw.tobytes()
    g6 = gzip.compress(rb, 6)
    bg = synth.bgzf(rb, level=6)
    nl = np.flatnonzero(raw == 10).astype(np.uint64)
    exp_ends = nl[3::4] + np.uint64(1)
    print(json.dumps({"reads": args.reads, "inflated_bytes": len(rb), "gen_s": round(time.perf_counter() - t0, 1),
                      "inflate_threads": pool_threads()}), flush=True)
    store = MemoryStore.named("fq")
    store.create_bucket("genomics")
    store.create_bucket("genomics.meta")
    run_case("gzip6 zlib", g6, len(rb), exp_ends, args.reps, threads=1)
    run_case("gzip6", g6, len(rb), exp_ends, args.reps)
    # K copies of the member: a K x larger stream (multi-member), ends shifted per copy
    ek = np.concatenate([exp_ends + np.uint64(i * len(rb)) for i in range(args.repeat)])
    run_case(f"gzip6 x{args.repeat}", g6 * args.repeat, len(rb) * args.repeat, ek, 1)
    del ek
    run_case("bgzf", bg, len(rb), exp_ends, args.reps)
    # device-resident read-end index (every 4th newline + 1), HIP events around each launch, over the
    # inflated stream tiled to --device-gib GiB (whole reads per copy, so the expected ends are the copy's
    # ends shifted; a full-size launch instead of the 457 MB one, whose fixed grid start/tail dominate)
    ctx = get_context(0)
    copies = max(1, (args.device_gib << 30) // len(raw))
    n = copies * len(raw)
    d = ctx.workspace("fq_in", n + 64)
    for i in range(copies):
        ctx.h2d(d.ptr + i * len(raw), raw)
    exp_ends = np.concatenate([exp_ends + np.uint64(i * len(raw)) for i in range(copies)])
    cap = len(exp_ends) + 1024
    out = ctx.workspace("fq_out", 8 * cap)
    ctx.delim_index_async(d.ptr, n, 0, 0, n, 10, 4, 1, out.ptr, True, cap)
    ctx.delim_result()
    ctx.timing(True)
    ctx.timing_read()
    for _ in range(10):
        ctx.delim_index_async(d.ptr, n, 0, 0, n, 10, 4, 1, out.ptr, True, cap)
        n_out, _ = ctx.delim_result()
    ms, launches = ctx.timing_read()
    ctx.timing(False)
    ends = ctx.d2h(np.empty(n_out, np.uint64), out.ptr)
    k = ms / 1e3 / launches
    print(json.dumps({"device_read_index_bytes": n, "device_read_index_reads": int(n_out),
                      "device_read_index_kernel_us": round(k * 1e6, 1),
                      "device_read_index_GiB_per_s": round(n / k / GiB, 1),
                      "device_read_index_alg_GBps": round((n + 8.0 * n_out) / k / 1e9, 1),
                      "device_read_index_frac_of_8TBps": round((n + 8.0 * n_out) / k / 8e12, 3),
                      "verified": bool(np.array_equal(ends, exp_ends))}), flush=True)


if __name__ == "__main__":
    main()
