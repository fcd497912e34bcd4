"""End-to-end legs of bench.py's one JSON line (the ``e2e`` and ``fastq`` sub-objects; N = 1, rank 0 only).

The path starts and ends in host memory (BASELINE north_star): bytes arrive from storage, the index object is written
back.  These legs time ``co.preprocess()`` through the product path -- ranged GETs into pinned memory, per-part H2D,
the scan, D2H of the index, the index PUT (reference: preprocessing/handler.py:36-42 ranged GET, :82-129 index PUT;
formats/compressed/gzipped.py:46-153 for FASTQ.gz) -- and split the same object's stages.  Never bench.py's ``value``
(which is device-resident).

* ``e2e``: the configs[1] FASTA (4 GiB, chunk_size = size / 4, uint32 index) and a configs[2]-shaped CSV (cities.csv
  rows, 4 GiB by default: configs[2]'s 32 GiB would spend the leg's budget on generating and pinning host copies), each
  from an in-process store (memory://) and from the loopback HTTP S3 server in its own process (as MinIO serves the
  reference's examples).  Every stored index is read back and checked (FASTA against the C oracle, CSV offset by
  offset against the synthetic object's own newlines).
* ``fastq``: configs[4], a FASTQ.gz (one gzip member, level 6, deflated here on a thread pool as pigz does: sync-
  flushed pieces of one deflate stream) of a seeded read tile repeated, ``co.preprocess()`` of FASTQGZip end to end:
  one streamed GET, the parallel inflate into pinned pieces, H2D, the read-end scan with the ordinal carried across
  pieces, D2H, the index PUTs; every read end checked.
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import os
import subprocess
import sys
import time
import zlib

import numpy as np

GiB = float(1 << 30)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _timed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def parallel_gzip(raw: np.ndarray, level: int = 6, piece: int = 1 << 20, threads: int = 16) -> bytes:
    """ONE gzip member of ``raw``: pieces deflated on a thread pool (zlib releases the GIL), each ended by a sync flush
    (byte-aligned, not final) so their raw deflate streams concatenate into one, the last one finished; the trailer
    holds the CRC-32 and size of the whole stream.  (pigz's layout, without its dictionary carry-over.)"""
    mv = memoryview(np.ascontiguousarray(raw).view(np.uint8).reshape(-1))
    n = len(mv)
    starts = list(range(0, n, piece)) or [0]

    def one(i):
        a = starts[i]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        out = c.compress(mv[a:min(n, a + piece)])
        return out + c.flush(zlib.Z_FINISH if i == len(starts) - 1 else zlib.Z_SYNC_FLUSH)

    with cf.ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(one, range(len(starts))))
    crc = zlib.crc32(mv)
    head = b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff"
    return b"".join([head] + parts + [crc.to_bytes(4, "little"), (n & 0xFFFFFFFF).to_bytes(4, "little")])


class _Server:
    """The loopback S3 server in a child process, holding seeded synthetic objects it generates itself."""

    def __init__(self, port: int, objects, buckets):
        cmd = [sys.executable, "-m", "dataplug_amd.storage.server", "--port", str(port)]
        for dst, kind, size, seed in objects:
            cmd += ["--synth", f"{dst}={kind},{size},{seed}"]
        for b in buckets:
            cmd += ["--bucket", b]
        self.proc = subprocess.Popen(cmd, cwd=REPO, stdout=subprocess.PIPE, text=True)
        self.url = f"http://127.0.0.1:{port}"

    def wait_ready(self):
        line = self.proc.stdout.readline()
        if not line.startswith("serving"):
            raise RuntimeError(f"loopback server did not start: {line!r}")

    def stop(self):
        self.proc.terminate()
        try:
            self.proc.wait(timeout=30)
        except subprocess.TimeoutExpired:
            self.proc.kill()


def _stages(co, kind: str, size: int, chunk_size: int):
    """The stages of one preprocess on the same object (memory store), timed one by one on the caller's context:
    ranged GETs into pinned memory, H2D, the two pipelined (scan.objects.fetch_to_device), the scan (HIP events),
    D2H of the index, the index PUT."""
    from dataplug_amd.scan import get_context
    from dataplug_amd.scan import objects as so
    ctx = get_context(0)
    st, b, k = co.storage, co.path.bucket, co.path.key
    pin = ctx.pinned("object", size)
    d = ctx.workspace("input", size + 64)
    ctx.sync()
    t_get = _timed(lambda: so.read_range_into(st, b, k, 0, size, pin.view(size)), 2)

    def h2d():
        ctx.h2d_async(d.ptr, pin.ptr, size)
        ctx.sync()
    t_h2d = _timed(h2d, 2)

    def pipe():
        so.fetch_to_device(ctx, st, b, k, 0, size, d.ptr)
        ctx.sync()
    t_pipe = _timed(pipe, 2)
    if kind == "fasta":
        from dataplug_amd.preprocessing.handler import chunk_plan
        plan = chunk_plan(size, chunk_size)          # the reference's plan (preprocess.py:38, handler.py:36-38)
        ch = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))
        cap = size // 256 + 1024
        out = ctx.workspace("e2e_out", 8 * cap)

        def scan():
            ctx.fasta_index_async(d.ptr, size, 0, size, ch, out.ptr, False, cap)
            return ctx.fasta_result(len(plan))[0]
        n = scan()
        ctx.timing(True)
        ctx.timing_read()
        for _ in range(3):
            scan()
        ms, nl = ctx.timing_read()
        ctx.timing(False)
        idx_bytes = 8 * n
        host = np.empty(idx_bytes, np.uint8)
    else:
        rg = np.asarray([0, size], np.uint64)
        cap = size // 16 + 1024
        out = ctx.workspace("e2e_out", ctx.out_bytes(cap, 4, rg))

        def scan():                                  # the stored form, u8s (out_mode 4)
            ctx.delim_ranges_async(d.ptr, size, 0, rg, 10, 1, 0, 0, out.ptr, 4, cap)
            return ctx.delim_ranges_result(1)[0]
        n = scan()
        ctx.timing(True)
        ctx.timing_read()
        for _ in range(3):
            scan()
        ms, nl = ctx.timing_read()
        ctx.timing(False)
        idx_bytes = n + 2 * ctx.sub_table_size(rg)[1] + 8 * ctx.block_table_size(rg)[1]
        host = np.empty(idx_bytes, np.uint8)
    t_d2h = _timed(lambda: ctx.d2h(host, out.ptr), 2)
    mb = co.meta_path.bucket
    t_put = _timed(lambda: st.put_object(Body=host.tobytes(), Bucket=mb, Key=co.meta_path.key + ".e2e_stage"), 2)
    st.delete_object(Bucket=mb, Key=co.meta_path.key + ".e2e_stage")
    t_scan = ms / 1e3 / max(1, nl)
    return {"get_into_pinned_GiB_per_s": round(size / t_get / GiB, 2), "h2d_GiB_per_s": round(size / t_h2d / GiB, 2),
            "get_h2d_pipelined_GiB_per_s": round(size / t_pipe / GiB, 2),
            "scan_us": round(t_scan * 1e6, 1), "scan_GiB_per_s": round(size / t_scan / GiB, 1),
            "index_bytes": int(idx_bytes), "d2h_s": round(t_d2h, 4), "put_s": round(t_put, 4),
            "note": "each stage alone on the same object (memory store), best of 2 (scan: HIP events, mean of 3)"}


def _verify_fasta(co, host: np.ndarray, chunk_size: int) -> bool:
    from oracle import cpu_ref, dpref            # the checker (test infrastructure), outside every timed region
    plan = cpu_ref.chunk_plan(len(host), chunk_size)   # the reference's plan (preprocess.py:30-61), quirks included
    exp = dpref.fasta_pairs(host, plan).astype(np.uint32).reshape(-1)
    got = np.frombuffer(co.storage.get_object(Bucket=co.meta_path.bucket, Key=co.meta_path.key)["Body"].read(),
                        np.uint32)
    return bool(np.array_equal(got, exp))


def _verify_csv(co, obj, size: int, verify_blocked, verify_bytes) -> bool:
    """The stored newline index (u8s: low bytes + 256-byte counts + block table, or u16b: low words + block table)
    against the object's analytic newline positions."""
    st, mb = co.storage, co.meta_path.bucket

    def get(attr, dt):
        return np.frombuffer(st.get_object(Bucket=mb, Key=co.get_attribute(attr))["Body"].read(), dt)
    n = int(co.get_attribute("num_lines"))
    tab = get("line_index_blocks_key", "<u8")
    if co.get_attribute("line_index_dtype") == "u8s":
        ok = verify_bytes(obj, 0, size, get("line_index_key", "u1"), get("line_index_sub_key", "<u2"), tab, n)
    else:
        ok = verify_blocked(obj, 0, size, get("line_index_key", "<u2"), tab, n)
    return bool(n == obj.count_range(0, size) and ok)


def e2e_leg(fasta_size: int = 4 << 30, csv_size: int = 4 << 30, reps: int = 2, port: int = 19071,
            verify_blocked=None, verify_bytes=None, verify: bool = True, log=print) -> dict:
    """The ``e2e`` sub-object (see the module doc)."""
    from dataplug_amd import synth
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats.generic.csv import CSV
    from dataplug_amd.formats.genomics.fasta import FASTA
    from dataplug_amd.storage import MemoryStore
    t_leg = time.perf_counter()
    cs = math.ceil(fasta_size / 4)
    objs = [("fasta", FASTA, "genomics", "e2e.fasta", fasta_size, 1),
            ("csv", CSV, "data", "e2e.csv", csv_size, 9)]
    srv = _Server(port, [(f"{b}/{k}", kind, size, seed) for kind, _, b, k, size, seed in objs],
                  ["genomics.meta", "data.meta"])
    store = MemoryStore.named("bench_e2e")
    out = {"unit": "GiB/s", "note": "co.preprocess() end to end, host memory to host memory: ranged GETs -> pinned "
                                    "-> H2D -> scan -> D2H -> index PUT; best of %d after a warm call; never bench.py's "
                                    "value (device-resident)" % reps}
    ready = False
    try:
        for kind, fmt, bucket, key, size, seed in objs:
            t0 = time.perf_counter()
            if kind == "fasta":
                host = synth.tiled_fasta_host(size, seed=seed)
                obj = None
            else:
                obj = synth.tiled_csv(size, seed=seed)
                host = obj.bytes_range(0, size)
            for b in (bucket, bucket + ".meta"):
                if not store.has_bucket(b):
                    store.create_bucket(b)
            store.put(bucket, key, host)
            gen_s = time.perf_counter() - t0
            res = {"object_bytes": size, "gen_s": round(gen_s, 2)}
            if kind == "fasta":
                res["config"] = f"BASELINE configs[1]: {size / GiB:g} GiB FASTA, chunk_size={cs} (size/4), uint32 index"
            else:
                res["config"] = (f"configs[2]-shaped CSV (cities.csv rows) of {size / GiB:g} GiB, newline index stored as "
                                 f"uint8 low bytes + 256-byte counts + 64 KiB block table (u8s)")
            for src in ("memory", "loopback_http"):
                if src == "loopback_http" and not ready:
                    srv.wait_ready()                        # (it generated its copies while this process did)
                    ready = True
                cfg = {"endpoint_url": "memory://bench_e2e"} if src == "memory" else {"endpoint_url": srv.url}
                co = CloudObject.from_s3(fmt, f"s3://{bucket}/{key}", s3_config=cfg)
                call = (lambda: co.preprocess(chunk_size=cs, force=True)) if kind == "fasta" else \
                    (lambda: co.preprocess(force=True))
                call()                                      # warm: contexts, pinned + device buffers, imports
                t = _timed(call, reps)
                ok = None
                if verify:
                    ok = _verify_fasta(co, host, cs) if kind == "fasta" else _verify_csv(co, obj, size, verify_blocked, verify_bytes)
                res[src] = {"preprocess_s": round(t, 4), "value": round(size / t / GiB, 2), "verified": ok}
                log(f"e2e {kind} {src}: {res[src]}")
            co = CloudObject.from_s3(fmt, f"s3://{bucket}/{key}", s3_config={"endpoint_url": "memory://bench_e2e"})
            res["stages"] = _stages(co, kind, size, cs)
            out[kind] = res
            del host
            store.delete(bucket, key)
    finally:
        srv.stop()
    out["leg_s"] = round(time.perf_counter() - t_leg, 2)
    return out


def fastq_leg(tile_reads: int = 65536, tiles: int = 16, reps: int = 2, level: int = 6, threads: int = 16,
              verify: bool = True, log=print) -> dict:
    """The ``fastq`` sub-object (configs[4]; see the module doc)."""
    from dataplug_amd import synth
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats.genomics.fastq import FASTQGZip, load_read_index
    from dataplug_amd.scan.gzindex import pool_threads
    from dataplug_amd.storage import MemoryStore
    t_leg = time.perf_counter()
    tile = synth.fastq(tile_reads, seed=5)
    raw = np.tile(tile, tiles)
    t0 = time.perf_counter()
    blob = parallel_gzip(raw, level=level, threads=threads)
    gz_s = time.perf_counter() - t0
    nl = np.flatnonzero(tile == 10).astype(np.uint64)
    ends1 = nl[3::4] + np.uint64(1)
    exp = (ends1[None, :] + (np.arange(tiles, dtype=np.uint64) * np.uint64(len(tile)))[:, None]).reshape(-1)
    store = MemoryStore.named("bench_fq")
    for b in ("genomics", "genomics.meta"):
        if not store.has_bucket(b):
            store.create_bucket(b)
    store.put("genomics", "e2e.fastq.gz", blob)
    co = CloudObject.from_s3(FASTQGZip, "s3://genomics/e2e.fastq.gz", s3_config={"endpoint_url": "memory://bench_fq"})
    co.preprocess(force=True)                                # warm: pandas / pyarrow, context, pieces
    t = _timed(lambda: co.preprocess(force=True), reps)
    ok = bool(np.array_equal(load_read_index(co), exp)) if verify else None
    res = {"metric": "FASTQ.gz per-read index, end to end (BASELINE configs[4])", "unit": "GiB/s",
           "value": round(len(raw) / t / GiB, 3), "gzip_GiB_per_s": round(len(blob) / t / GiB, 3),
           "preprocess_s": round(t, 4), "reads": int(len(exp)), "inflated_bytes": int(len(raw)),
           "gzip_bytes": len(blob), "gzip_members": int(co.attributes.gzip_members),
           "inflate_threads": pool_threads(), "verified_every_read_end": ok,
           "config": f"one gzip member (level {level}) of {tiles} copies of a seeded {tile_reads}-read FASTQ tile "
                     f"(100 bp reads), in-process store: one streamed GET, parallel inflate into pinned pieces, H2D, "
                     f"read ends on the GPU (every 4th newline + 1, ordinal carried across pieces), D2H, index PUTs; "
                     f"best of {reps} after a warm call",
           "gzip_gen_s": round(gz_s, 2)}
    store.delete("genomics", "e2e.fastq.gz")
    res["leg_s"] = round(time.perf_counter() - t_leg, 2)
    log(f"fastq: {res['value']} GiB/s inflated, verified {ok}")
    return res
