"""End-to-end (PCIe-inclusive) rate of the FASTA index build, for DESIGN.md §6 (never bench.py's value).

    python tools/e2e_rate.py [--size BYTES] [--reps N] [--devices 0,0] [--only memory,loopback_http]

co.preprocess(chunk_size=size/4) on a synthetic FASTA held by (a) an in-process store (memory://), (b) the
loopback HTTP S3 server in its own process, and (c) the same server as a thread of this process: ranged
GETs into pinned host memory -> H2D -> scan -> D2H of the index -> PUT of index + attrs.  Also times the
stages separately on the same object.  ``--devices`` passes ``dataplug_devices`` to every preprocess (e.g.
``0,0,0,0`` rehearses the multi-GPU split on one GPU: four groups, four persistent workers), and each rep
reports the library's device / pinned allocations made during it (dp_alloc_counts: 0 once warm).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from dataplug_amd import synth  # noqa: E402
from dataplug_amd.cloudobject import CloudObject  # noqa: E402
from dataplug_amd.formats.genomics.fasta import FASTA  # noqa: E402
from dataplug_amd.scan import get_context  # noqa: E402
from dataplug_amd.scan import objects as so  # noqa: E402
from dataplug_amd.storage import LoopbackS3Server, MemoryStore  # noqa: E402

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4 << 30)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--port", type=int, default=19001)
    ap.add_argument("--devices", default=None, help="dataplug_devices for every preprocess, e.g. 0,0,0,0")
    ap.add_argument("--only", default=None, help="comma-separated subset of the store configurations")
    ap.add_argument("--no-stages", action="store_true")
    args = ap.parse_args()
    from dataplug_amd.scan._lib import alloc_counts
    pc = {"dataplug_devices": [int(x) for x in args.devices.split(",")]} if args.devices else {}
    size = args.size
    host = synth.tiled_fasta_host(size, seed=1)
    store = MemoryStore.named("e2e")
    store.create_bucket("genomics")
    store.create_bucket("genomics.meta")
    store.put("genomics", "x.fasta", memoryview(host))
    del host
    cs = math.ceil(size / 4)
    res = {"object_bytes": size, "chunk_size": cs, "dataplug_devices": pc.get("dataplug_devices")}
    srv = LoopbackS3Server(store).start()
    # the loopback server in its own process, as MinIO serves the reference's examples (an in-process server
    # shares the GIL with the client's GET threads: tools/http_probe.py)
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=False) as f:
        f.write(memoryview(store.get("genomics", "x.fasta").data))
        path = f.name
    port = args.port
    proc = subprocess.Popen([sys.executable, "-m", "dataplug_amd.storage.server", "--port", str(port),
                             "--put", f"genomics/x.fasta={path}", "--bucket", "genomics.meta"],
                            cwd=REPO, stdout=subprocess.PIPE, text=True)
    line = proc.stdout.readline()
    assert line.startswith("serving"), line
    os.unlink(path)
    configs = (("memory", {"endpoint_url": "memory://e2e"}),
               ("loopback_http", {"endpoint_url": f"http://127.0.0.1:{port}"}),
               ("loopback_http_in_process", srv.storage_config))
    for name, cfg in configs:
        if args.only and name not in args.only.split(","):
            continue
        co = CloudObject.from_s3(FASTA, "s3://genomics/x.fasta", s3_config=cfg)
        co.preprocess(chunk_size=cs, force=True, parallel_config=pc)   # warm: contexts, pinned + device buffers
        ts, allocs = [], []
        for _ in range(args.reps):
            a0 = alloc_counts()
            t0 = time.perf_counter()
            co.preprocess(chunk_size=cs, force=True, parallel_config=pc)
            ts.append(time.perf_counter() - t0)
            a1 = alloc_counts()
            allocs.append([a1[0] - a0[0], a1[1] - a0[1]])
        t = min(ts)
        res[f"{name}_preprocess_s"] = round(t, 3)
        res[f"{name}_GiB_per_s"] = round(size / t / GiB, 2)
        res[f"{name}_allocs_per_rep"] = allocs
        print(name, res, flush=True)
    if args.no_stages:
        srv.stop()
        proc.terminate()
        proc.wait(timeout=30)
        print(json.dumps(res), flush=True)
        return
    # stage breakdown (memory store)
    co = CloudObject.from_s3(FASTA, "s3://genomics/x.fasta", s3_config={"endpoint_url": "memory://e2e"})
    ctx = get_context(0)
    pin = ctx.pinned("object", size)
    t0 = time.perf_counter()
    so.read_range_into(co.storage, "genomics", "x.fasta", 0, size, pin.view(size))
    t_get = time.perf_counter() - t0
    d = ctx.workspace("input", size + 64)
    ctx.sync()
    t0 = time.perf_counter()
    ctx.h2d_async(d.ptr, pin.ptr, size)
    ctx.sync()
    t_h2d = time.perf_counter() - t0
    ctx.sync()
    t0 = time.perf_counter()
    so.fetch_to_device(ctx, co.storage, "genomics", "x.fasta", 0, size, d.ptr)
    ctx.sync()
    t_pipe = time.perf_counter() - t0
    plan = [(i * cs, min(size, (i + 1) * cs)) for i in range(size // cs)]
    ctx.fasta_index(d.ptr, size, 0, size, plan)
    t0 = time.perf_counter()
    pairs, _, _ = ctx.fasta_index(d.ptr, size, 0, size, plan)
    t_scan = time.perf_counter() - t0
    res.update({"stage_get_into_pinned_GiB_per_s": round(size / t_get / GiB, 2),
                "stage_h2d_GiB_per_s": round(size / t_h2d / GiB, 2),
                "stage_get_h2d_pipelined_GiB_per_s": round(size / t_pipe / GiB, 2),
                "stage_scan_plus_d2h_s": round(t_scan, 4), "index_bytes": int(pairs.nbytes)})
    srv.stop()
    proc.terminate()
    proc.wait(timeout=30)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
