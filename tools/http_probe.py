"""Loopback HTTP GET rate into pinned memory: the server in this process vs in its own process.

    python tools/http_probe.py [--size BYTES] [--reps N] [--port P]

read_range_into (16 threads, 32 MiB ranged GETs) of a synthetic object from (a) a LoopbackS3Server thread
inside this process, sharing its GIL with the client threads, and (b) the same server started as a separate
process (`python -m dataplug_amd.storage.server`), which is how MinIO serves the reference's examples.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from dataplug_amd.scan.objects import read_range_into  # noqa: E402
from dataplug_amd.storage import LoopbackS3Server, MemoryStore  # noqa: E402
from dataplug_amd.storage.client import make_client  # noqa: E402

GiB = float(1 << 30)


def rate(url: str, n: int, out: np.ndarray, reps: int):
    cl = make_client(url)
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        read_range_into(cl, "b", "k", 0, n, memoryview(out))
        best = max(best, n / (time.perf_counter() - t0) / GiB)
    return round(best, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=2 << 30)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--port", type=int, default=19000)
    args = ap.parse_args()
    n = args.size
    data = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
    out = np.empty(n, np.uint8)
    res = {"object_bytes": n}
    store = MemoryStore()
    store.create_bucket("b")
    store.put("b", "k", memoryview(data))
    with LoopbackS3Server(store) as srv:
        res["in_process_server_GiB_per_s"] = rate(srv.endpoint_url, n, out, args.reps)
    print(json.dumps(res), flush=True)
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=False) as f:
        f.write(memoryview(data))
        path = f.name
    proc = subprocess.Popen([sys.executable, "-m", "dataplug_amd.storage.server", "--port", str(args.port),
                             "--put", f"b/k={path}"], cwd=REPO, stdout=subprocess.PIPE, text=True)
    try:
        line = proc.stdout.readline()                 # "serving http://..." once the object is loaded
        assert line.startswith("serving"), line
        res["separate_process_server_GiB_per_s"] = rate(f"http://127.0.0.1:{args.port}", n, out, args.reps)
        assert np.array_equal(out, data)
    finally:
        proc.terminate()
        proc.wait(timeout=30)
        os.unlink(path)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
