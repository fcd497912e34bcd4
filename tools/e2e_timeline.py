"""Timeline of one CSV ``co.preprocess()`` through the streamed index store: per piece, when its worker started and
finished (GETs + H2D + scan + D2H), when the consumer took it; per multipart part, when its upload started and
ended (ms from the call's start).  Memory store and/or the loopback HTTP server in a child process.

    python tools/e2e_timeline.py [--gib 4] [--src memory,http] [--piece-mib 512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4)
    ap.add_argument("--src", default="memory,http")
    ap.add_argument("--piece-mib", type=int, default=512)
    ap.add_argument("--detail", action="store_true", help="mark GET parts, H2D issue, launches and read-backs")
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--profile-ms", type=float, default=0, help="profile the main thread's first ms of every call")
    ap.add_argument("--all-calls", action="store_true", help="print every call's events (not only the last's)")
    args = ap.parse_args()
    from dataplug_amd import synth
    from dataplug_amd.cloudobject import CloudObject
    from dataplug_amd.formats import _lines
    from dataplug_amd.formats.generic.csv import CSV
    from dataplug_amd.scan import objects
    from dataplug_amd.storage import MemoryStore
    size = int(args.gib * (1 << 30))
    _lines.index_object.__defaults__ = (0, "auto", args.piece_mib << 20)
    ev = []
    t0 = [0.0]
    lock = threading.Lock()

    def mark(what, **kw):
        with lock:
            ev.append(dict(t_ms=round((time.perf_counter() - t0[0]) * 1e3, 2), what=what,
                           thread=threading.current_thread().name, **kw))
    real_group = objects._delim_group

    def group(dev, co, lo, hi, *a, **kw):
        mark("piece_start", lo=lo)
        r = real_group(dev, co, lo, hi, *a, **kw)
        mark("piece_end", lo=lo)
        return r
    objects._delim_group = group
    real_flush, real_close = _lines.MultipartWriter._flush, _lines.MultipartWriter.close

    def flush(self):
        mark("part_submit", key=self.key[-10:], n=len(self.futs) + 1, bytes=self.npend)
        real_flush(self)
        f = self.futs[-1]
        n = len(self.futs)
        f.add_done_callback(lambda _f, n=n, k=self.key[-10:]: mark("part_done", key=k, n=n))

    def close(self):
        mark("close_start", key=self.key[-10:])
        r = real_close(self)
        mark("close_end", key=self.key[-10:])
        return r
    _lines.MultipartWriter._flush, _lines.MultipartWriter.close = flush, close
    real_pieces = objects.line_index_pieces

    def pieces(*a, **kw):
        for p in real_pieces(*a, **kw):
            mark("consume", n=len(p[0]))
            yield p
    objects.line_index_pieces = pieces
    from dataplug_amd.formats.generic import csv as fcsv
    from dataplug_amd.preprocessing import handler, preprocess as pre
    from dataplug_amd import cloudobject as cob

    def wrap(mod, name):
        real = getattr(mod, name)

        def w(*a, **kw):
            mark(name + "_start")
            try:
                return real(*a, **kw)
            finally:
                mark(name + "_end")
        setattr(mod, name, w)
    wrap(fcsv, "index_object")
    wrap(objects, "line_index_form")
    for mod in (handler, pre):
        if hasattr(mod, "upload_metadata"):
            wrap(mod, "upload_metadata")
    real_fetch = cob.CloudObject.fetch

    def fetch(self, *a, **kw):
        mark("fetch_start")
        r = real_fetch(self, *a, **kw)
        mark("fetch_end")
        return r
    cob.CloudObject.fetch = fetch
    import gc
    from dataplug_amd.storage import client as stc
    for cls in (stc.LocalS3Client, stc.HTTPS3Client):
        for meth in ("put_object", "complete_multipart_upload", "get_object", "head_object"):
            real_m = getattr(cls, meth)

            def m(self, *a, _real=real_m, _meth=meth, **kw):
                big = _meth != "get_object" or kw.get("Range") is None
                if big:
                    mark(_meth + "_start", key=str(kw.get("Key", ""))[-12:])
                try:
                    return _real(self, *a, **kw)
                finally:
                    if big:
                        mark(_meth + "_end", key=str(kw.get("Key", ""))[-12:])
            setattr(cls, meth, m)
    wrap(_lines, "store_line_index_stream")
    import pandas as pd
    wrap(pd, "read_csv")
    wrap(cob, "open_object")
    # inside the streamed pieces: GET parts (per thread), the H2D issue loop, the scan launch, the read-back wait
    if args.detail:
        from dataplug_amd.scan import device as sdev
        real_rri = objects.read_range_into

        def rri(storage, bucket, key, lo, hi, *a, **kw):
            mark("get_start", lo=lo)
            try:
                return real_rri(storage, bucket, key, lo, hi, *a, **kw)
            finally:
                mark("get_end", lo=lo)
        objects.read_range_into = rri
        real_land = objects.land_gets

        def land(ctx, gets, dp):
            mark("land_start", n=gets[1])
            try:
                return real_land(ctx, gets, dp)
            finally:
                mark("land_end", n=gets[1])
        objects.land_gets = land
        for meth in ("delim_ranges_async", "delim_ranges_result", "sync"):
            real_m = getattr(sdev.ScanContext, meth)

            def m(self, *a, _real=real_m, _meth=meth, **kw):
                mark(_meth + "_start", slot=getattr(self, "slot", None))
                try:
                    return _real(self, *a, **kw)
                finally:
                    mark(_meth + "_end", slot=getattr(self, "slot", None))
            setattr(sdev.ScanContext, meth, m)
    # a sampler of the main thread's stack every 0.5 ms while a call runs: what it does in the gaps between marks
    samples = []
    sampling = threading.Event()
    main_id = threading.main_thread().ident

    def sampler():
        import traceback
        while True:
            sampling.wait()
            f = sys._current_frames().get(main_id)
            if f is not None:
                st = traceback.extract_stack(f)[-3:]
                samples.append((round((time.perf_counter() - t0[0]) * 1e3, 2),
                                " < ".join(f"{os.path.basename(x.filename)}:{x.lineno}:{x.name}" for x in reversed(st))))
            time.sleep(0.0005)
    threading.Thread(target=sampler, daemon=True).start()

    def gc_cb(phase, info):
        mark("gc_" + phase, gen=info.get("generation"))
    gc.callbacks.append(gc_cb)
    real_pcsv = fcsv.CSV.preprocessing_function if hasattr(fcsv.CSV, "preprocessing_function") else None
    bucket = "data"
    store = MemoryStore.named("e2e_tl")
    for b in (bucket, bucket + ".meta"):
        store.create_bucket(b)
    store.put(bucket, "x", synth.tiled_csv(size, seed=9).bytes_range(0, size))
    for src in args.src.split(","):
        cfg = {"endpoint_url": "memory://e2e_tl"}
        srv = None
        if src == "http":
            from e2e_legs import _Server
            srv = _Server(19074, [(f"{bucket}/x", "csv", size, 9)], [bucket + ".meta"])
            srv.wait_ready()
            cfg = {"endpoint_url": srv.url}
        co = CloudObject.from_s3(CSV, f"s3://{bucket}/x", s3_config=cfg)
        prof = []
        if args.profile_ms:
            def hook(frame, event, arg, _lim=args.profile_ms / 1e3):
                t = time.perf_counter() - t0[0]
                if 0 <= t < _lim:
                    name = getattr(arg, "__qualname__", None) if event.startswith("c_") else frame.f_code.co_name
                    prof.append((t, threading.current_thread().name, event,
                                 f"{os.path.basename(frame.f_code.co_filename)}:{frame.f_lineno}", name))
            threading.setprofile(hook)            # every thread started from here on (the pools start in call 0)
        for i in range(args.calls):
            if args.all_calls:
                for e in ev:
                    print(json.dumps(dict(e, call=i - 1)))
            ev.clear()
            samples.clear()
            t0[0] = time.perf_counter()
            mark("call_start")
            sampling.set()
            prof.clear()
            if args.profile_ms:
                # every thread's calls and returns (Python and C) over the call's first ms: a gap between two of the
                # main thread's is time spent inside one C call or waiting for the GIL; the other threads' events in
                # that gap show who had it
                sys.setprofile(hook)
            co.preprocess(force=True)
            sys.setprofile(None)
            mainp = [x for x in prof if x[1] == "MainThread"]
            for (ta, _, ea, wa, na), (tb, _, eb, wb, nb) in zip(mainp, mainp[1:]):
                if tb - ta > 0.5e-3:
                    print(json.dumps({"prof_gap_ms": round((tb - ta) * 1e3, 2), "at_ms": round(ta * 1e3, 2),
                                      "from": [ea, wa, na], "to": [eb, wb, nb]}))
                    if tb - ta > 3e-3:
                        others = [x for x in prof if x[1] != "MainThread" and ta - 1e-3 <= x[0] <= tb]
                        for x in others[:12] + (others[-12:] if len(others) > 24 else others[12:]):
                            print(json.dumps({"in_gap": [round(x[0] * 1e3, 3)] + list(x[1:])}))
            sampling.clear()
            mark("call_end")
            dt = ev[-1]["t_ms"]
            print(json.dumps({"src": src, "call": i, "ms": dt, "GiB_per_s": round(size / (dt / 1e3) / (1 << 30), 2)}),
                  flush=True)
        for e in ev:
            print(json.dumps(e))
        last = None
        for t, where in samples:                  # the main thread's stack, one line per change
            if where != last:
                print(json.dumps({"sample_ms": t, "main": where}))
                last = where
        if srv is not None:
            srv.stop()


if __name__ == "__main__":
    main()
