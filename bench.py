#!/usr/bin/env python3
"""Benchmark: device-resident FASTA header-index scan (BASELINE.json configs[1]) on 1..N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size BYTES] [--no-cpu-baseline]
    python bench.py --workload csv|vcf ...    (BASELINE configs[2] / configs[3]: newline index)

The workload is ONE synthetic FASTA object of N x 4 GiB (N = --gpus) with the reference's chunk plan at
chunk_size = 1 GiB (size / 4N: 4 chunks per GPU, the configs[1] plan at N = 1), split over the N GPUs by
the product's multi-GPU split (``scan.objects.fasta_groups``: contiguous chunk groups, one per GPU, no
collective; the reference runs the chunks as independent map jobs, preprocess.py:39-51).  Each GPU holds
its group's bytes (+ a 64 KiB look-ahead halo) in HBM before the timed region.

One step = on every GPU, one dp_fasta_index over its chunk group: the chunk-table check, the single-pass
scan kernel, the split-header resolve kernel and the read-back of pair count / per-chunk state (the index
stays in HBM; the H2D/D2H-inclusive end-to-end rate is in DESIGN.md §6).  Steps alternate between two
scan contexts (streams) and step k + 1 is enqueued before step k's result is collected, so the host round
trip hides behind the next scan.  The library runs one scan grid at a time per GPU (a scan launch waits on
the device for the device's previous scan), while step k's resolve kernel and read-back overlap scan k + 1,
as consecutive objects do in production: ``value`` is this pipelined rate, provided its ``ms_per_step`` is
at least the scan kernel's own average duration (checked in the run; otherwise ``value`` falls back to the
``serialized`` rate, where each step also waits on the device for the previous step's tail, which is always
reported as a secondary field).

Launch modes (the same worker code in both):
  * ``python bench.py --gpus N``: one process, one host thread per GPU (how ``co.preprocess`` runs a
    multi-GPU object, scan/objects.py); exits non-zero if fewer than N devices are visible
    (``--devices 0,0,0,0`` maps workers to devices explicitly, e.g. to rehearse the split on one GPU).
  * ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``: one rank per GPU; barriers and
    the max/sum reductions go over a gloo CPU group, so RCCL is never initialised (nothing is exchanged).

Also measured in this run: every GPU's scan-kernel average duration from HIP events on its own stream
(-> roofline, with a read-only stream kernel's rate on the same buffer as the measured peak), the fixed-
total ("strong") curve point — the configs[1] 4 GiB object split over the same N GPUs — and, at N = 1, the
reference algorithm on the host cores (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12   # B/s, MI355X spec (MI355X_MICROARCH.md §Chip-level parameters)
GiB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["fasta", "csv", "vcf"], default="fasta",
                   help="fasta: configs[1] (default, the headline line); csv: configs[2], a 32 GiB CSV per GPU; "
                        "vcf: configs[3], one 64 GiB VCF whose body is cut into one part per GPU")
    p.add_argument("--size", type=int, default=None,
                   help="bytes per GPU (default 4 GiB fasta, 32 GiB csv) / object bytes (vcf, default 64 GiB)")
    p.add_argument("--chunks", type=int, default=4, help="FASTA map chunks per GPU (chunk_size = size / (chunks*N))")
    p.add_argument("--index-dtype", choices=["u16b", "u32p", "u64"], default="u16b",
                   help="csv/vcf newline index form: u16b = uint16 low words + 64 KiB block table (what "
                        "co.preprocess stores), u32p = uint32 low words + 4 GiB page counts, u64 = plain uint64")
    p.add_argument("--devices", default=None,
                   help="comma-separated device of each worker / local rank (default 0..N-1); e.g. 0,0,0,0 "
                        "rehearses the multi-GPU split on one GPU")
    p.add_argument("--no-strong", action="store_true", help="skip the fixed-total (strong scaling) point")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--traffic-bytes", type=float, default=None,
                   help="HBM bytes per scan launch from a rocprofv3 --pmc pass (overrides --traffic-from)")
    p.add_argument("--traffic-from", default=None,
                   help="pmc_summary.json (tools/pmc_summary.py) of this same command: FETCH_SIZE x2 (gfx950) "
                        "+ WRITE_SIZE per scan-kernel launch (default profiles/latest_pmc_summary[_<workload>].json)")
    return p.parse_args()


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------ team of workers
class Team:
    """The workers of one run: host threads of this process (one per GPU), or this process as one rank of
    a torch.distributed.run launch (gloo CPU group: barriers and the final gather only, never RCCL)."""

    def __init__(self, n_local: int, pg=None):
        self._tb = threading.Barrier(n_local)
        self.pg = pg

    def barrier(self):
        self._tb.wait()
        if self.pg is not None:
            self.pg.barrier()

    def gather(self, results):
        """rank 0: every rank's list of worker results, concatenated; other ranks: None."""
        if self.pg is None:
            return results
        out = [None] * self.pg.get_world_size()
        self.pg.all_gather_object(out, results)
        return [r for rs in out for r in rs] if self.pg.get_rank() == 0 else None


def launch_mode(args):
    """(world, rank, [devices of this process's workers], process group or None)."""
    from dataplug_amd.scan import device_count
    if "TORCHELASTIC_RUN_ID" in os.environ or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus not in (1, world):
            log(f"--gpus {args.gpus} != WORLD_SIZE {world}: one rank per GPU, using {world}")
        dev = local
        if args.devices:                                  # rehearsal: map local ranks to devices explicitly
            dev = [int(x) for x in args.devices.split(",")][local]
        if dev >= device_count():
            log(f"rank {rank}: device {dev} but only {device_count()} device(s) visible")
            sys.exit(2)
        # gloo prints "[Gloo] Rank r is connected to ..." on stdout from C++; keep stdout to the ONE JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        return world, rank, [dev], dist
    n = args.gpus
    devs = [int(x) for x in args.devices.split(",")] if args.devices else list(range(n))
    if len(devs) != n:
        log(f"--devices names {len(devs)} device(s) for --gpus {n}")
        sys.exit(2)
    visible = device_count()
    if max(devs) >= visible:
        log(f"--gpus {n} needs devices {sorted(set(devs))}, but only {visible} visible")
        sys.exit(2)
    return n, 0, devs, None


def run_workers(fn, devs, rank0_index, team):
    """fn(worker index, device) on one thread per device (inline when there is one); the results in order."""
    if len(devs) == 1:
        return [fn(rank0_index, devs[0])]
    res, errs = [None] * len(devs), []

    def body(i):
        try:
            res[i] = fn(rank0_index + i, devs[i])
        except BaseException as e:      # a failed worker must not leave the others waiting in a barrier
            errs.append(e)
            team._tb.abort()

    th = [threading.Thread(target=body, args=(i,)) for i in range(len(devs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return res


class Steps:
    """K steps of one scan workload alternating between two contexts of one GPU (see the module doc)."""

    def __init__(self, team, ctxs, launch, collect):
        self.team, self.ctxs, self.launch, self.collect = team, ctxs, launch, collect

    def warm(self, n):
        for i in range(max(2, n)):                    # both contexts (workspaces, code objects)
            self.launch(i)
            self.collect(i)

    def timed(self, steps, serialize=True, timing=False):
        """Wall seconds of ``steps`` steps between barrier + device sync on both sides; with ``timing``
        also (kernel ms total, launches) from HIP events around every scan launch; and the last result."""
        c0, c1 = self.ctxs
        if timing:
            for c in self.ctxs:
                c.timing(True)
                c.timing_read()
        c0.sync()
        c1.sync()
        self.team.barrier()
        t0 = time.perf_counter()
        self.launch(0)
        for i in range(1, steps):
            if serialize:
                self.ctxs[i % 2].wait_for(self.ctxs[(i - 1) % 2])
            self.launch(i)
            self.collect(i - 1)
        res = self.collect(steps - 1)
        c0.sync()
        c1.sync()
        self.team.barrier()
        dt = time.perf_counter() - t0
        kern = (0.0, 0)
        if timing:
            ms, n = 0.0, 0
            for c in self.ctxs:
                a, b = c.timing_read()
                c.timing(False)
                ms += a
                n += b
            kern = (ms, n)
        return dt, kern, res


def stream_peak(ctx, d_ptr, nbytes, reps=5, write_per_read=0.0, d_out=0):
    """Rate (B/s, read + written bytes) of a calibration stream kernel over this buffer: read-only (the
    measured read roofline), or reading it while writing ``write_per_read`` bytes per input byte contiguously
    (``stream_rw_kernel``: a same-run reference for a scan that also writes its index, not a bound)."""
    n16 = nbytes // 16 * 16

    def go():
        if write_per_read:
            ctx.stream_rw(d_ptr, n16, d_out, write_per_read)
        else:
            ctx.stream_read(d_ptr, n16)

    go()
    ctx.sync()
    ctx.timing(True)
    ctx.timing_read()
    for _ in range(reps):
        go()
    ms, n = ctx.timing_read()
    ctx.timing(False)
    return n16 * (1.0 + write_per_read) / (ms / 1e3 / max(1, n))


# ------------------------------------------------------------------------------------------ CPU baseline
_CPU_OBJ = b""


def _regex_chunk(args):
    """cpu_baseline worker: the reference's per-chunk scan (fasta.py:36-56), restated in oracle/cpu_ref, over
    the object the pool inherited at fork; returns (pid, seconds spent in the scan)."""
    from oracle import cpu_ref
    c0, c1 = args
    t0 = time.perf_counter()
    cpu_ref.fasta_chunk_pairs(_CPU_OBJ, c0, c1)
    return os.getpid(), time.perf_counter() - t0


def _delim_chunk(args):
    """cpu_baseline worker for csv/vcf: the newline offsets of one chunk (oracle/cpu_ref.delim_index)."""
    from oracle import cpu_ref
    c0, c1 = args
    t0 = time.perf_counter()
    cpu_ref.delim_index(_CPU_OBJ, c0, c1)
    return os.getpid(), time.perf_counter() - t0


def _warm(_):
    """Pool warm-up task: the worker has started and imported the oracle before the timed map."""
    from oracle import cpu_ref  # noqa: F401
    return os.getpid()


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def pool_workers():
    """Fork-pool size: every CPU this process may use, capped by the box's CPU share (OMP_NUM_THREADS=16
    on the GPU box, where os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _pool_scan(host: np.ndarray, worker_fn, chunks_per_worker: int = 8):
    """Time ``worker_fn`` over the whole object cut into chunks_per_worker x workers chunks on a fork pool.
    The pool is created and warmed (every worker started, the oracle imported) before the clock starts, and
    the object is shared with the workers copy-on-write (no per-task copy): the timed region is the scan.
    Returns (wall s, busiest worker's scan s, workers, chunks, one-core s over the same chunks)."""
    import multiprocessing as mp
    global _CPU_OBJ
    _CPU_OBJ = host
    workers = pool_workers()
    n = len(host)
    nch = max(1, chunks_per_worker * workers)
    cs = -(-n // nch)
    plan = [(i * cs, min(n, (i + 1) * cs)) for i in range(-(-n // cs))]
    with mp.get_context("fork").Pool(workers) as pool:
        pool.map(_warm, range(4 * workers), chunksize=1)
        t0 = time.perf_counter()
        res = pool.map(worker_fn, plan, chunksize=1)
        t_pool = time.perf_counter() - t0
    busy = {}
    for pid, t in res:
        busy[pid] = busy.get(pid, 0.0) + t
    t0 = time.perf_counter()
    for c in plan:
        worker_fn(c)
    t_one = time.perf_counter() - t0
    _CPU_OBJ = b""
    return t_pool, max(busy.values()), workers, len(plan), t_one


def cpu_baseline(host: np.ndarray, chunk_size: int):
    """The reference algorithm (re.finditer per chunk + split-header fix-up, fasta.py:24-63) on the host:
    (1) a warm fork pool over every usable core scanning the WHOLE object in 8 chunks per core;
    (2) one core, the same chunks; (3) the reference's default shape, parallel_config={} (sequential): the
    configs[1] chunk plan over the whole object, each chunk copied out first (the ranged GET's bytes,
    handler.py:39-42)."""
    from oracle import cpu_ref
    t_pool, t_busy, workers, nch, t_one = _pool_scan(host, _regex_chunk)
    seq_plan = cpu_ref.chunk_plan(len(host), chunk_size)
    t0 = time.perf_counter()
    for c0, c1 in seq_plan:
        data = host[c0:c1].tobytes()              # the chunk's GET body
        pairs = [(c0 + m.start(), c0 + m.end()) for m in cpu_ref._HEADER_RE.finditer(data)]
        np.array(pairs, dtype=np.uint64)
        del data
    t_seq = time.perf_counter() - t0
    n = len(host)
    seq_bytes = sum(c1 - c0 for c0, c1 in seq_plan)
    return {"value": round(n / t_pool / GiB, 3), "unit": "GiB/s", "cores": workers, "kind": "port",
            "sample": f"the whole {n / GiB:g} GiB object, {nch} chunks ({nch // workers} per core), "
                      f"re.finditer(rb'>.+(\\n)?') + fix-up per chunk (fasta.py:36-56) on a warm {workers}-process "
                      f"fork pool sharing the object (pool start-up outside the timed region)",
            "value_1core": round(n / t_one / GiB, 3),
            "speedup_vs_1core": round(t_one / t_pool, 2),
            "busiest_worker_s": round(t_busy, 4), "wall_s": round(t_pool, 4),
            "sequential_default": {"value": round(seq_bytes / t_seq / GiB, 3), "unit": "GiB/s", "cores": 1,
                                   "sample": f"the whole {n / GiB:g} GiB object, {len(seq_plan)} chunks "
                                             f"of {chunk_size} B in order (parallel_config={{}}): chunk copy + "
                                             f"regex + uint32 packing"},
            "host": host_info()}


def cpu_baseline_delim(host: np.ndarray):
    """The CPU newline index (numpy restatement of the '\\n' search CSVSlice.get / VCFSlice.get do per slice,
    csv.py:60-98, vcf.py:98-140) on the host cores, bounded sample: the first 4 GiB of the scanned range."""
    sample = host[: min(len(host), 4 << 30)]
    t_pool, t_busy, workers, nch, t_one = _pool_scan(sample, _delim_chunk)
    n = len(sample)
    return {"value": round(n / t_pool / GiB, 3), "unit": "GiB/s", "cores": workers, "kind": "port",
            "sample": f"first {n / GiB:.2f} GiB of the scanned range, {nch} chunks ({nch // workers} per core), "
                      f"numpy flatnonzero(== '\\n') per chunk on a warm {workers}-process fork pool",
            "value_1core": round(n / t_one / GiB, 3), "speedup_vs_1core": round(t_one / t_pool, 2),
            "busiest_worker_s": round(t_busy, 4), "wall_s": round(t_pool, 4), "host": host_info()}


def load_traffic(args, size, kernel):
    """(HBM bytes per scan launch, source) from --traffic-bytes or a committed rocprofv3 PMC summary of the
    same workload and per-GPU size (tools/pmc_summary.py), else (None, None)."""
    if args.traffic_bytes:
        return args.traffic_bytes, "--traffic-bytes"
    suffix = "" if args.workload == "fasta" else "_" + args.workload
    path = args.traffic_from or os.path.join(REPO, "profiles", f"latest_pmc_summary{suffix}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pmc = json.load(f)
    if pmc.get("object_bytes", size) != size or "hbm_traffic_bytes" not in pmc \
            or not pmc.get("kernel", kernel).startswith(kernel):
        return None, None
    if args.workload != "fasta" and pmc.get("index_dtype", "u64") != args.index_dtype:
        return None, None                              # a profile of the other index form
    return pmc["hbm_traffic_bytes"], os.path.relpath(os.path.realpath(path), REPO)


# ------------------------------------------------------------------------------------------ FASTA
# The FASTA index is two kernels (libdpscan: the map over 16 KiB ranges, then the placement); their HIP-event
# span is one "launch" (DP_FASTA_ONEPASS=1: round 2's one-pass look-back kernel, for A/B runs)
_ONEPASS = os.environ.get("DP_FASTA_ONEPASS", "0") not in ("", "0")
FASTA_KERNEL = "scan_kernel<FASTA>" if _ONEPASS else "map_kernel<FASTA> + fasta_place_kernel (one HIP-event span)"
FASTA_PMC_KERNELS = "scan_kernel<0" if _ONEPASS else "map_kernel<0>,fasta_place_kernel"


class FastaSpec:
    """One FASTA object and its chunk plan, split over n workers by the product's split
    (scan.objects.fasta_split: byte-balanced groups, chunks cut where a group boundary falls inside one).
    ``scan_plan`` holds the launch chunks (whole chunks, or pieces of cut ones)."""

    def __init__(self, size: int, chunks_total: int, n_workers: int, seed: int = 1):
        from dataplug_amd import synth
        from dataplug_amd.scan.objects import fasta_split
        self.size = size
        self.chunk_size = math.ceil(size / chunks_total)
        n = size // self.chunk_size
        self.plan = [(i * self.chunk_size, size if self.chunk_size == n - 1 else (i + 1) * self.chunk_size)
                     for i in range(n)]
        self.pieces, self.scan_plan, self.groups = fasta_split(self.plan, n_workers, size)
        self.obj = synth.TiledFasta(size, seed=seed)
        # the reference's uint32 index holds every offset < 2^32 (ends <= size; the synthetic object never
        # ends inside a header line); larger objects need the opt-in uint64 index (index_dtype="uint64")
        self.u64 = size > (1 << 32)


def fasta_worker(args, team, spec: FastaSpec, strong: FastaSpec | None, k: int, dev: int, keep_host: bool):
    from dataplug_amd.scan import ScanContext
    out = {"worker": k, "device": dev}
    ctxs = (ScanContext(dev), ScanContext(dev))

    def prepare(sp: FastaSpec, tag: str, gi: int):
        if gi >= len(sp.groups):
            return None
        g = sp.groups[gi]
        host = sp.obj.bytes_range(g.lo, g.buf_hi)
        d_in = ctxs[0].workspace(f"in_{tag}", len(host) + 64)
        ctxs[0].h2d(d_in.ptr, host)
        chunks = np.ascontiguousarray(np.asarray(g.chunks(sp.scan_plan), np.uint64).reshape(-1))
        nch = len(chunks) // 2
        cap = (g.hi - g.lo) // 256 + 1024
        osz = 2 * cap * (8 if sp.u64 else 4)
        d_outs = (ctxs[0].workspace(f"out_{tag}", osz), ctxs[1].workspace(f"out_{tag}", osz))

        def launch(i):
            ctxs[i % 2].fasta_index_async(d_in.ptr, len(host), g.lo, sp.size, chunks, d_outs[i % 2].ptr,
                                           sp.u64, cap)

        def collect(i):
            return ctxs[i % 2].fasta_result(nch)

        scanned = sum(p.b - p.a for p in sp.pieces[g.i0:g.i1])         # the plan's bytes (not the overlap byte)
        return {"g": g, "host": host, "d_in": d_in, "d_outs": d_outs, "steps": Steps(team, ctxs, launch, collect),
                "scanned": scanned, "chunks": chunks}

    def verify(sp: FastaSpec, st, res, i_last):
        n_pairs, pending, _ = res
        if args.no_verify:
            return None
        from oracle import dpref          # the checker (test infrastructure), outside every timed region
        g = st["g"]
        rel = [(c0 - g.lo, c1 - g.lo) for c0, c1 in g.chunks(sp.scan_plan)]
        exp = dpref.fasta_pairs(st["host"], rel)
        got = np.empty((n_pairs, 2), np.uint64 if sp.u64 else np.uint32)
        ctxs[0].d2h(got, st["d_outs"][i_last % 2].ptr)
        return bool((pending == -1).all() and np.array_equal(got.astype(np.uint64) - np.uint64(g.lo), exp))

    t0 = time.perf_counter()
    st = prepare(spec, "main", 0)                     # weak: this worker's own configs[1] object
    ss = prepare(strong, "strong", k) if strong is not None else None
    out["gen_s"] = time.perf_counter() - t0
    team.barrier()                    # every worker's uploads are done before any scan (shared-GPU rehearsals)
    S = st["steps"]
    S.warm(args.warmup)
    # (1) HIP events on each context's own stream around every scan launch: the kernel's own duration
    dt_t, (kms, kn), _ = S.timed(args.steps, timing=True)
    # (2) the K steps with each scan also waiting for the previous step's tail (the secondary `serialized`)
    dt, _, _ = S.timed(args.steps)
    # (3) the K timed steps of `value`: pipelined (no events); its last result is the one verified
    dt_ov, _, res = S.timed(args.steps, serialize=False)
    out.update(dt=dt, dt_overlap=dt_ov, kern_s=kms / 1e3 / max(1, kn), scanned=st["scanned"], pairs=res[0],
               alg_bytes=st["scanned"] + (16 if spec.u64 else 8) * res[0],
               stream_peak=stream_peak(ctxs[0], st["d_in"].ptr, st["g"].hi - st["g"].lo))
    out["verified"] = verify(spec, st, res, args.steps - 1)
    if ss is not None:
        ss["steps"].warm(args.warmup)
        dts, (sms, sn), sres = ss["steps"].timed(args.steps, timing=True)
        out["strong"] = {"dt": dts, "scanned": ss["scanned"], "pairs": sres[0], "kern_s": sms / 1e3 / max(1, sn),
                         "verified": verify(strong, ss, sres, args.steps - 1)}
    elif strong is not None:
        team.barrier()                 # no group for this worker in the strong split: keep the barriers paired
        team.barrier()
    if keep_host:
        out["host"] = st["host"]
    for c in ctxs:
        c.close()
    return out


def main_fasta(args, world, rank, devs, team):
    per_gpu = args.size or (4 << 30)
    size = per_gpu
    # weak: every GPU indexes its own configs[1] object (the reference's plan, chunk_size = size / 4, uint32
    # index) -- N x the N = 1 workload; strong: ONE such object cut over the N GPUs by the product's split
    spec = FastaSpec(size, args.chunks, 1)
    strong = None
    if world > 1 and not args.no_strong:
        strong = FastaSpec(per_gpu, args.chunks, world)
    log(f"{world} GPU(s): a {size / GiB:g} GiB FASTA per GPU, {len(spec.plan)} chunks of {spec.chunk_size} B, "
        f"{'uint64' if spec.u64 else 'uint32'} index, devices {devs} (rank {rank})")
    keep = world == 1 and not args.no_cpu_baseline
    res = run_workers(lambda k, d: fasta_worker(args, team, spec, strong, k, d, keep), devs, rank * len(devs), team)
    host = res[0].pop("host", None) if keep else None
    allres = team.gather(res)
    if allres is None:
        return
    K = args.steps
    dt_ser = max(r["dt"] for r in allres)
    dt_ov = max(r["dt_overlap"] for r in allres)
    scanned = sum(r["scanned"] for r in allres)
    pairs = sum(r["pairs"] for r in allres)
    kern = max(r["kern_s"] for r in allres)
    pipelined = dt_ov / K >= kern            # one scan at a time: a step is never shorter than the scan
    dt = dt_ov if pipelined else dt_ser
    ach = min(r["alg_bytes"] / r["kern_s"] for r in allres)
    peak_meas = min(r["stream_peak"] for r in allres)
    verified = None if args.no_verify else all(r["verified"] for r in allres)
    cpu = cpu_baseline(host, spec.chunk_size) if host is not None else None
    traffic, traffic_src = load_traffic(args, per_gpu, FASTA_PMC_KERNELS) if world == 1 else (None, None)
    strong_out = None
    if strong is not None:
        sr = [r["strong"] for r in allres if "strong" in r]
        sdt = max(r["dt"] for r in sr)
        strong_out = {"value": round(sum(r["scanned"] for r in sr) * K / sdt / GiB, 3), "unit": "GiB/s",
                      "ms_per_step": round(sdt / K * 1e3, 4), "object_bytes": strong.size,
                      "chunks": len(strong.plan), "gpus_used": len(sr),
                      "kernel_avg_us_max": round(max(r["kern_s"] for r in sr) * 1e6, 2),
                      "verified_bit_exact": None if args.no_verify else all(r["verified"] for r in sr),
                      "pieces": len(strong.pieces), "cut_chunks": sum(not p.first for p in strong.pieces),
                      "note": "fixed total: ONE configs[1] 4 GiB object with the caller's plan (chunk_size = "
                              "size/4) cut into byte-balanced groups over the same N GPUs by the product split "
                              "(scan.objects.fasta_split; chunks cut where a group boundary falls inside one) "
                              "-- the strong scaling point of SURVEY.md §8(e)"}
    r0 = allres[0]
    out = {
        "metric": "GiB/s scanned (device-resident) + offsets/s, FASTA index at 1/2/4/8 MI355X",
        "value": round(scanned * K / dt / GiB, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(dt / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"FASTA '>' header index of a {size / GiB:g} GiB synthetic object per GPU "
                               f"(BASELINE configs[1]: chunk_size={spec.chunk_size} = size/{len(spec.plan)}), "
                               f"{world} object(s)",
                   "object_bytes": size, "objects": world, "chunks": len(spec.plan), "pairs": int(pairs),
                   "index_dtype": "uint64" if spec.u64 else "uint32",
                   "parallelism": f"independent objects x{world}, "
                                  f"{'one rank per GPU (gloo for barriers)' if team.pg is not None else 'one host thread per GPU'}, "
                                  f"no collective; one object over N GPUs: the `strong` point"},
        "offsets_per_s": round(2.0 * pairs * K / dt, 1),
        "timing": "pipelined" if pipelined else "serialized",
        "serialized": {"value": round(scanned * K / dt_ser / GiB, 3), "unit": "GiB/s",
                       "ms_per_step": round(dt_ser / K * 1e3, 4),
                       "note": "the same K steps with each scan also waiting on the device for the previous "
                               "step's resolve kernel and read-back"},
        "strong": strong_out,
        "roofline": {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK, 4),
                     "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                     "kernel": FASTA_KERNEL, "kernel_avg_us": round(kern * 1e6, 2),
                     "alg_bytes_per_launch": int(r0["alg_bytes"]),
                     "alg_bytes_def": "N + 8 * H (N chunk bytes read once, H headers x two uint32 offsets)",
                     "measured_peak": round(peak_meas / 1e9, 1),
                     "frac_of_measured_peak": round(ach / peak_meas, 4),
                     "note": "per GPU (the slowest GPU's algorithmic bytes / its average scan launch); "
                             "measured_peak = read-only stream kernel over the same buffer, same run"},
        "cpu_baseline": cpu,
        "verified_bit_exact": verified,
        "gen_s": round(max(r["gen_s"] for r in allres), 2),
    }
    if world > 1:
        out["per_gpu"] = [{"worker": r["worker"], "device": r["device"], "bytes": r["scanned"],
                           "ms_per_step": round((r["dt_overlap"] if pipelined else r["dt"]) / K * 1e3, 4),
                           "kernel_avg_us": round(r["kern_s"] * 1e6, 2),
                           "verified": r["verified"]} for r in allres]
    print(json.dumps(out), flush=True)


# ------------------------------------------------------------------------------------------ CSV / VCF
def delim_worker(args, team, k, world, dev, keep_host):
    """configs[2] (csv: a 32 GiB cities.csv-shaped object per GPU, weak scaling) and configs[3] (vcf: ONE
    64 GiB VCF whose body [body_offset, size) is cut into one raw byte range per GPU, strong scaling): the
    newline index as co.preprocess builds it — uint32 low words with the ranges split at 4 GiB page
    boundaries (dp_delim_ranges out_mode 2; --index-dtype u64: plain uint64) — device-resident, timed like
    the FASTA line."""
    from dataplug_amd import synth
    from dataplug_amd.dist import rank_byte_range
    from dataplug_amd.scan import ScanContext
    from dataplug_amd.scan.objects import page_ranges
    csv_mode = args.workload == "csv"
    fmt = args.index_dtype
    size = args.size or ((32 << 30) if csv_mode else (64 << 30))
    t0 = time.perf_counter()
    obj = synth.tiled_csv(size, seed=9 + k) if csv_mode else synth.tiled_vcf(size, seed=9)
    begin, end = (0, size) if csv_mode else rank_byte_range(len(obj.head), size, k, world)
    nbytes = end - begin
    n_exp = obj.count_range(begin, end)
    ctxs = (ScanContext(dev), ScanContext(dev))
    d_buf = ctxs[0].workspace("bench_in", nbytes + 64)
    d_ptr = d_buf.ptr + (begin & 15)                       # object offset and device address congruent mod 16
    step = 4 << 30                                           # materialize + upload 4 GiB at a time
    stage = np.empty(min(step, nbytes), np.uint8)
    for p in range(begin, end, step):
        q = min(end, p + step)
        ctxs[0].h2d(d_ptr + (p - begin), obj.bytes_range(p, q, out=stage))
    del stage
    gen_s = time.perf_counter() - t0
    cap = n_exp + 1024
    item = {"u16b": 2, "u32p": 4, "u64": 8}[fmt]
    mode = {"u16b": 3, "u32p": 2, "u64": 1}[fmt]
    rg = np.ascontiguousarray(np.asarray(page_ranges(begin, end) if fmt == "u32p" else [(begin, end)],
                                         np.uint64).reshape(-1))
    nr = len(rg) // 2
    ob = ScanContext.out_bytes(cap, mode, rg)
    d_outs = (ctxs[0].workspace("bench_out", ob), ctxs[1].workspace("bench_out", ob))

    def launch(i):
        ctxs[i % 2].delim_ranges_async(d_ptr, nbytes, begin, rg, 10, 1, 0, 0, d_outs[i % 2].ptr, mode, cap)

    def collect(i):
        return ctxs[i % 2].delim_ranges_result(nr)

    two_max = ctxs[0].forms()[1]
    kernel = ("map_kernel<DELIM> + delim_place_kernel (one HIP-event span)" if nbytes <= two_max
              else "scan_kernel<DELIM> (one-pass)")
    S = Steps(team, ctxs, launch, collect)
    team.barrier()
    S.warm(args.warmup)
    dt_t, (kms, kn), _ = S.timed(args.steps, timing=True)
    dt, _, _ = S.timed(args.steps)                                         # serialized (secondary)
    dt_ov, _, (n_out, _, ends) = S.timed(args.steps, serialize=False)      # pipelined (`value`), verified
    verified = None
    if not args.no_verify:
        # every offset, against the object's analytic newline positions (synth.TiledText)
        last = d_outs[(args.steps - 1) % 2].ptr
        got = ctxs[0].d2h(np.empty(n_out, {"u16b": np.uint16, "u32p": np.uint32, "u64": np.uint64}[fmt]), last)
        page_first = [0] + [int(e) for e in ends[:-1]]          # entry index where each page range starts
        page_of = [int(rg[2 * j]) >> 32 for j in range(nr)]
        tab = ctxs[0].block_table(last, cap, rg).astype(np.int64) if fmt == "u16b" else None
        ok, i = n_out == n_exp, 0
        for piece in obj.delims_range(begin, end):
            if not ok:
                break
            seg = got[i:i + len(piece)].astype(np.uint64)
            idx = np.arange(i, i + len(piece))
            if fmt == "u32p":                                    # rebuild uint64 from the page of each entry
                j = np.searchsorted(np.asarray(page_first[1:], np.int64), idx, side="right")
                seg |= np.asarray(page_of, np.uint64)[j] << np.uint64(32)
            elif fmt == "u16b":                                  # ... from the 64 KiB block of each entry
                blk = np.searchsorted(tab, idx, side="right").astype(np.uint64) - np.uint64(1)
                seg |= (blk + np.uint64(begin >> 16)) << np.uint64(16)
            ok = np.array_equal(seg, piece)
            i += len(piece)
        verified = bool(ok and i == n_out)
        del got
    wpr = item * n_out / nbytes
    d_mix = ctxs[0].workspace("bench_mix", int(wpr * nbytes) + (1 << 20))
    out = {"dt": dt, "dt_overlap": dt_ov, "kern_s": kms / 1e3 / max(1, kn), "scanned": nbytes, "offsets": n_out,
           "kernel": kernel,
           "alg_bytes": nbytes + item * n_out + (8 * ScanContext.block_table_size(rg)[1] if fmt == "u16b" else 0),
           "verified": verified, "gen_s": gen_s, "size": size,
           "stream_peak": stream_peak(ctxs[0], d_buf.ptr, nbytes),
           "mixed_peak": stream_peak(ctxs[0], d_buf.ptr, nbytes, write_per_read=wpr, d_out=d_mix.ptr)}
    if keep_host:
        out["host"] = obj.bytes_range(begin, min(end, begin + (1 << 30)))
    for c in ctxs:
        c.close()
    return out


def main_delim(args, world, rank, devs, team):
    keep = world == 1 and not args.no_cpu_baseline
    res = run_workers(lambda k, d: delim_worker(args, team, k, world, d, keep), devs, rank * len(devs), team)
    host = res[0].pop("host", None) if keep else None
    allres = team.gather(res)
    if allres is None:
        return
    csv_mode = args.workload == "csv"
    K = args.steps
    size = allres[0]["size"]
    dt_ser = max(r["dt"] for r in allres)
    dt_ov = max(r["dt_overlap"] for r in allres)
    scanned = sum(r["scanned"] for r in allres)
    offs = sum(r["offsets"] for r in allres)
    kern = max(r["kern_s"] for r in allres)
    pipelined = dt_ov / K >= kern            # one scan at a time: a step is never shorter than the scan
    dt = dt_ov if pipelined else dt_ser
    ach = min(r["alg_bytes"] / r["kern_s"] for r in allres)
    peak_meas = min(r["stream_peak"] for r in allres)
    mixed = min(r["mixed_peak"] for r in allres)
    cpu = cpu_baseline_delim(host) if host is not None else None
    traffic, traffic_src = load_traffic(args, allres[0]["scanned"], "scan_kernel<1") if world == 1 else (None, None)
    name = "CSV" if csv_mode else "VCF"
    idx = {"u16b": "uint16 low words + 64 KiB block table", "u32p": "uint32 low words + 4 GiB pages",
           "u64": "uint64"}[args.index_dtype]
    cfg = (f"'\\n' index ({idx}), {size / GiB:g} GiB cities.csv-shaped object per GPU (BASELINE configs[2])"
           if csv_mode else
           f"'\\n' index ({idx}) of one {size / GiB:g} GiB VCF body cut into {world} part(s), one per GPU "
           f"(BASELINE configs[3])")
    out = {
        "metric": f"GiB/s scanned (device-resident) + offsets/s, {name} newline index",
        "value": round(scanned * K / dt / GiB, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(dt / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if csv_mode else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": cfg, "object_bytes": size, "scanned_bytes_per_gpu": allres[0]["scanned"],
                   "offsets_per_gpu": int(allres[0]["offsets"]),
                   "parallelism": f"independent {'objects' if csv_mode else 'body parts'} x{world}, no collective"},
        "offsets_per_s": round(offs * K / dt, 1),
        "timing": "pipelined" if pipelined else "serialized",
        "serialized": {"value": round(scanned * K / dt_ser / GiB, 3), "unit": "GiB/s",
                       "ms_per_step": round(dt_ser / K * 1e3, 4)},
        "roofline": {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK, 4),
                     "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                     "kernel": allres[0]["kernel"], "kernel_avg_us": round(kern * 1e6, 2),
                     "alg_bytes_per_launch": int(allres[0]["alg_bytes"]),
                     "alg_bytes_def": "N + %d * L (N input bytes read once, L offsets written)%s" % (
                         {"u16b": 2, "u32p": 4, "u64": 8}[args.index_dtype],
                         " + 8 B per 64 KiB block" if args.index_dtype == "u16b" else ""),
                     "measured_peak": round(peak_meas / 1e9, 1),
                     "frac_of_measured_peak": round(ach / peak_meas, 4),
                     "measured_mixed_ref": round(mixed / 1e9, 1),
                     "frac_of_mixed_ref": round(ach / mixed, 4),
                     "note": "measured_peak: read-only stream kernel (same run, same buffer); measured_mixed_ref: "
                             "the best plain streaming shape measured (stream_rw_kernel) reading the same buffer "
                             "while writing the index's bytes per input byte: a same-run reference for the "
                             "read/write mix, not a bound (reads and writes share the HBM bus)"},
        "cpu_baseline": cpu,
        "verified_bit_exact": None if args.no_verify else all(r["verified"] for r in allres),
        "gen_s": round(max(r["gen_s"] for r in allres), 2),
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    world, rank, devs, pg = launch_mode(args)
    team = Team(len(devs), pg)
    try:
        if args.workload == "fasta":
            main_fasta(args, world, rank, devs, team)
        else:
            main_delim(args, world, rank, devs, team)
    finally:
        if pg is not None:
            pg.destroy_process_group()


if __name__ == "__main__":
    main()
