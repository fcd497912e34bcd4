#!/usr/bin/env python3
"""Benchmark: the device-resident record-boundary index of BASELINE.json on 1..N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--legs fasta,csv,vcf] [--no-cpu-baseline]
    python bench.py --workload csv|vcf ...        (one newline leg alone as the headline line)

ONE JSON line (rank 0).  Its headline is BASELINE configs[1], the FASTA '>' header index; the BASELINE
configs[2] and configs[3] newline indexes ride along as the ``csv`` and ``vcf`` sub-objects of the same line
(``--legs`` picks them; a failing leg reports ``{"error": ...}`` and never drops the headline).

Workloads (synthetic bytes of the named shapes, resident in HBM before any timed region):
  * FASTA (configs[1]): every GPU indexes its own 4 GiB FASTA object with the reference's chunk plan
    ``chunk_size = size / 4`` (uint32 index): ``value`` is the WEAK-scaling rate, N x the N = 1 workload.
    ``strong`` (N > 1): ONE such object's plan cut over the N GPUs by the product split
    (``scan.objects.fasta_split``: byte-balanced groups, chunks cut where a boundary falls inside one, no
    collective; the reference runs chunks as independent map jobs, preprocess.py:39-51).
  * CSV (configs[2]): a 32 GiB cities.csv-shaped object per GPU (weak), the newline index as co.preprocess
    stores it (u8s: uint8 low bytes + 256-byte counts + 64 KiB block table, dp_delim_ranges out_mode 4).
  * VCF (configs[3]): ONE 64 GiB VCF whose body is cut into one byte part per GPU (strong: the 1/2/4/8-GPU
    curve of north_star), same index form.

One step = on every GPU, one scan call over its bytes: FASTA = dp_fasta_index_async + dp_fasta_result (the
chunk-table check, the two scan kernels -- map_kernel<FASTA> over 16 KiB ranges, then fasta_place_kernel --,
the split-header resolve kernel, the read-back of count / pending / chunk ends); newline = dp_delim_ranges
(one launch: the lockstep line_kernel for the stored u8s form at every size; for the other forms (--index-dtype) up
to 4 GiB, above it the kernel a density probe picks on the device from the launch's own bytes -- line_kernel for
CSV-dense input, the one-pass look-back scan_kernel for sparser; the kernel that ran, dp_last_delim_form, is named in
each leg's roofline).  The index stays in HBM (the H2D/D2H-inclusive end-to-end
rate is DESIGN.md §6).  Steps
alternate between two contexts and step k + 1 is enqueued before step k's result is collected; the library
runs one scan at a time per GPU (its scan stream), so ``value`` is this pipelined rate provided
``ms_per_step`` >= the scan's own average span (checked; a pipelined step measured below the span counts at the span,
``timing: "kernel-bound"``); the ``serialized`` rate (each scan also waiting for the previous step's tail) is
always reported next to it.

Launch modes (the same worker code in both):
  * ``python bench.py --gpus N``: one process, one host thread per GPU (``--devices 0,0`` maps workers to
    devices explicitly, e.g. to rehearse the multi-GPU split on one GPU);
  * ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``: one rank per GPU; barriers and
    the final gather go over a gloo CPU group, RCCL is never initialised (nothing is exchanged).

At N = 1 the line also carries two end-to-end sub-objects (tools/e2e_legs.py; never ``value``): ``e2e`` --
co.preprocess() of the configs[1] FASTA and of a configs[2]-shaped CSV from host memory to host memory (ranged GETs,
pinned staging, H2D, scan, D2H, index PUT) over an in-process store and over the loopback HTTP server in its own
process, with the stage split -- and ``fastq`` -- configs[4], a FASTQ.gz's per-read index end to end; every stored
index read back and checked.

Also in the line: per leg the scan's average span from HIP events on the device's scan stream (-> roofline:
algorithmic bytes / span vs 8 TB/s; ``traffic`` from a committed rocprofv3 PMC summary of the same command),
the same run's read-only calibration kernel (``measured_peak``, measured behind a barrier with no worker
scanning; null when workers share a device), for the newline legs a same-run mixed read/write reference, every
offset verified after the timed loops, and at N = 1 the reference algorithm on the host cores (cpu_baseline,
pool sized from the cgroup CPU quota).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import resource
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12   # B/s, MI355X spec (MI355X_MICROARCH.md §Chip-level parameters)
GiB = float(1 << 30)
LEGS = ("fasta", "csv", "vcf")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=list(LEGS), default="fasta",
                   help="the headline leg: fasta = configs[1] (default); csv = configs[2]; vcf = configs[3]")
    p.add_argument("--legs", default=None,
                   help="comma-separated legs in the line (default with --workload fasta: fasta,csv,vcf; "
                        "otherwise the workload alone); the first non-headline legs become sub-objects")
    p.add_argument("--size", type=int, default=None,
                   help="bytes of the headline leg (per GPU: fasta 4 GiB, csv 32 GiB; vcf: the object, 64 GiB)")
    p.add_argument("--fasta-size", type=int, default=4 << 30, help="fasta leg: bytes per GPU")
    p.add_argument("--csv-size", type=int, default=32 << 30, help="csv leg: bytes per GPU")
    p.add_argument("--vcf-size", type=int, default=64 << 30, help="vcf leg: object bytes (cut over the GPUs)")
    p.add_argument("--chunks", type=int, default=4, help="FASTA map chunks per object (chunk_size = size / chunks)")
    p.add_argument("--index-dtype", choices=["u8s", "u16b", "u32p", "u64"], default="u8s",
                   help="csv/vcf newline index form: u8s = uint8 low bytes + 256-byte counts + 64 KiB block table, "
                        "u16b = uint16 low words + 64 KiB block table, u32p = uint32 low words + 4 GiB page counts, "
                        "u64 = plain uint64")
    p.add_argument("--devices", default=None,
                   help="comma-separated device of each worker / local rank (default 0..N-1); e.g. 0,0,0,0 "
                        "rehearses the multi-GPU split on one GPU")
    p.add_argument("--no-strong", action="store_true", help="skip the fixed-total (strong scaling) FASTA point")
    p.add_argument("--fasta-onepass", action="store_true",
                   help="A/B: the FASTA index with the one-pass look-back kernel (dp_ctx_set_form) instead of map + placement")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the end-to-end `e2e` and `fastq` sub-objects (N = 1)")
    p.add_argument("--e2e-fasta-size", type=int, default=4 << 30, help="e2e leg: the configs[1] FASTA's bytes")
    p.add_argument("--e2e-csv-size", type=int, default=4 << 30, help="e2e leg: the configs[2]-shaped CSV's bytes")
    p.add_argument("--fastq-tiles", type=int, default=16, help="fastq leg: copies of the 65,536-read tile")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--traffic-bytes", type=float, default=None,
                   help="HBM bytes per headline scan launch from a rocprofv3 --pmc pass (overrides --traffic-from)")
    p.add_argument("--traffic-from", default=None,
                   help="pmc_summary.json (tools/pmc_summary.py) of the headline leg: FETCH_SIZE x2 (gfx950) "
                        "+ WRITE_SIZE per scan launch (default profiles/latest_pmc_summary[_<leg>].json)")
    a = p.parse_args(argv)
    legs = a.legs.split(",") if a.legs else (list(LEGS) if a.workload == "fasta" else [a.workload])
    if a.workload not in legs:
        legs = [a.workload] + legs
    bad = [x for x in legs if x not in LEGS]
    if bad:
        p.error(f"unknown leg(s) {bad}")
    a.legs = [a.workload] + [x for x in legs if x != a.workload]
    return a


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def peak_rss_gib() -> float:
    """Peak resident set of this process so far (ru_maxrss: KiB on Linux)."""
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / float(1 << 20), 3)


# ------------------------------------------------------------------------------------------ team of workers
class Team:
    """The workers of one run: host threads of this process (one per GPU), or this process as one rank of
    a torch.distributed.run launch (gloo CPU group: barriers and gathers only, never RCCL).  ``devices``:
    every worker's device, all ranks (a device listed twice = workers sharing a GPU, a rehearsal)."""

    def __init__(self, n_local: int, pg=None, local_devices=()):
        self._tb = threading.Barrier(n_local)
        self.pg = pg
        devs = list(local_devices)
        if pg is not None:
            out = [None] * pg.get_world_size()
            pg.all_gather_object(out, devs)
            devs = [d for ds in out for d in ds]
        self.devices = devs
        self.shared = len(set(devs)) < len(devs)

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


# host-side verification holds one group's bytes at a time per slot: at most this many workers at once
_VERIFY_SLOTS = threading.Semaphore(2)


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


def calibrate(team, fn):
    """Run a calibration ``fn()`` with no worker scanning: behind a team barrier (every worker's timed steps
    are over) and followed by one, so no worker starts anything else on the GPU meanwhile.  When workers
    share a device (a rehearsal) the calibrations of one device would overlap each other: None."""
    team.barrier()
    v = None if team.shared else fn()
    team.barrier()
    return v


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


def cgroup_cpu_quota():
    """(CPUs the cgroup quota allows or None when unlimited/absent, the raw setting): cgroup v2 cpu.max
    ("<quota> <period>" or "max <period>"), else cgroup v1 cpu.cfs_quota_us / cpu.cfs_period_us."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            raw = f.read().strip()
        q, per = raw.split()[:2]
        return (None if q == "max" else int(q) / int(per)), f"cpu.max={raw}"
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return (None if q <= 0 else q / per), f"cfs_quota_us={q} cfs_period_us={per}"
    except (OSError, ValueError):
        return None, "no cgroup cpu controller found"


def pool_plan():
    """(fork-pool size, host facts): every CPU this process may run on (affinity) capped by the cgroup CPU
    quota; with no quota (unlimited), by OMP_NUM_THREADS -- the box's stated CPU share (16 per GPU), where
    os.cpu_count() and the affinity report the whole machine."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota, raw = cgroup_cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if quota is not None:
        n, basis = max(1, min(aff, int(math.floor(quota + 1e-9)))), "cgroup CPU quota"
    elif omp > 0:
        n, basis = max(1, min(aff, omp)), "OMP_NUM_THREADS (the cgroup sets no CPU quota)"
    else:
        n, basis = aff, "affinity (no cgroup quota, no OMP_NUM_THREADS)"
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
               "cgroup_cpu": raw, "cgroup_quota_cpus": None if quota is None else round(quota, 2),
               "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "pool_processes": n, "pool_basis": basis}


def _pool_scan(host: np.ndarray, worker_fn, chunks_per_worker: int = 8):
    """Time ``worker_fn`` over the whole sample cut into chunks_per_worker x workers chunks on a fork pool.
    The pool is created and warmed (every worker started, the oracle imported) before the clock starts, and
    the bytes are shared with the workers copy-on-write (no per-task copy): the timed region is the scan.
    Returns (wall s, busiest worker's scan s, workers, chunks, one-core s over the same chunks, host facts)."""
    import multiprocessing as mp
    global _CPU_OBJ
    _CPU_OBJ = host
    workers, hinfo = pool_plan()
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
    return t_pool, max(busy.values()), workers, len(plan), t_one, hinfo


def cpu_baseline(host: np.ndarray, chunk_size: int):
    """The reference algorithm (re.finditer per chunk + split-header fix-up, fasta.py:24-63) on the host:
    (1) a warm fork pool over every core the cgroup allows scanning the WHOLE object in 8 chunks per core;
    (2) one core, the same chunks; (3) the reference's default shape, parallel_config={} (sequential): the
    configs[1] chunk plan over the whole object, each chunk copied out first (the ranged GET's bytes,
    handler.py:39-42)."""
    from oracle import cpu_ref
    t_pool, t_busy, workers, nch, t_one, hinfo = _pool_scan(host, _regex_chunk)
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
            "host": hinfo}


def cpu_baseline_delim(sample: np.ndarray):
    """The CPU newline index (numpy restatement of the '\\n' search CSVSlice.get / VCFSlice.get do per slice,
    csv.py:60-98, vcf.py:98-140) on the host cores over a bounded sample of the scanned range."""
    t_pool, t_busy, workers, nch, t_one, hinfo = _pool_scan(sample, _delim_chunk)
    n = len(sample)
    return {"value": round(n / t_pool / GiB, 3), "unit": "GiB/s", "cores": workers, "kind": "port",
            "sample": f"first {n / GiB:.2f} GiB of the scanned range, {nch} chunks ({nch // workers} per core), "
                      f"numpy flatnonzero(== '\\n') per chunk on a warm {workers}-process fork pool",
            "value_1core": round(n / t_one / GiB, 3), "speedup_vs_1core": round(t_one / t_pool, 2),
            "busiest_worker_s": round(t_busy, 4), "wall_s": round(t_pool, 4), "host": hinfo}


def load_traffic(args, leg, size, kernel, index_dtype=None):
    """(HBM bytes per scan launch, source) from --traffic-bytes (headline leg only) or the committed rocprofv3
    PMC summary of the same leg and per-GPU size (profiles/latest_pmc_summary[_<leg>].json, written by
    tools/pmc_summary.py), else (None, None)."""
    if leg == args.workload and args.traffic_bytes:
        return args.traffic_bytes, "--traffic-bytes"
    suffix = "" if leg == "fasta" else "_" + leg
    path = (args.traffic_from if leg == args.workload else None) or \
        os.path.join(REPO, "profiles", f"latest_pmc_summary{suffix}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pmc = json.load(f)
    if pmc.get("object_bytes", size) != size or "hbm_traffic_bytes" not in pmc \
            or not pmc.get("kernel", kernel).startswith(kernel):
        return None, None
    if leg != "fasta" and pmc.get("index_dtype", "u64") != index_dtype:
        return None, None                              # a profile of the other index form
    src = pmc.get("source") or os.path.relpath(os.path.realpath(path), REPO)
    return pmc["hbm_traffic_bytes"], src


# ------------------------------------------------------------------------------------------ FASTA
# The FASTA index is two kernels (libdpscan: the map over 16 KiB ranges, then the placement); their HIP-event
# span is one "launch" (--fasta-onepass: round 2's one-pass look-back kernel, for A/B runs, dp_ctx_set_form)
def fasta_kernel_names(args):
    """(label, rocprof kernel names of one launch) of the FASTA form the run uses."""
    if args.fasta_onepass:
        return "scan_kernel<FASTA>", "scan_kernel<0"
    return "map_kernel<FASTA> + fasta_place_kernel (one HIP-event span)", "map_kernel,fasta_place_kernel"


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


def fasta_worker(args, team, spec: FastaSpec, strong: FastaSpec | None, k: int, dev: int):
    from dataplug_amd.scan import ScanContext
    out = {"worker": k, "device": dev}
    ctxs = (ScanContext(dev), ScanContext(dev))
    if args.fasta_onepass:
        for c in ctxs:
            c.set_form(fasta=1)

    def prepare(sp: FastaSpec, tag: str, gi: int):
        if gi >= len(sp.groups):
            return None
        g = sp.groups[gi]
        host = sp.obj.bytes_range(g.lo, g.buf_hi)
        d_in = ctxs[0].workspace(f"in_{tag}", len(host) + 64, placed=True)
        ctxs[0].h2d(d_in.ptr, host)
        n_buf = len(host)
        del host                        # the host copy is not kept: verify() regenerates the bytes it checks
        chunks = np.ascontiguousarray(np.asarray(g.chunks(sp.scan_plan), np.uint64).reshape(-1))
        nch = len(chunks) // 2
        cap = (g.hi - g.lo) // 256 + 1024
        osz = 2 * cap * (8 if sp.u64 else 4)
        d_outs = (ctxs[0].workspace(f"out_{tag}", osz), ctxs[1].workspace(f"out_{tag}", osz))

        def launch(i):
            ctxs[i % 2].fasta_index_async(d_in.ptr, n_buf, g.lo, sp.size, chunks, d_outs[i % 2].ptr, sp.u64, cap)

        def collect(i):
            return ctxs[i % 2].fasta_result(nch)

        scanned = sum(p.b - p.a for p in sp.pieces[g.i0:g.i1])         # the plan's bytes (not the overlap byte)
        return {"g": g, "d_in": d_in, "d_outs": d_outs, "steps": Steps(team, ctxs, launch, collect),
                "scanned": scanned, "chunks": chunks}

    def verify(sp: FastaSpec, st, res, i_last):
        n_pairs, pending, _ = res
        if args.no_verify:
            return None
        from oracle import dpref          # the checker (test infrastructure), outside every timed region
        g = st["g"]
        rel = [(c0 - g.lo, c1 - g.lo) for c0, c1 in g.chunks(sp.scan_plan)]
        got = np.empty((n_pairs, 2), np.uint64 if sp.u64 else np.uint32)
        ctxs[0].d2h(got, st["d_outs"][i_last % 2].ptr)
        with _VERIFY_SLOTS:
            exp = dpref.fasta_pairs(sp.obj.bytes_range(g.lo, g.buf_hi), rel)
        return bool((pending == -1).all() and np.array_equal(got.astype(np.uint64) - np.uint64(g.lo), exp))

    t0 = time.perf_counter()
    st = prepare(spec, "main", 0)                     # weak: this worker's own configs[1] object
    ss = prepare(strong, "strong", k) if strong is not None else None
    out["gen_s"] = time.perf_counter() - t0
    team.barrier()                    # every worker's uploads are done before any scan (shared-GPU rehearsals)
    S = st["steps"]
    S.warm(args.warmup)
    # (1) HIP events on the device's scan stream around every scan launch: the kernels' own span
    dt_t, (kms, kn), _ = S.timed(args.steps, timing=True)
    # (2) the K steps with each scan also waiting for the previous step's tail (the secondary `serialized`)
    dt, _, _ = S.timed(args.steps)
    # (3) the K timed steps of `value`: pipelined (no events); its last result is the one verified
    dt_ov, _, res = S.timed(args.steps, serialize=False)
    nbytes = st["g"].hi - st["g"].lo
    out.update(dt=dt, dt_overlap=dt_ov, kern_s=kms / 1e3 / max(1, kn), scanned=st["scanned"], pairs=res[0],
               alg_bytes=st["scanned"] + (16 if spec.u64 else 8) * res[0],
               stream_peak=calibrate(team, lambda: stream_peak(ctxs[0], st["d_in"].ptr, nbytes)))
    if ss is not None:
        ss["steps"].warm(args.warmup)
        dts, (sms, sn), sres = ss["steps"].timed(args.steps, timing=True)
        out["strong"] = {"dt": dts, "scanned": ss["scanned"], "pairs": sres[0], "kern_s": sms / 1e3 / max(1, sn),
                         "verified": verify(strong, ss, sres, args.steps - 1)}
    elif strong is not None:
        team.barrier()                 # no group for this worker in the strong split: keep the barriers paired
        team.barrier()
    out["verified"] = verify(spec, st, res, args.steps - 1)
    out["placement"] = list(ctxs[0].placements)
    for c in ctxs:
        c.close()
    out["rss_gib"] = peak_rss_gib()
    return out


def leg_fasta(args, world, rank, devs, team):
    """The configs[1] leg: every worker's result (rank 0: all ranks'; others: None) and the specs."""
    per_gpu = args.size if (args.size and args.workload == "fasta") else args.fasta_size
    # weak: every GPU indexes its own configs[1] object (the reference's plan, chunk_size = size / 4, uint32
    # index) -- N x the N = 1 workload; strong: ONE such object cut over the N GPUs by the product's split
    spec = FastaSpec(per_gpu, args.chunks, 1)
    strong = None
    if world > 1 and not args.no_strong:
        strong = FastaSpec(per_gpu, args.chunks, world)
    log(f"fasta: {world} GPU(s), a {per_gpu / GiB:g} GiB FASTA per GPU, {len(spec.plan)} chunks of "
        f"{spec.chunk_size} B, {'uint64' if spec.u64 else 'uint32'} index, devices {devs} (rank {rank})")
    res = run_workers(lambda k, d: fasta_worker(args, team, spec, strong, k, d), devs, rank * len(devs), team)
    return team.gather(res), spec, strong


def report_fasta(args, world, team, allres, spec, strong, t_leg):
    from dataplug_amd.scan import device as sdev
    K = args.steps
    dt_ser = max(r["dt"] for r in allres)
    dt_ov = max(r["dt_overlap"] for r in allres)
    scanned = sum(r["scanned"] for r in allres)
    pairs = sum(r["pairs"] for r in allres)
    kern = max(r["kern_s"] for r in allres)
    # one scan at a time per GPU: a step is never shorter than its scan.  A pipelined run measured below the scan's
    # own event-timed span (which carries the events' cost) counts every step at that span ("kernel-bound")
    pipelined = dt_ov / K >= kern
    dt = dt_ov if pipelined else K * kern
    ach = min(r["alg_bytes"] / r["kern_s"] for r in allres)
    peaks = [r["stream_peak"] for r in allres]
    peak_meas = None if any(p is None for p in peaks) else min(peaks)
    verified = None if args.no_verify else all(r["verified"] for r in allres)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        host = spec.obj.bytes_range(0, spec.size)        # regenerated: the worker kept no host copy
        cpu = cpu_baseline(host, spec.chunk_size)
        del host
    fasta_label, fasta_pmc = fasta_kernel_names(args)
    traffic, traffic_src = load_traffic(args, "fasta", spec.size, fasta_pmc) if world == 1 else (None, None)
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
        "config": {"workload": f"FASTA '>' header index of a {spec.size / GiB:g} GiB synthetic object per GPU "
                               f"(BASELINE configs[1]: chunk_size={spec.chunk_size} = size/{len(spec.plan)}), "
                               f"{world} object(s)",
                   "object_bytes": spec.size, "objects": world, "chunks": len(spec.plan), "pairs": int(pairs),
                   "index_dtype": "uint64" if spec.u64 else "uint32",
                   "parallelism": f"independent objects x{world}, "
                                  f"{'one rank per GPU (gloo for barriers)' if team.pg is not None else 'one host thread per GPU'}, "
                                  f"no collective; one object over N GPUs: the `strong` point"},
        "offsets_per_s": round(2.0 * pairs * K / dt, 1),
        "timing": "pipelined" if pipelined else "kernel-bound",
        "serialized": {"value": round(scanned * K / dt_ser / GiB, 3), "unit": "GiB/s",
                       "ms_per_step": round(dt_ser / K * 1e3, 4),
                       "note": "the same K steps with each scan also waiting on the device for the previous "
                               "step's resolve kernel and read-back"},
        "strong": strong_out,
        "roofline": {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK, 4),
                     "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                     "kernel": fasta_label, "kernel_avg_us": round(kern * 1e6, 2),
                     "alg_bytes_per_launch": int(r0["alg_bytes"]),
                     "alg_bytes_def": "N + 8 * H (N chunk bytes read once, H headers x two uint32 offsets)",
                     "measured_peak": None if peak_meas is None else round(peak_meas / 1e9, 1),
                     "frac_of_measured_peak": None if peak_meas is None else round(ach / peak_meas, 4),
                     "note": "per GPU (the slowest GPU's algorithmic bytes / its average scan span); measured_peak"
                             " = read-only stream kernel over the same buffer, same run, behind a barrier with no "
                             "worker scanning (null when workers share a GPU)"},
        "cpu_baseline": cpu,
        "verified_bit_exact": verified,
        "input_placement": {"probes": [r.get("placement") for r in allres], "note": "per worker, per placed input buffer: read-while-writing / read-only time ratio of each candidate allocation (ScanContext.workspace(placed=True): above PLACEMENT_SLOW = the slow placement mode, another buffer tried, at most PLACEMENT_TRIES, the best kept)",
                            "slow_above": sdev.PLACEMENT_SLOW, "tries": sdev.PLACEMENT_TRIES},
        "gen_s": round(max(r["gen_s"] for r in allres), 2),
        "leg_s": round(t_leg, 2),
        "rss_gib_max_worker": max(r["rss_gib"] for r in allres),
    }
    if world > 1:
        out["per_gpu"] = [{"worker": r["worker"], "device": r["device"], "bytes": r["scanned"],
                           "ms_per_step": round(max(r["dt_overlap"], K * r["kern_s"]) / K * 1e3, 4),
                           "kernel_avg_us": round(r["kern_s"] * 1e6, 2),
                           "verified": r["verified"]} for r in allres]
    return out


# ------------------------------------------------------------------------------------------ CSV / VCF
def _verify_blocked(obj, begin, end, got, tab, n_out):
    """Every offset of a uint16 + 64 KiB-block-table index against the object's analytic newline positions
    (synth.TiledText): the low words equal the expected offsets' low 16 bits, and every table entry equals the
    number of expected offsets below its boundary (0 for a boundary at or below ``begin``); together they pin
    every full offset."""
    j0 = begin >> 16
    nb = len(tab)
    i, nxt = 0, j0                                   # offsets checked so far; the next boundary to check
    for piece in obj.delims_range(begin, end):
        if len(piece) == 0:
            continue
        if i + len(piece) > n_out or not np.array_equal(got[i:i + len(piece)],
                                                        (piece & np.uint64(0xFFFF)).astype(np.uint16)):
            return False
        hi = min(int(piece[-1]) >> 16, j0 + nb - 1)  # boundaries at or below this piece's last offset
        if hi >= nxt:
            bnd = np.arange(nxt, hi + 1, dtype=np.uint64) << np.uint64(16)
            exp = np.uint64(i) + np.searchsorted(piece, bnd).astype(np.uint64)
            if not np.array_equal(tab[nxt - j0:hi + 1 - j0], exp):
                return False
            nxt = hi + 1
        i += len(piece)
    # boundaries past the last offset: every entry before them
    return bool(i == n_out and (tab[nxt - j0:] == np.uint64(n_out)).all())


def _verify_bytes(obj, begin, end, got, sub, tab, n_out):
    """Every offset of a uint8 + 256-byte + 64 KiB table index (out_mode 4) against the object's analytic newline
    positions: the low bytes equal the expected offsets' low 8 bits, every 256-byte entry equals the low 16 bits of
    the expected offsets below its boundary, and the block table as in _verify_blocked; together they pin every
    offset."""
    s0, j0 = begin >> 8, begin >> 16
    ns, nb = len(sub), len(tab)
    i, nxt_s, nxt_j = 0, s0 + (1 if begin & 0xFF else 0), j0 + (1 if begin & 0xFFFF else 0)
    if (begin & 0xFF and sub[0] != 0) or (begin & 0xFFFF and tab[0] != 0):
        return False
    for piece in obj.delims_range(begin, end):
        if len(piece) == 0:
            continue
        if i + len(piece) > n_out or not np.array_equal(got[i:i + len(piece)],
                                                        (piece & np.uint64(0xFF)).astype(np.uint8)):
            return False
        hs = min(int(piece[-1]) >> 8, s0 + ns - 1)
        if hs >= nxt_s:
            bnd = np.arange(nxt_s, hs + 1, dtype=np.uint64) << np.uint64(8)
            exp = (np.uint64(i) + np.searchsorted(piece, bnd).astype(np.uint64)) & np.uint64(0xFFFF)
            if not np.array_equal(sub[nxt_s - s0:hs + 1 - s0].astype(np.uint64), exp):
                return False
            nxt_s = hs + 1
        hj = min(int(piece[-1]) >> 16, j0 + nb - 1)
        if hj >= nxt_j:
            bnd = np.arange(nxt_j, hj + 1, dtype=np.uint64) << np.uint64(16)
            if not np.array_equal(tab[nxt_j - j0:hj + 1 - j0], np.uint64(i) + np.searchsorted(piece, bnd).astype(np.uint64)):
                return False
            nxt_j = hj + 1
        i += len(piece)
    return bool(i == n_out and (sub[nxt_s - s0:].astype(np.uint64) == np.uint64(n_out & 0xFFFF)).all()
                and (tab[nxt_j - j0:] == np.uint64(n_out)).all())


def delim_worker(args, team, leg, k, world, dev):
    """configs[2] (csv: a 32 GiB cities.csv-shaped object per GPU, weak scaling) and configs[3] (vcf: ONE
    64 GiB VCF whose body [body_offset, size) is cut into one raw byte range per GPU, strong scaling): the
    newline index as co.preprocess builds it (u8s: uint8 low bytes + 256-byte counts + 64 KiB block table,
    dp_delim_ranges out_mode 4; --index-dtype u16b / u32p / u64: the other forms) -- device-resident, timed like the
    FASTA leg."""
    from dataplug_amd import synth
    from dataplug_amd.dist import rank_byte_range
    from dataplug_amd.scan import ScanContext
    from dataplug_amd.scan.objects import page_ranges
    csv_mode = leg == "csv"
    fmt = args.index_dtype
    head = args.size if (args.size and args.workload == leg) else None
    size = head or (args.csv_size if csv_mode else args.vcf_size)
    t0 = time.perf_counter()
    obj = synth.tiled_csv(size, seed=9 + k) if csv_mode else synth.tiled_vcf(size, seed=9)
    begin, end = (0, size) if csv_mode else rank_byte_range(len(obj.head), size, k, world)
    nbytes = end - begin
    n_exp = obj.count_range(begin, end)
    ctxs = (ScanContext(dev), ScanContext(dev))
    d_buf = ctxs[0].workspace("bench_in", nbytes + 64, placed=True)
    d_ptr = d_buf.ptr + (begin & 15)                       # object offset and device address congruent mod 16
    step = 2 << 30                                           # materialize + upload 2 GiB at a time
    stage = np.empty(min(step, max(1, nbytes)), np.uint8)
    for p in range(begin, end, step):
        q = min(end, p + step)
        ctxs[0].h2d(d_ptr + (p - begin), obj.bytes_range(p, q, out=stage))
    del stage
    gen_s = time.perf_counter() - t0
    cap = n_exp + 1024
    item = {"u8s": 1, "u16b": 2, "u32p": 4, "u64": 8}[fmt]
    mode = {"u8s": 4, "u16b": 3, "u32p": 2, "u64": 1}[fmt]
    rg = np.ascontiguousarray(np.asarray(page_ranges(begin, end) if fmt == "u32p" else [(begin, end)],
                                         np.uint64).reshape(-1))
    nr = len(rg) // 2
    ob = ScanContext.out_bytes(cap, mode, rg)
    d_outs = (ctxs[0].workspace("bench_out", ob), ctxs[1].workspace("bench_out", ob))

    def launch(i):
        ctxs[i % 2].delim_ranges_async(d_ptr, nbytes, begin, rg, 10, 1, 0, 0, d_outs[i % 2].ptr, mode, cap)

    def collect(i):
        return ctxs[i % 2].delim_ranges_result(nr)

    S = Steps(team, ctxs, launch, collect)
    team.barrier()
    S.warm(args.warmup)
    dt_t, (kms, kn), _ = S.timed(args.steps, timing=True)
    # the kernel the timed launches ran: line_kernel up to 4 GiB per launch, above it the density probe's pick from
    # the launch's own bytes (dp_last_delim_form reads it back with each launch's results)
    kernel = " / ".join(ScanContext.DELIM_FORMS[f] for f in sorted({c.last_delim_form() for c in ctxs}))
    dt, _, _ = S.timed(args.steps)                                         # serialized (secondary)
    dt_ov, _, (n_out, _, ends) = S.timed(args.steps, serialize=False)      # pipelined (`value`), verified
    wpr = item * n_out / max(1, nbytes)
    d_mix = ctxs[0].workspace("bench_mix", int(wpr * nbytes) + (1 << 20))
    peak = calibrate(team, lambda: stream_peak(ctxs[0], d_buf.ptr, nbytes))
    mixed = calibrate(team, lambda: stream_peak(ctxs[0], d_buf.ptr, nbytes, write_per_read=wpr, d_out=d_mix.ptr))
    verified, t_ver = None, time.perf_counter()
    if not args.no_verify:
        last = d_outs[(args.steps - 1) % 2].ptr
        got = ctxs[0].d2h(np.empty(n_out, {"u8s": np.uint8, "u16b": np.uint16, "u32p": np.uint32, "u64": np.uint64}[fmt]),
                          last)
        with _VERIFY_SLOTS:
            if fmt == "u8s":
                verified = n_out == n_exp and _verify_bytes(obj, begin, end, got, ctxs[0].sub_table(last, cap, rg),
                                                            ctxs[0].block_table(last, cap, rg, 4), n_out)
            elif fmt == "u16b":
                verified = n_out == n_exp and _verify_blocked(obj, begin, end, got, ctxs[0].block_table(last, cap, rg),
                                                              n_out)
            else:
                page_first = [0] + [int(e) for e in ends[:-1]]      # entry index where each page range starts
                page_of = [int(rg[2 * j]) >> 32 for j in range(nr)]
                ok, i = n_out == n_exp, 0
                for piece in obj.delims_range(begin, end):
                    if not ok:
                        break
                    seg = got[i:i + len(piece)].astype(np.uint64)
                    if fmt == "u32p":                             # rebuild uint64 from the page of each entry
                        idx = np.arange(i, i + len(piece))
                        j = np.searchsorted(np.asarray(page_first[1:], np.int64), idx, side="right")
                        seg |= np.asarray(page_of, np.uint64)[j] << np.uint64(32)
                    ok = np.array_equal(seg, piece)
                    i += len(piece)
                verified = bool(ok and i == n_out)
        del got
    t_ver = time.perf_counter() - t_ver
    out = {"worker": k, "device": dev, "dt": dt, "dt_overlap": dt_ov, "kern_s": kms / 1e3 / max(1, kn),
           "scanned": nbytes, "offsets": n_out, "kernel": kernel,
           "alg_bytes": nbytes + item * n_out + (8 * ScanContext.block_table_size(rg)[1] if fmt in ("u8s", "u16b") else 0)
                        + (2 * ScanContext.sub_table_size(rg)[1] if fmt == "u8s" else 0),
           "verified": verified, "verify_s": t_ver, "gen_s": gen_s, "size": size, "wpr": wpr,
           "stream_peak": peak, "mixed_peak": mixed, "range": (begin, end), "placement": list(ctxs[0].placements)}
    for c in ctxs:
        c.close()
    out["rss_gib"] = peak_rss_gib()
    return out


def leg_delim(args, world, rank, devs, team, leg):
    res = run_workers(lambda k, d: delim_worker(args, team, leg, k, world, d), devs, rank * len(devs), team)
    return team.gather(res)


def report_delim(args, world, team, allres, leg, t_leg, headline: bool):
    from dataplug_amd.scan import device as sdev
    csv_mode = leg == "csv"
    K = args.steps
    size = allres[0]["size"]
    dt_ser = max(r["dt"] for r in allres)
    dt_ov = max(r["dt_overlap"] for r in allres)
    scanned = sum(r["scanned"] for r in allres)
    offs = sum(r["offsets"] for r in allres)
    kern = max(r["kern_s"] for r in allres)
    # one scan at a time per GPU: a step is never shorter than its scan.  A pipelined run measured below the scan's
    # own event-timed span (which carries the events' cost) counts every step at that span ("kernel-bound")
    pipelined = dt_ov / K >= kern
    dt = dt_ov if pipelined else K * kern
    ach = min(r["alg_bytes"] / r["kern_s"] for r in allres)
    peaks = [r["stream_peak"] for r in allres]
    mixes = [r["mixed_peak"] for r in allres]
    peak_meas = None if any(p is None for p in peaks) else min(peaks)
    mixed = None if any(p is None for p in mixes) else min(mixes)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from dataplug_amd import synth
        obj = synth.tiled_csv(size, seed=9) if csv_mode else synth.tiled_vcf(size, seed=9)
        b0, b1 = allres[0]["range"]
        sample = obj.bytes_range(b0, min(b1, b0 + (1 << 30)))     # bounded sample: the first GiB scanned
        cpu = cpu_baseline_delim(sample)
        del sample
    k = allres[0]["kernel"]
    pmc_kernel = "line_kernel<" if k.startswith("line_kernel") else "scan_kernel<1"
    traffic, traffic_src = (load_traffic(args, leg, allres[0]["scanned"], pmc_kernel, args.index_dtype)
                            if world == 1 else (None, None))
    name = "CSV" if csv_mode else "VCF"
    idx = {"u8s": "uint8 low bytes + 256-byte counts + 64 KiB block table",
           "u16b": "uint16 low words + 64 KiB block table", "u32p": "uint32 low words + 4 GiB pages",
           "u64": "uint64"}[args.index_dtype]
    cfg = (f"'\\n' index ({idx}), {size / GiB:g} GiB cities.csv-shaped object per GPU (BASELINE configs[2])"
           if csv_mode else
           f"'\\n' index ({idx}) of one {size / GiB:g} GiB VCF body cut into {world} part(s), one per GPU "
           f"(BASELINE configs[3])")
    verified = None if args.no_verify else all(r["verified"] for r in allres)
    out = {
        "metric": f"GiB/s scanned (device-resident) + offsets/s, {name} newline index",
        "value": round(scanned * K / dt / GiB, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "ms_per_step": round(dt / K * 1e3, 4),
        "scaling": "weak" if csv_mode else "strong",
        "config": {"workload": cfg, "object_bytes": size, "scanned_bytes_per_gpu": allres[0]["scanned"],
                   "offsets_per_gpu": int(allres[0]["offsets"]),
                   "parallelism": f"independent {'objects' if csv_mode else 'body parts'} x{world}, no collective"},
        "offsets_per_s": round(offs * K / dt, 1),
        "timing": "pipelined" if pipelined else "kernel-bound",
        "serialized": {"value": round(scanned * K / dt_ser / GiB, 3), "unit": "GiB/s",
                       "ms_per_step": round(dt_ser / K * 1e3, 4)},
        "roofline": {"bound": "hbm", "achieved": round(ach / 1e9, 1), "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK, 4),
                     "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                     "kernel": allres[0]["kernel"], "kernel_avg_us": round(kern * 1e6, 2),
                     "alg_bytes_per_launch": int(allres[0]["alg_bytes"]),
                     "alg_bytes_def": "N + %d * L (N input bytes read once, L offsets written)%s%s" % (
                         {"u8s": 1, "u16b": 2, "u32p": 4, "u64": 8}[args.index_dtype],
                         " + 2 B per 256 B" if args.index_dtype == "u8s" else "",
                         " + 8 B per 64 KiB block" if args.index_dtype in ("u8s", "u16b") else ""),
                     "measured_peak": None if peak_meas is None else round(peak_meas / 1e9, 1),
                     "frac_of_measured_peak": None if peak_meas is None else round(ach / peak_meas, 4),
                     "measured_mixed_ref": None if mixed is None else round(mixed / 1e9, 1),
                     "frac_of_mixed_ref": None if mixed is None else round(ach / mixed, 4),
                     "note": "measured_peak: read-only stream kernel (same run, same buffer); measured_mixed_ref: "
                             "the best plain streaming shape measured (stream_rw_kernel) reading the same buffer "
                             "while writing the index's bytes per input byte: a same-run reference for the "
                             "read/write mix, not a bound (reads and writes share the HBM bus); both behind a "
                             "barrier with no worker scanning, null when workers share a GPU"},
        "cpu_baseline": cpu,
        "verified_every_offset": verified,
        "input_placement": {"probes": [r.get("placement") for r in allres], "note": "per worker, per placed input buffer: read-while-writing / read-only time ratio of each candidate allocation (ScanContext.workspace(placed=True): above PLACEMENT_SLOW = the slow placement mode, another buffer tried, at most PLACEMENT_TRIES, the best kept)",
                            "slow_above": sdev.PLACEMENT_SLOW, "tries": sdev.PLACEMENT_TRIES},
        "gen_s": round(max(r["gen_s"] for r in allres), 2),
        "verify_s": round(max(r["verify_s"] for r in allres), 2),
        "leg_s": round(t_leg, 2),
        "rss_gib_max_worker": max(r["rss_gib"] for r in allres),
    }
    if headline:
        out.update(steps=K, warmup=args.warmup, higher_is_better=True, vs_baseline=None, dtype="u8",
                   data="synthetic", verified_bit_exact=verified)
    if world > 1:
        out["per_gpu"] = [{"worker": r["worker"], "device": r["device"], "bytes": r["scanned"],
                           "kernel_avg_us": round(r["kern_s"] * 1e6, 2), "verified": r["verified"]} for r in allres]
    return out


# ------------------------------------------------------------------------------------------ main
def run_leg(args, world, rank, devs, team, leg, headline):
    t0 = time.perf_counter()
    if leg == "fasta":
        allres, spec, strong = leg_fasta(args, world, rank, devs, team)
        if allres is None:
            return None
        return report_fasta(args, world, team, allres, spec, strong, time.perf_counter() - t0)
    allres = leg_delim(args, world, rank, devs, team, leg)
    if allres is None:
        return None
    return report_delim(args, world, team, allres, leg, time.perf_counter() - t0, headline)


def main(argv=None):
    args = parse(argv)
    world, rank, devs, pg = launch_mode(args)
    team = Team(len(devs), pg, devs)
    t_all = time.perf_counter()
    try:
        head = run_leg(args, world, rank, devs, team, args.workload, True)   # the headline: errors propagate
        for leg in args.legs[1:]:
            try:
                sub = run_leg(args, world, rank, devs, team, leg, False)
            except Exception as e:            # a failing extra leg never drops the headline line
                log(f"leg {leg} failed: {type(e).__name__}: {e}")
                sub = {"error": f"{type(e).__name__}: {e}"}
                if pg is not None:            # the other ranks may wait in a barrier of the failed leg
                    raise
                team._tb.reset()              # a failed worker aborted the threads' barrier
            if head is not None:
                head[leg] = sub
        if world == 1 and not args.no_e2e and head is not None:
            sys.path.insert(0, os.path.join(REPO, "tools"))
            import e2e_legs
            budgets = {"e2e": 90.0, "fastq": 45.0}
            for name, fn in (("e2e", lambda: e2e_legs.e2e_leg(args.e2e_fasta_size, args.e2e_csv_size,
                                                               verify_blocked=_verify_blocked,
                                                               verify_bytes=_verify_bytes,
                                                               verify=not args.no_verify, log=log)),
                             ("fastq", lambda: e2e_legs.fastq_leg(tiles=args.fastq_tiles, verify=not args.no_verify,
                                                                  log=log))):
                try:
                    sub = fn()
                    sub["budget_s"] = budgets[name]
                    sub["fits_in_driver_run"] = bool(sub["leg_s"] <= budgets[name])
                except Exception as e:        # an end-to-end leg never drops the headline
                    log(f"leg {name} failed: {type(e).__name__}: {e}")
                    sub = {"error": f"{type(e).__name__}: {e}"}
                head[name] = sub
        if head is not None:
            rss = [head.get("rss_gib_max_worker", 0.0)] + [(head.get(x) or {}).get("rss_gib_max_worker", 0.0)
                                                           for x in args.legs[1:]]
            head["peak_rss_gib"] = max([peak_rss_gib()] + [r or 0.0 for r in rss])
            head["bench_wall_s"] = round(time.perf_counter() - t_all, 2)
            print(json.dumps(head), flush=True)
    finally:
        if pg is not None:
            pg.destroy_process_group()


if __name__ == "__main__":
    main()
