#!/usr/bin/env python3
"""Benchmark: device-resident FASTA header-index scan (BASELINE.json configs[1]) on 1..N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size BYTES] [--no-cpu-baseline]
    python bench.py --workload csv|vcf ...    (BASELINE configs[2] / configs[3]: newline index)

One step = one whole co.preprocess(chunk_size=size/4) equivalent over one synthetic 4 GiB FASTA object
that is already resident in HBM: chunk-plan upload, the single-pass scan kernel, the split-header
resolve kernel and the read-back of the pair count / per-chunk state (the index itself stays in HBM;
the H2D/D2H-inclusive end-to-end rate is reported separately).

Steps are issued the way a caller indexing a stream of objects would: two scan contexts (streams)
alternate, and step k + 1 is enqueued before step k's result is collected, so one step's host round trip
hides behind the next step's scan.  Every step does the whole pass and reads back its result.  `value`
comes from K such steps whose scans may overlap on the GPU (the next object's scan starts on the CUs the
previous one's last workgroups leave idle); `serialized` repeats the K steps with each scan waiting on the
device for the previous one.

Multi-GPU (``torch.distributed.run --nproc-per-node N``): one process per GPU, each indexing its own
object (independent objects/chunks, no collective on the data path; weak scaling).  Barrier + device
sync bracket the K timed steps; the max time over ranks is reported.

Also measured inside this run: the scan kernel's average duration from HIP events on its own stream
over the K serialized launches (-> roofline), and, on rank 0 at N = 1, the reference algorithm on the
host cores (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
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
                   help="object bytes (default 4 GiB fasta, 32 GiB csv, 64 GiB vcf)")
    p.add_argument("--chunks", type=int, default=4, help="chunk_size = ceil(size / chunks) (fasta_example.py)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--traffic-bytes", type=float, default=None,
                   help="HBM bytes per scan launch from a rocprofv3 --pmc pass (overrides --traffic-from)")
    p.add_argument("--traffic-from", default=None,
                   help="pmc_summary.json (tools/pmc_summary.py) of this same command: FETCH_SIZE x2 (gfx950) "
                        "+ WRITE_SIZE per scan-kernel launch (default profiles/latest_pmc_summary[_<workload>].json)")
    return p.parse_args()


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # any launch by torch.distributed.run (even one rank) takes the RCCL path the N > 1 runs take
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(local)
        dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = dist_mod
    return world, rank, local, dist


def barrier(dist, local):
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize(local)


def max_over_ranks(dist, local, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, local, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def _regex_chunk(args):
    """cpu_baseline worker: the reference's per-chunk scan (fasta.py:36-56), restated in oracle/cpu_ref."""
    from oracle import cpu_ref
    c0, c1 = args
    return len(cpu_ref.fasta_chunk_pairs(_CPU_OBJ, c0, c1))


_CPU_OBJ = b""


def cpu_baseline(host: np.ndarray, chunk_size: int):
    """The reference algorithm (re.finditer per chunk + fix-up) on the host cores, bounded sample."""
    import multiprocessing as mp
    global _CPU_OBJ
    sample = min(len(host), 1 << 30)                 # bounded sample: the object's first GiB
    _CPU_OBJ = host[:sample].tobytes()
    cs = max(1, min(chunk_size, sample // 64))       # fan chunks out over a fork pool
    plan = [(i * cs, (i + 1) * cs) for i in range(sample // cs)]
    cores = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        pool.map(_regex_chunk, plan, chunksize=1)
    t_pool = time.perf_counter() - t0
    one = _CPU_OBJ[: 256 << 20]
    t0 = time.perf_counter()
    from oracle import cpu_ref
    cpu_ref.fasta_chunk_pairs(one, 0, len(one))
    t_one = time.perf_counter() - t0
    scanned = len(plan) * cs
    return {"value": round(scanned / t_pool / GiB, 3), "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": f"first {scanned / GiB:.2f} GiB of the object, {len(plan)} chunks of {cs} B, "
                      f"re.finditer(rb'>.+(\\n)?') + fix-up per chunk (fasta.py:36-56) over a fork pool",
            "value_1core": round(len(one) / t_one / GiB, 3)}


def load_traffic(args, size):
    """(HBM bytes per scan launch, source) from --traffic-bytes or a committed rocprofv3 PMC summary of the
    same workload (tools/pmc_summary.py), else (None, None)."""
    if args.traffic_bytes:
        return args.traffic_bytes, "--traffic-bytes"
    suffix = "" if args.workload == "fasta" else "_" + args.workload
    path = args.traffic_from or os.path.join(REPO, "profiles", f"latest_pmc_summary{suffix}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pmc = json.load(f)
    kernel = "scan_kernel<0" if args.workload == "fasta" else "scan_kernel<1"
    if pmc.get("object_bytes", size) != size or "hbm_traffic_bytes" not in pmc \
            or not pmc.get("kernel", kernel).startswith(kernel):
        return None, None
    return pmc["hbm_traffic_bytes"], os.path.relpath(os.path.realpath(path), REPO)


def _delim_chunk(args):
    """cpu_baseline worker for csv/vcf: the newline offsets of one chunk (oracle/cpu_ref.delim_index)."""
    from oracle import cpu_ref
    c0, c1 = args
    return len(cpu_ref.delim_index(_CPU_OBJ, c0, c1))


def cpu_baseline_delim(host: np.ndarray):
    """The CPU newline index (numpy restatement of the '\\n' search CSVSlice.get / VCFSlice.get do per slice,
    csv.py:60-98, vcf.py:98-140) on the host cores, bounded sample."""
    import multiprocessing as mp
    global _CPU_OBJ
    _CPU_OBJ = host[: min(len(host), 1 << 30)]
    cs = max(1, len(_CPU_OBJ) // 64)
    plan = [(i * cs, (i + 1) * cs) for i in range(len(_CPU_OBJ) // cs)]
    cores = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        pool.map(_delim_chunk, plan, chunksize=1)
    t_pool = time.perf_counter() - t0
    from oracle import cpu_ref
    one = _CPU_OBJ[: 256 << 20]
    t0 = time.perf_counter()
    cpu_ref.delim_index(one)
    t_one = time.perf_counter() - t0
    scanned = len(plan) * cs
    return {"value": round(scanned / t_pool / GiB, 3), "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": f"first {scanned / GiB:.2f} GiB of the scanned range, {len(plan)} chunks of {cs} B, "
                      f"numpy flatnonzero(== '\\n') per chunk over a fork pool",
            "value_1core": round(len(one) / t_one / GiB, 3)}


def main_delim(args, world, rank, local, dist):
    """BASELINE configs[2] (csv: a 32 GiB cities.csv-shaped object per GPU, weak scaling) and configs[3]
    (vcf: ONE 64 GiB VCF whose body [body_offset, size) is cut into one raw byte range per GPU, strong
    scaling): the uint64 newline index (dp_delim_index), device-resident, timed like the FASTA line."""
    from dataplug_amd import synth
    from dataplug_amd.scan import ScanContext

    def log(msg):
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)

    csv_mode = args.workload == "csv"
    size = args.size or ((32 << 30) if csv_mode else (64 << 30))
    t0 = time.perf_counter()
    obj = synth.tiled_csv(size, seed=9 + rank) if csv_mode else synth.tiled_vcf(size, seed=9)
    if csv_mode:
        begin, end = 0, size
    else:
        from dataplug_amd.dist import rank_byte_range
        begin, end = rank_byte_range(len(obj.head), size, rank, world)   # body [body_offset, size), vcf.py:19-67
    nbytes = end - begin
    n_exp = obj.count_range(begin, end)
    ctx = ScanContext(local)
    ctx2 = ScanContext(local)
    d_in = ctx.workspace("bench_in", nbytes + 64)
    step = 4 << 30                                           # materialize + upload 4 GiB at a time
    stage = np.empty(min(step, nbytes), np.uint8)
    for p in range(begin, end, step):
        q = min(end, p + step)
        ctx.h2d(d_in.ptr + (p - begin), obj.bytes_range(p, q, out=stage))
        log(f"uploaded {q - begin} / {nbytes} B")
    del stage
    gen_s = time.perf_counter() - t0
    cap = n_exp + 1024
    ctxs = (ctx, ctx2)
    d_outs = (ctx.workspace("bench_out", 8 * cap), ctx2.workspace("bench_out", 8 * cap))

    def launch(i):
        ctxs[i % 2].delim_index_async(d_in.ptr, nbytes, begin, begin, end, 10, 1, 0, d_outs[i % 2].ptr, True, cap)

    def collect(i):
        return ctxs[i % 2].delim_result()

    for i in range(max(2, args.warmup)):
        launch(i)
        collect(i)

    def run_steps(serialize: bool):
        barrier(dist, local)
        ctx.sync()
        ctx2.sync()
        t0 = time.perf_counter()
        launch(0)
        for i in range(1, args.steps):
            if serialize:
                ctxs[i % 2].wait_for(ctxs[(i - 1) % 2])
            launch(i)
            collect(i - 1)
        res = collect(args.steps - 1)
        ctx.sync()
        ctx2.sync()
        barrier(dist, local)
        return time.perf_counter() - t0, res

    for c in ctxs:
        c.timing(True)
        c.timing_read()
    dt_ser, _ = run_steps(serialize=True)
    kern_ms, launches = 0.0, 0
    for c in ctxs:
        ms, n = c.timing_read()
        c.timing(False)
        kern_ms += ms
        launches += n
    dt, (n_out, _) = run_steps(serialize=False)
    d_out = d_outs[(args.steps - 1) % 2]
    log(f"timed {args.steps} steps: {dt:.3f} s, {n_out} offsets")

    dt_max = max_over_ranks(dist, local, dt)
    dt_ser_max = max_over_ranks(dist, local, dt_ser)
    total_bytes = sum_over_ranks(dist, local, float(nbytes) * args.steps)
    total_offsets = sum_over_ranks(dist, local, float(n_out) * args.steps)
    kern_avg_max = max_over_ranks(dist, local, kern_ms / 1e3 / max(1, launches))

    verified = None
    if not args.no_verify:
        # every offset, against the object's analytic newline positions (synth.TiledText)
        got = ctx.d2h(np.empty(n_out, np.uint64), d_out.ptr)
        ok, i = n_out == n_exp, 0
        for piece in obj.delims_range(begin, end):
            if not ok:
                break
            ok = np.array_equal(got[i:i + len(piece)], piece)
            i += len(piece)
        verified = bool(ok and i == n_out)
        del got
        verified = bool(sum_over_ranks(dist, local, float(verified)) == world)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_delim(obj.bytes_range(begin, min(end, begin + (1 << 30))))

    traffic, traffic_src = load_traffic(args, nbytes)
    if rank == 0:
        alg_bytes = nbytes + 8.0 * n_out                # N input bytes read once + one uint64 per newline
        achieved = alg_bytes / kern_avg_max
        name = "CSV" if csv_mode else "VCF"
        cfg = ("'\\n' index (uint64), 32 GiB cities.csv-shaped object per GPU (BASELINE configs[2])" if csv_mode else
               f"'\\n' index (uint64) of one {size / GiB:g} GiB VCF body cut into {world} part(s), one per GPU "
               f"(BASELINE configs[3])")
        if args.size and csv_mode:
            cfg = cfg.replace("32 GiB", f"{size / GiB:g} GiB")
        out = {
            "metric": f"GiB/s scanned (device-resident) + offsets/s, {name} newline index",
            "value": round(total_bytes / dt_max / GiB, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if csv_mode else "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": cfg, "object_bytes": size, "scanned_bytes_per_gpu": nbytes,
                       "offsets_per_gpu": int(n_out),
                       "parallelism": f"independent {'objects' if csv_mode else 'body parts'} x{world}, "
                                      f"no collective"},
            "offsets_per_s": round(total_offsets / dt_max, 1),
            "serialized": {"value": round(total_bytes / dt_ser_max / GiB, 3), "unit": "GiB/s",
                           "ms_per_step": round(dt_ser_max / args.steps * 1e3, 4),
                           "note": "same K steps, each scan waiting on the device for the previous one"},
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src,
                         "kernel": "scan_kernel<DELIM>", "kernel_avg_us": round(kern_avg_max * 1e6, 2),
                         "alg_bytes_per_launch": int(alg_bytes)},
            "cpu_baseline": cpu,
            "verified_bit_exact": verified,
            "gen_s": round(gen_s, 2),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    world, rank, local, dist = init_dist(args)
    if args.workload != "fasta":
        return main_delim(args, world, rank, local, dist)
    if args.size is None:
        args.size = 4 << 30
    from dataplug_amd import synth
    from dataplug_amd.scan import ScanContext

    ctx = ScanContext(local)
    ctx2 = ScanContext(local)       # second stream + workspace: step k+1 is queued while step k's result is read
    size = args.size
    chunk_size = math.ceil(size / args.chunks)
    plan = [(i * chunk_size, size if chunk_size == size // chunk_size - 1 else (i + 1) * chunk_size)
            for i in range(size // chunk_size)]
    chunks = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))

    # synthetic object for this rank (seeded; repeated non-power-of-two base block), resident in HBM
    t0 = time.perf_counter()
    host = synth.tiled_fasta_host(size, seed=1 + rank)
    gen_s = time.perf_counter() - t0
    d_in = ctx.workspace("bench_in", size + 64)
    ctx.h2d(d_in.ptr, host)
    cap = size // 256 + 1024
    ctxs = (ctx, ctx2)
    d_outs = (ctx.workspace("bench_out", 8 * cap), ctx2.workspace("bench_out", 8 * cap))

    def launch(i):
        ctxs[i % 2].fasta_index_async(d_in.ptr, size, 0, size, chunks, d_outs[i % 2].ptr, False, cap)

    def collect(i):
        return ctxs[i % 2].fasta_result(len(plan))

    for i in range(max(2, args.warmup)):            # warms both contexts (workspaces, code objects)
        launch(i)
        collect(i)

    def run_steps(serialize: bool):
        """K steps; returns (wall seconds, last result).  Step k + 1 is enqueued on the other context's
        stream before step k's result is collected, so the host round trip of one step hides behind the
        next step's scan.  serialize: step k + 1 waits on the device for step k (no kernel overlap)."""
        barrier(dist, local)
        ctx.sync()
        ctx2.sync()
        t0 = time.perf_counter()
        launch(0)
        for i in range(1, args.steps):
            if serialize:
                ctxs[i % 2].wait_for(ctxs[(i - 1) % 2])
            launch(i)
            collect(i - 1)
        res = collect(args.steps - 1)
        ctx.sync()
        ctx2.sync()
        barrier(dist, local)
        return time.perf_counter() - t0, res

    # (1) serialized steps, HIP events on each context's own stream around every scan launch: the scan
    #     kernel's own duration (roofline.achieved), and the throughput without any kernel overlap
    for c in ctxs:
        c.timing(True)
        c.timing_read()
    dt_ser, _ = run_steps(serialize=True)
    kern_ms, launches = 0.0, 0
    for c in ctxs:
        ms, n = c.timing_read()
        c.timing(False)
        kern_ms += ms
        launches += n
    # (2) the K timed steps of `value`: consecutive objects' scans may overlap on the GPU (the next one
    #     starts on the CUs the previous one's last workgroups leave idle)
    dt, (n_pairs, pending, cend) = run_steps(serialize=False)
    d_out = d_outs[(args.steps - 1) % 2]

    dt_max = max_over_ranks(dist, local, dt)
    dt_ser_max = max_over_ranks(dist, local, dt_ser)
    total_bytes = sum_over_ranks(dist, local, float(size) * args.steps)
    total_offsets = sum_over_ranks(dist, local, 2.0 * n_pairs * args.steps)
    kern_avg_s = kern_ms / 1e3 / max(1, launches)
    kern_avg_max = max_over_ranks(dist, local, kern_avg_s)

    verified = None
    if not args.no_verify and rank == 0:
        from oracle import dpref
        exp = dpref.fasta_pairs(host, plan)
        got = np.empty((n_pairs, 2), np.uint32)
        ctx.d2h(got, d_out.ptr)
        verified = bool(np.array_equal(got.astype(np.uint64), exp))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(host, chunk_size)

    traffic, traffic_src = load_traffic(args, size)

    if rank == 0:
        alg_bytes = size + 8.0 * n_pairs            # N input bytes read once + 8 B per (start, end) pair
        achieved = alg_bytes / kern_avg_max
        value = total_bytes / dt_max / GiB
        out = {
            "metric": "GiB/s scanned (device-resident) + offsets/s, FASTA index at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"FASTA '>' header index, {size / GiB:g} GiB synthetic object per GPU, "
                                   f"chunk_size=size/{args.chunks} (BASELINE configs[1])",
                       "object_bytes": size, "chunks": len(plan), "pairs": int(n_pairs),
                       "parallelism": f"independent objects x{world}, no collective"},
            "offsets_per_s": round(total_offsets / dt_max, 1),
            "serialized": {"value": round(total_bytes / dt_ser_max / GiB, 3), "unit": "GiB/s",
                           "ms_per_step": round(dt_ser_max / args.steps * 1e3, 4),
                           "note": "same K steps, each scan waiting on the device for the previous one"},
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 4),
                         "traffic": None if traffic is None else int(traffic),
                         "traffic_source": traffic_src,
                         "kernel": "scan_kernel<FASTA>", "kernel_avg_us": round(kern_avg_max * 1e6, 2),
                         "alg_bytes_per_launch": int(alg_bytes)},
            "cpu_baseline": cpu,
            "verified_bit_exact": verified,
            "gen_s": round(gen_s, 2),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
