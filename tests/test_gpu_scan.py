"""GPU parity: the HIP kernels (through the C ABI) against the reference's golden vectors and the oracle.

Bit-exact for every case (integer/byte work).  Sizes here finish in seconds; the BASELINE-size cases
(4 GiB FASTA, GiB-scale CSV) are in test_gpu_full_size.py.
"""
import math
import os

import numpy as np
import pytest

from dataplug_amd import synth
from dataplug_amd.scan._lib import DPScanError
from oracle import cpu_ref, dpref

pytestmark = pytest.mark.gpu


def _gpu_pairs(ctx, obj: np.ndarray, chunks, u64=False, offset=0):
    """Upload ``obj`` (optionally at a misaligned device address) and index the chunk plan."""
    buf = ctx.workspace("t_in", len(obj) + 64)
    ctx.h2d(buf.ptr + offset, obj)
    pairs, pending, cend = ctx.fasta_index(buf.ptr + offset, len(obj), 0, len(obj), chunks, u64=u64)
    assert (pending == -1).all()
    return pairs, cend


def test_golden_fuzz_and_sample(ctx, fasta_cases):
    z = fasta_cases
    bad = []
    for i in range(len(z["chunk_size"])):
        obj = z["data"][z["data_off"][i]:z["data_off"][i + 1]]
        exp = z["expected"][z["expected_off"][i]:z["expected_off"][i + 1]]
        plan = cpu_ref.chunk_plan(len(obj), int(z["chunk_size"][i]))
        pairs, cend = _gpu_pairs(ctx, obj, plan, offset=i % 16)
        if not np.array_equal(pairs.reshape(-1), exp) or len(pairs) != z["num_sequences"][i]:
            bad.append(i)
    assert not bad, f"{len(bad)} mismatching golden cases, first {bad[:5]}"


def test_golden_synthetic(ctx, fasta_cases):
    z = fasta_cases
    off = z["syn_index_off"]
    for j in range(len(z["syn_seed"])):
        a = synth.fasta(int(z["syn_size"][j]), int(z["syn_seed"][j]))
        assert synth.sha256(a) == z["syn_sha256"][j]
        pairs, _ = _gpu_pairs(ctx, a, cpu_ref.chunk_plan(len(a), int(z["syn_chunk_size"][j])))
        np.testing.assert_array_equal(pairs.reshape(-1), z["syn_index"][off[j]:off[j + 1]])


def _adversarial(kind: str, size: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, size, dtype=np.uint8)
    if kind == "long_lines":      # lines far longer than a 32 KiB unit, sparse '>'
        a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)]
        a[rng.integers(0, size, 40)] = 10
        a[rng.integers(0, size, 400)] = 62
        return a
    if kind == "no_newline":
        a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)]
        a[rng.integers(0, size, 300)] = 62
        return a
    if kind == "dense":           # '>' and '\n' everywhere (up to 6 headers per 16 bytes)
        return np.frombuffer(b">\nA", np.uint8)[rng.integers(0, 3, size)]
    if kind == "all_gt":
        return np.full(size, 62, np.uint8)
    if kind == "all_nl":
        return np.full(size, 10, np.uint8)
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["random", "long_lines", "no_newline", "dense", "all_gt", "all_nl"])
@pytest.mark.parametrize("div", [1, 3, 64, 1000])
def test_adversarial_vs_oracle(ctx, kind, div):
    a = _adversarial(kind, 3_000_017, 7)
    plan = cpu_ref.chunk_plan(len(a), math.ceil(len(a) / div))
    exp = dpref.fasta_pairs(a, plan)
    pairs, cend = _gpu_pairs(ctx, a, plan, u64=True, offset=5)
    np.testing.assert_array_equal(pairs, exp)
    # per-chunk split == per-chunk reference partials
    k = 0
    for i, (c0, c1) in enumerate(plan):
        n = len(dpref.fasta_pairs(a, [(c0, c1)]))
        k += n
        assert int(cend[i]) == k


@pytest.mark.parametrize("size,seed", [(64 << 20, 1), ((48 << 20) + 12345, 2)])
@pytest.mark.parametrize("div", [1, 4, 7, 64])
def test_synthetic_fasta_vs_oracle(ctx, size, seed, div):
    a = synth.fasta(size, seed)
    plan = cpu_ref.chunk_plan(len(a), math.ceil(len(a) / div))
    exp = dpref.fasta_pairs(a, plan)
    pairs, _ = _gpu_pairs(ctx, a, plan)
    np.testing.assert_array_equal(pairs.astype(np.uint64), exp)


def _long_header_fasta(size: int, seed: int, hmax: int) -> np.ndarray:
    """Headers as long as the sequences (1 B .. ``hmax``): about half of the 16 MiB placement blocks start inside
    a header line, some of them many 16 KiB ranges before its newline."""
    rng = np.random.default_rng(seed)
    a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)]
    a[60::61] = 10
    pos = 0
    while pos < size:
        h = int(rng.integers(1, hmax))
        a[pos] = 62
        a[pos + 1:pos + h] = 72
        if pos + h < size:
            a[pos + h] = 10
        pos += h + 1 + int(rng.integers(1, hmax))
    return a


@pytest.mark.parametrize("hmax", [300, 40 << 10, 400 << 10])
@pytest.mark.parametrize("div,u64", [(1, False), (5, True), (13, False)])
def test_blocks_starting_inside_headers(ctx, hmax, div, u64):
    """Placement blocks whose incoming line state is "inside a header" (about half of them here, some many 16 KiB
    ranges before that header's newline) resolve it by the look-back and give the oracle's pairs, in uint32 and
    uint64, with one, five and thirteen chunks."""
    a = _long_header_fasta((96 << 20) + 4097, 11 + div, hmax)
    plan = cpu_ref.chunk_plan(len(a), math.ceil(len(a) / div))
    exp = dpref.fasta_pairs(a, plan)
    pairs, _ = _gpu_pairs(ctx, a, plan, u64=u64, offset=3)
    np.testing.assert_array_equal(pairs.astype(np.uint64), exp)


def test_quirk_chunk_size_eq_num_chunks_minus_one(ctx):
    a = synth.fasta(12 * 1024 + 3, 9)
    size = len(a)
    cs = next(c for c in range(1, size) if size // c == c + 1)
    plan = cpu_ref.chunk_plan(size, cs)
    assert all(c1 == size for _, c1 in plan)          # every chunk reads to EOF: duplicates
    exp = np.frombuffer(cpu_ref.fasta_index(bytes(a), cs)[0], np.uint32)
    pairs, _ = _gpu_pairs(ctx, a, plan)
    np.testing.assert_array_equal(pairs.reshape(-1), exp)


def test_uint32_overflow_raises_like_reference(ctx):
    # a window of an object that straddles 2**32: the reference's np.array(..., uint32) raises
    a = synth.fasta(1 << 20, 3)
    base = (1 << 32) - (1 << 19)
    buf = ctx.workspace("t_in", len(a) + 64)
    ctx.h2d(buf.ptr, a)
    with pytest.raises(OverflowError):
        ctx.fasta_index(buf.ptr, len(a), base, base + len(a), [(base, base + len(a))], u64=False)
    pairs, _, _ = ctx.fasta_index(buf.ptr, len(a), base, base + len(a), [(base, base + len(a))], u64=True)
    exp = dpref.fasta_pairs(a, [(0, len(a))]) + np.uint64(base)
    np.testing.assert_array_equal(pairs, exp)


def test_pending_end_beyond_buffer(ctx):
    # the chunk ends inside a header line and the buffer stops there too: the end is reported pending
    a = np.frombuffer(b"ACGT\n>seq1 a long header line\nACGT\n", np.uint8)
    cut = 10
    buf = ctx.workspace("t_in", 64)
    ctx.h2d(buf.ptr, a[:cut])
    pairs, pending, _ = ctx.fasta_index(buf.ptr, cut, 0, len(a), [(0, cut)])
    assert pairs.shape == (1, 2) and pairs[0, 0] == 5 and pending[0] == 0
    halo = a[cut:]
    pos = ctx.find_delim_host(halo, cut, cut)
    assert pos == 29
    # same object, whole buffer: resolved on device
    pairs, _ = _gpu_pairs(ctx, a, [(0, cut)])
    assert pairs.tolist() == [[5, 30]]


@pytest.mark.parametrize("k,add", [(1, 0), (4, 1), (3, 0)])
@pytest.mark.parametrize("begin,end", [(0, None), (17, -12345)])
def test_delim_vs_oracle(ctx, k, add, begin, end):
    a = synth.csv((32 << 20) + 77, 4)
    end = len(a) if end is None else len(a) + end
    buf = ctx.workspace("t_in", len(a) + 64)
    ctx.h2d(buf.ptr + 3, a)
    got, nd = ctx.delim_index(buf.ptr + 3, len(a), 0, begin, end, 10, k, add, u64=True)
    exp, end_nd = dpref.delim(a, begin, end, 10, k, add)
    assert nd == end_nd
    np.testing.assert_array_equal(got, exp)


def test_delim_fastq_reads(ctx):
    a = synth.fastq(200_003, 5)
    got, nd = ctx.delim_index_host(a, 0, 0, len(a), delim=10, every_k=4, emit_add=1)
    assert nd == 4 * 200_003 and len(got) == 200_003
    np.testing.assert_array_equal(got, cpu_ref.delim_index(a, 0, len(a), 10, 4, 1))


def test_find_delim(ctx):
    a = np.frombuffer(b"x" * 5000 + b"\n" + b"y" * 10, np.uint8)
    assert ctx.find_delim_host(a, 100, 100) == 5100
    assert ctx.find_delim_host(a, 100, 5101) == -1


def test_two_contexts_ordered_by_ctx_wait():
    # bench.py's issue pattern: two contexts alternate, each launch behind a device-side wait on the other
    from dataplug_amd.scan import ScanContext
    a = synth.fasta((8 << 20) + 99, 11)
    plan = cpu_ref.chunk_plan(len(a), math.ceil(len(a) / 4))
    exp = dpref.fasta_pairs(a, plan)
    ctxs = (ScanContext(0), ScanContext(0))
    d = ctxs[0].workspace("in", len(a) + 64)
    ctxs[0].h2d(d.ptr, a)
    chunks = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))
    cap = len(a) // 256
    outs = [c.workspace("out", 8 * cap) for c in ctxs]
    ctxs[0].fasta_index_async(d.ptr, len(a), 0, len(a), chunks, outs[0].ptr, False, cap)
    for i in range(1, 6):
        ctxs[i % 2].wait_for(ctxs[(i - 1) % 2])
        ctxs[i % 2].fasta_index_async(d.ptr, len(a), 0, len(a), chunks, outs[i % 2].ptr, False, cap)
        n, pending, _ = ctxs[(i - 1) % 2].fasta_result(len(plan))
        got = ctxs[(i - 1) % 2].d2h(np.empty((n, 2), np.uint32), outs[(i - 1) % 2].ptr)
        assert (pending == -1).all() and np.array_equal(got.astype(np.uint64), exp)
    n, _, _ = ctxs[1].fasta_result(len(plan))
    assert n == len(exp)
    for c in ctxs:
        c.close()


def _check_plan(ctx, d, a, plan, u64=False):
    pairs, pending, cend = ctx.fasta_index(d.ptr, len(a), 0, len(a), plan, u64=u64)
    exp = dpref.fasta_pairs(a, plan)
    assert (pending == -1).all()
    np.testing.assert_array_equal(pairs.astype(np.uint64), exp)
    k = 0
    for i, (c0, c1) in enumerate(plan):
        k += len(dpref.fasta_pairs(a, [(c0, c1)]))
        assert int(cend[i]) == k, (i, plan)


def test_state_carried_between_launches():
    # no per-launch reset of the look-back descriptors or control words: changing plans (with empty
    # chunks, an all-empty plan), a delimiter scan, an overflow error and repeated plans on one context
    from dataplug_amd.scan import ScanContext
    ctx = ScanContext(0)
    try:
        a = synth.fasta((6 << 20) + 4321, 21)
        d = ctx.workspace("in", len(a) + 64)
        ctx.h2d(d.ptr, a)
        n = len(a)
        p1 = cpu_ref.chunk_plan(n, math.ceil(n / 5))
        p2 = [(0, 1 << 20), (1 << 20, 1 << 20), ((1 << 20), 3 << 20), (3 << 20, 3 << 20), (3 << 20, n)]
        p3 = [(100, 100), (2000, 2000)]
        for plan in (p1, p2, p1, p3, p2, p2, p1):
            _check_plan(ctx, d, a, plan)
        got, nd = ctx.delim_index(d.ptr, n, 0, 0, n, 10, 1, 0, u64=True)
        exp, end_nd = dpref.delim(a, 0, n, 10, 1, 0)
        assert nd == end_nd and np.array_equal(got, exp)
        _check_plan(ctx, d, a, p2)
        base = (1 << 32) - (1 << 21)                      # an overflowing launch (err bit set), then clean ones
        with pytest.raises(OverflowError):
            ctx.fasta_index(d.ptr, n, base, base + n, [(base, base + n)], u64=False)
        _check_plan(ctx, d, a, p2)
        _check_plan(ctx, d, a, p1, u64=True)
    finally:
        ctx.close()


def test_descriptor_epochs_wrap():
    # more launches than descriptor epochs (4095) on one context, alternating two objects of one size and
    # plan (same units, different descriptors): a stale descriptor read as current would change the counts
    from dataplug_amd.scan import ScanContext
    ctx = ScanContext(0)
    try:
        objs = [synth.fasta((1 << 20) + 17, s) for s in (31, 32)]
        objs.append(_adversarial("dense", (1 << 20) + 17, 33))
        plan = cpu_ref.chunk_plan(len(objs[0]), math.ceil(len(objs[0]) / 3))
        exps = [dpref.fasta_pairs(o, plan) for o in objs]
        assert len({len(e) for e in exps}) == 3
        bufs = [ctx.workspace(f"in{i}", len(o) + 64) for i, o in enumerate(objs)]
        for b, o in zip(bufs, objs):
            ctx.h2d(b.ptr, o)
        chunks = np.ascontiguousarray(np.asarray(plan, np.uint64).reshape(-1))
        cap = max(len(e) for e in exps) + 16
        out = ctx.workspace("out", 8 * cap)
        for i in range(4200):
            j = i % 3
            ctx.fasta_index_async(bufs[j].ptr, len(objs[j]), 0, len(objs[j]), chunks, out.ptr, False, cap)
            cnt, pending, _ = ctx.fasta_result(len(plan))
            assert cnt == len(exps[j]) and (pending == -1).all(), i
            if i % 700 == 0 or 4090 <= i <= 4100:
                got = ctx.d2h(np.empty((cnt, 2), np.uint32), out.ptr)
                np.testing.assert_array_equal(got.astype(np.uint64), exps[j])
    finally:
        ctx.close()


def test_two_contexts_unserialized_every_step_exact():
    """bench.py's issue pattern WITHOUT dp_ctx_wait: two contexts on one GPU, step k + 1 enqueued before step
    k is collected, two different objects (and a FASTA / newline mix) so a stale or mixed-up output shows.
    Every step's index is checked and no launch may time out (DP_ERR_TIMEOUT)."""
    from dataplug_amd.scan import ScanContext
    objs = [synth.fasta((24 << 20) + 99, 12), synth.fasta((20 << 20) + 4097, 13)]
    plans = [cpu_ref.chunk_plan(len(o), math.ceil(len(o) / 4)) for o in objs]
    exps = [dpref.fasta_pairs(o, p) for o, p in zip(objs, plans)]
    nl_exp = [dpref.delim(o, 0, len(o))[0] for o in objs]
    ctxs = (ScanContext(0), ScanContext(0))
    try:
        ds = []
        for c, o in zip(ctxs, objs):
            d = c.workspace("in", len(o) + 64)
            c.h2d(d.ptr, o)
            ds.append(d)
        chunks = [np.ascontiguousarray(np.asarray(p, np.uint64).reshape(-1)) for p in plans]
        caps = [len(o) // 8 for o in objs]
        outs = [c.workspace("out", 8 * cap) for c, cap in zip(ctxs, caps)]

        def launch(i):
            j = i % 2
            if i % 3 == 2:
                ctxs[j].delim_index_async(ds[j].ptr, len(objs[j]), 0, 0, len(objs[j]), 10, 1, 0, outs[j].ptr, True,
                                          caps[j])
            else:
                ctxs[j].fasta_index_async(ds[j].ptr, len(objs[j]), 0, len(objs[j]), chunks[j], outs[j].ptr, False,
                                          caps[j])

        def check(i):
            j = i % 2
            if i % 3 == 2:
                n, nd = ctxs[j].delim_result()
                got = ctxs[j].d2h(np.empty(n, np.uint64), outs[j].ptr)
                assert np.array_equal(got, nl_exp[j]), i
            else:
                n, pending, _ = ctxs[j].fasta_result(len(plans[j]))
                got = ctxs[j].d2h(np.empty((n, 2), np.uint32), outs[j].ptr)
                assert (pending == -1).all() and np.array_equal(got.astype(np.uint64), exps[j]), i

        launch(0)
        for i in range(1, 24):
            launch(i)
            check(i - 1)
        check(23)
    finally:
        for c in ctxs:
            c.close()


def test_concurrent_threads_one_device():
    """Several host threads launching scans on ONE GPU at the same moment (what DATAPLUG_AMD_DEVICES=0,0,0,0
    and bench.py --devices 0,0,0,0 do): every result exact, no look-back timeout."""
    import concurrent.futures as cf
    from dataplug_amd.scan import ScanContext
    objs = [synth.fasta((12 << 20) + 31 * i, 40 + i) for i in range(4)]
    plans = [cpu_ref.chunk_plan(len(o), math.ceil(len(o) / 3)) for o in objs]
    exps = [dpref.fasta_pairs(o, p) for o, p in zip(objs, plans)]

    def worker(i):
        ctx = ScanContext(0)
        try:
            d = ctx.workspace("in", len(objs[i]) + 64)
            ctx.h2d(d.ptr, objs[i])
            for _ in range(6):
                pairs, pending, _ = ctx.fasta_index(d.ptr, len(objs[i]), 0, len(objs[i]), plans[i])
                assert (pending == -1).all() and np.array_equal(pairs.astype(np.uint64), exps[i])
        finally:
            ctx.close()
        return True

    with cf.ThreadPoolExecutor(4) as ex:
        assert all(ex.map(worker, range(4)))


def test_two_processes_one_gpu():
    """Two processes scanning on the same GPU at once (torchrun ranks sharing a device): nothing in the
    library orders their grids, so the two persistent grids split the CUs between them.  Units are claimed
    by running workgroups only, so neither grid waits on a workgroup that cannot start: every scan exact,
    no look-back timeout."""
    import subprocess
    import sys
    helper = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_proc_scan.py")
    procs = [subprocess.Popen([sys.executable, helper, str(seed), "40"], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for seed in (3, 4)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    assert [p.returncode for p in procs] == [0, 0], outs


@pytest.mark.parametrize("k,add", [(1, 0), (4, 1), (3, 0)])
def test_delim_pieces_with_carry_equal_whole(ctx, k, add):
    """A stream indexed piece by piece (FASTQ.gz: inflated pieces as they come): each launch continues the
    every_k selection from the carried delimiter count, so the pieces' outputs concatenate to the whole."""
    a = synth.fastq(30_000, seed=8)
    whole, nd_whole = dpref.delim(a, 0, len(a), 10, k, add)
    rng = np.random.default_rng(5)
    cuts = np.sort(rng.choice(np.arange(1, len(a)), 9, replace=False)).tolist()
    bounds = [0] + cuts + [len(a)]
    d = ctx.workspace("t_in", len(a) + 64)
    ctx.h2d(d.ptr, a)
    got, carry = [], 0
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        out, nd, ends = ctx.delim_ranges(d.ptr + lo, hi - lo, lo, [(lo, hi)], 10, k, add, carry=carry)
        assert int(ends[-1]) == nd == int(np.count_nonzero(a[lo:hi] == 10))
        got.append(out)
        carry += nd
    assert carry == nd_whole and np.array_equal(np.concatenate(got), whole)


def test_delim_ranges_with_gaps_and_empty(ctx):
    a = synth.vcf(3 << 20, seed=12)
    d = ctx.workspace("t_in", len(a) + 64)
    ctx.h2d(d.ptr, a)
    ranges = [(0, 1000), (1000, 1000), (5000, 700_001), (700_001, 700_001), (1_000_000, 2_500_003),
              (3_000_000, len(a))]
    exp = np.concatenate([dpref.delim(a, lo, hi)[0] for lo, hi in ranges])
    got, nd, ends = ctx.delim_ranges(d.ptr, len(a), 0, ranges)
    assert np.array_equal(got, exp) and nd == len(exp)
    assert ends.tolist() == np.cumsum([len(dpref.delim(a, lo, hi)[0]) for lo, hi in ranges]).tolist()
    got4, nd4, _ = ctx.delim_ranges(d.ptr, len(a), 0, ranges, every_k=4, emit_add=1)
    assert np.array_equal(got4, exp[3::4] + np.uint64(1))


def test_delim_low_words_across_4gib_boundary(ctx):
    """out_mode 2 (paged uint32 index): object bytes straddling offset 2^32, ranges split there; the low
    words plus each page's first entry (range_end) rebuild the uint64 offsets."""
    a = synth.csv((6 << 20) + 3, seed=14)
    base = (1 << 32) - (3 << 20) - 7
    d = ctx.workspace("t_in", len(a) + 64)
    ctx.h2d(d.ptr, a)
    split = 1 << 32
    ranges = [(base, split), (split, base + len(a))]
    with pytest.raises(OverflowError):
        ctx.delim_ranges(d.ptr, len(a), base, ranges, out_mode=0)
    low, nd, ends = ctx.delim_ranges(d.ptr, len(a), base, ranges, out_mode=2)
    exp = dpref.delim(a, 0, len(a))[0] + np.uint64(base)
    page = np.zeros(nd, np.uint64)
    page[int(ends[0]):] = 1
    assert np.array_equal((page << np.uint64(32)) | low.astype(np.uint64), exp)


def _rebuild(r, mode, first):
    """uint64 offsets from an out_mode 3 (uint16 + 64 KiB table) or 4 (uint8 + 256-byte + 64 KiB tables) result."""
    from dataplug_amd.scan.objects import ByteOffsets
    if mode == 3:
        low, _, _, tab = r
        blk = np.searchsorted(tab.astype(np.int64), np.arange(len(low)), side="right").astype(np.uint64) - np.uint64(1)
        return ((blk + np.uint64(first >> 16)) << np.uint64(16)) | low.astype(np.uint64)
    low, _, _, tab, sub = r
    return ByteOffsets(low, sub, tab, first >> 8, first >> 16).to_u64()


@pytest.mark.parametrize("mode", [3, 4])
@pytest.mark.parametrize("base", [0, 1337, (1 << 32) - (5 << 20) - 3])
def test_delim_u16_blocks(ctx, base, mode):
    """out_mode 3 (uint16 low words plus the entries before every 64 KiB boundary) and out_mode 4 (uint8 low bytes,
    the low 16 bits of the entries before every 256-byte boundary, the 64 KiB table): the library splits each range
    at its first 64 KiB boundary so every later one starts a wave range.  Rebuilt offsets equal the oracle's, for
    unaligned starts, several contiguous ranges, offsets past 2^32, dense blocks (every byte a newline: the
    one-pass kernel's rescan) and empty blocks (none); the tables equal the counts the oracle's offsets give."""
    a = synth.csv((9 << 20) + 17, seed=15)
    a[(2 << 20):(2 << 20) + 70_000] = 10                     # dense: > kDenseMax events per wave range
    a[(5 << 20):(5 << 20) + 300_000] = ord("x")               # several blocks without a newline
    d = ctx.workspace("t_in", len(a) + 64)
    dp = d.ptr + (base & 15)                                   # object and device addresses congruent mod 16
    ctx.h2d(dp, a)
    n = len(a)
    with pytest.raises(Exception):
        ctx.delim_ranges(d.ptr + ((base + 1) & 15), n, base, [(base, base + n)], out_mode=mode)
    exp = dpref.delim(a, 0, n)[0] + np.uint64(base)
    for form in (dict(delim=1), dict(delim=3)):                 # line_kernel, the one-pass kernel
        ctx.set_form(**form)
        for ranges in ([(base, base + n)], [(base, base + 4097), (base + 4097, base + (3 << 20) + 5),
                                           (base + (3 << 20) + 5, base + n)], [(base, base + 65540),
                                           (base + 65540, base + n)]):
            r = ctx.delim_ranges(dp, n, base, ranges, out_mode=mode)
            low, nd, ends, tab = r[:4]
            assert nd == len(exp) and len(low) == len(exp) and ends[-1] == nd
            assert np.array_equal(_rebuild(r, mode, base), exp), (form, ranges)
            j0 = base >> 16
            bounds = np.arange(j0, ((base + n - 1) >> 16) + 1, dtype=np.uint64) << np.uint64(16)
            assert np.array_equal(tab[1:], np.searchsorted(exp, bounds[1:]).astype(np.uint64))
            if mode == 4:
                s0 = base >> 8
                sb = np.arange(s0, ((base + n - 1) >> 8) + 1, dtype=np.uint64) << np.uint64(8)
                assert np.array_equal(r[4][1:], (np.searchsorted(exp, sb[1:]) & 0xFFFF).astype(np.uint16))
    ctx.set_form(delim=0)



def _form_ctx(onepass):
    from dataplug_amd.scan import ScanContext
    c = ScanContext(0)
    assert c.get_form("fasta") == 0                       # the shipped default: map + placement kernels
    c.set_form(fasta=int(onepass))
    assert c.get_form("fasta") == int(onepass)
    return c


# sizes around the two-kernel form's geometry: 1 map group (16 ranges of 16 KiB), fewer groups than
# workgroups, one placement block (1024 ranges) +- a range, several blocks, a partial last group
_FORM_SIZES = [1, 5_000, 16 * 16384 - 7, 16 * 16384 + 1, 64 * 16 * 16384 - 1, 64 * 16 * 16384 + 16385,
               (9 << 20) + 333, (300 << 20) + 17]


@pytest.mark.parametrize("size", _FORM_SIZES)
def test_fasta_forms_equal(size):
    """The two-kernel form (the default) and the one-pass kernel give the oracle's pairs and chunk ends, on
    plans that cut ranges, groups and blocks, also through a capacity retry."""
    ctxs = [_form_ctx(False), _form_ctx(True)]
    try:
        rng = np.random.default_rng(size)
        a = synth.fasta(size, size % 97) if size > 4096 else _adversarial("dense", size, 3)
        for div in (1, 3, 64):
            plan = cpu_ref.chunk_plan(len(a), max(1, math.ceil(len(a) / div)))
            exp = dpref.fasta_pairs(a, plan)
            off = int(rng.integers(0, 16))
            for c in ctxs:
                pairs, cend = _gpu_pairs(c, a, plan, u64=bool(div == 3), offset=off)
                np.testing.assert_array_equal(pairs.astype(np.uint64), exp)
                # a capacity below the count: the kernel clamps its stores, reports the count, and the retry fits
                buf = c.workspace("t_in", len(a) + 64)
                p2, _, cend2 = c.fasta_index(buf.ptr + off, len(a), 0, len(a), plan, cap=max(1, len(exp) // 3))
                np.testing.assert_array_equal(p2.astype(np.uint64), exp)
                assert np.array_equal(cend2, cend)
    finally:
        for c in ctxs:
            c.close()


def test_repeated_launches_and_sizes():
    """Back-to-back launches of different sizes on one context: both kernels' tickets are put back for the
    next launch by the kernels themselves (no per-launch memset)."""
    c = _form_ctx(False)
    try:
        for i, size in enumerate([(40 << 20) + 1, 70_000, (40 << 20) + 1, 16 * 16384, (17 << 20) + 5] * 3):
            a = synth.fasta(size, i)
            plan = cpu_ref.chunk_plan(len(a), math.ceil(len(a) / (1 + i % 5)))
            pairs, _ = _gpu_pairs(c, a, plan, offset=i % 16)
            np.testing.assert_array_equal(pairs.astype(np.uint64), dpref.fasta_pairs(a, plan))
    finally:
        c.close()


_DELIM_FORM_IDS = {"line": 1, "one": 3}


def _delim_ctx(form, **kw):
    """A context pinned to one newline form (dp_ctx_set_form): "line" (line_kernel), "one" (the one-pass look-back
    kernel), or "auto" (the default) with its settings in kw, e.g. delim_line_max=0 so that every launch runs the
    density probe."""
    from dataplug_amd.scan import ScanContext
    c = ScanContext(0)
    assert c.get_form("delim") == 0 and c.get_form("delim_line_max") == 4 << 30 and c.get_form("delim_dense") == 20000
    if form != "auto":
        c.set_form(delim=_DELIM_FORM_IDS[form])
    c.set_form(**kw)
    return c


@pytest.mark.parametrize("size", [1, 5_000, 64 * 16384 - 3, 64 * 16384 + 16385, (7 << 20) + 11, (70 << 20) + 5])
def test_newline_forms_equal(size):
    """The newline index's two kernels (line_kernel; the one-pass look-back kernel) and the auto form's density
    probe picking either one (the other enqueued and returning at once) give the oracle's offsets in every output
    form, with every_k / emit_add / carry, on CSV rows (some ranges over line_kernel's 640-entry LDS list and the
    one-pass kernel's 1024-entry list: dense rescans), a run of newlines and newline-free spans; all of them write
    the same block table.  The removed map + placement form (round 3) is refused."""
    one, line = _delim_ctx("one"), _delim_ctx("line")
    with pytest.raises(DPScanError, match="DP_FORM_DELIM"):
        line.set_form(delim=2)
    auto_l = _delim_ctx("auto", delim_line_max=0, delim_dense=0)                # the probe always picks line
    auto_o = _delim_ctx("auto", delim_line_max=0, delim_dense=1 << 40)          # ... always the one-pass kernel
    try:
        a = synth.csv(size, seed=size % 89) if size > 4096 else np.full(size, 10, np.uint8)
        if size > (1 << 20):
            a[size // 3: size // 3 + 40_000] = 10                      # every byte a newline: dense ranges
            a[size // 2: size // 2 + 200_000] = ord("x")               # no newline for 12 ranges
        n = len(a)
        d1 = one.workspace("t_in", n + 64)
        one.h2d(d1.ptr + 3, a)
        d2 = line.workspace("t_in", n + 64)
        line.h2d(d2.ptr + 3, a)
        d3 = auto_l.workspace("t_in", n + 64)
        auto_l.h2d(d3.ptr + 3, a)
        d4 = auto_o.workspace("t_in", n + 64)
        auto_o.h2d(d4.ptr + 3, a)
        base = 3
        full = dpref.delim(a, 0, n)[0] + np.uint64(base)
        for k, add, carry in ((1, 0, 0), (4, 1, 2), (3, 0, 7)):
            sel = np.arange(len(full), dtype=np.uint64) + np.uint64(carry)
            exp = full[(sel % np.uint64(k)) == np.uint64(k - 1)] + np.uint64(add)
            for mode in (1, 0, 3, 4):
                outs = []
                for c, dp, want in ((one, d1.ptr + 3, 3), (line, d2.ptr + 3, 1), (auto_l, d3.ptr + 3, 1),
                                    (auto_o, d4.ptr + 3, 3)):
                    if mode >= 3 and (k != 1 or add != 0):
                        # the block tables count delimiters: an entry index only when every delimiter is one
                        with pytest.raises(DPScanError, match=f"out_mode {mode} needs every_k == 1"):
                            c.delim_ranges(dp, n, base, [(base, base + n)], every_k=k, emit_add=add, carry=carry,
                                           out_mode=mode)
                        continue
                    r = c.delim_ranges(dp, n, base, [(base, base + n)], every_k=k, emit_add=add, carry=carry,
                                       out_mode=mode)
                    # auto takes line_kernel for the uint8 index at every size
                    assert c.last_delim_form() == (1 if mode == 4 and c is auto_o else want)
                    outs.append(r)
                    if mode >= 3:
                        assert np.array_equal(_rebuild(r, mode, base), exp), (k, add, carry, mode)
                    else:
                        assert np.array_equal(r[0].astype(np.uint64), exp), (k, add, carry, mode)
                if not outs:
                    continue
                for o in outs[1:]:
                    assert np.array_equal(outs[0][0], o[0]) and outs[0][1] == o[1]
                    assert np.array_equal(np.asarray(outs[0][2]), np.asarray(o[2]))
                    if mode >= 3:                                 # the forms' block tables too
                        assert all(np.array_equal(x, y) for x, y in zip(outs[0][3:], o[3:]))
    finally:
        for c in (one, line, auto_l, auto_o):
            c.close()


def test_forms_alternate_on_one_context():
    """One context switching between every newline form (and both FASTA forms) launch after launch: the one-pass
    kernel's unit ticket shares a control word with the FASTA placement kernel's block ticket, which a two-kernel
    FASTA launch leaves non-zero, line_kernel's ticket parity advances with every launch, and the auto form
    enqueues line_kernel and the one-pass kernel with only the probe's pick running; every result stays exact."""
    c = _delim_ctx("auto")
    forms = [dict(delim=3), dict(delim=1), dict(delim=0, delim_line_max=0, delim_dense=1 << 40),
             dict(delim=0, delim_line_max=0, delim_dense=0), dict(delim=0, delim_line_max=4 << 30, delim_dense=20000)]
    try:
        a = synth.csv((3 << 20) + 333, seed=4)
        n = len(a)
        d = c.workspace("t_in", n + 64)
        c.h2d(d.ptr, a)
        full = dpref.delim(a, 0, n)[0]
        f = synth.fasta((2 << 20) + 5, seed=6)
        df = c.workspace("t_fa", len(f) + 64)
        c.h2d(df.ptr, f)
        plan = cpu_ref.chunk_plan(len(f), -(-len(f) // 3))
        fexp = dpref.fasta_pairs(f, plan)
        for it in range(6):
            for j, (lo, hi) in enumerate(((0, 700_000), (0, n), (1000, 900_000), (5, n - 7))):
                for mode in (1, 3, 4):
                    c.set_form(**forms[(it + j + mode) % len(forms)])
                    r = c.delim_ranges(d.ptr, n, 0, [(lo, hi)], out_mode=mode)
                    exp = full[(full >= lo) & (full < hi)]
                    got = _rebuild(r, mode, lo) if mode >= 3 else r[0]
                    assert np.array_equal(got, exp), (it, lo, hi, mode)
            if it % 2:
                c.set_form(fasta=(it // 2) % 2)
                pairs, pending, _ = c.fasta_index(df.ptr, len(f), 0, len(f), plan)
                assert (pending == -1).all() and np.array_equal(pairs.astype(np.uint64), fexp)
    finally:
        c.close()


@pytest.mark.gpu
def test_form_follows_delimiter_density():
    """The auto newline form: up to DP_FORM_DELIM_LINE_MAX bytes per launch line_kernel; above it, the density
    probe reads 256 sampled rows of THIS launch's bytes on the device and picks line_kernel for CSV-dense input
    (>= 20 delimiters per KiB), the one-pass kernel for sparser input (VCF): the choice follows each launch's own
    bytes, not the context's history (dp_last_delim_form reads the pick back).  Every launch, whichever kernel,
    equals the oracle (the split set to 1 MiB so small launches exercise both sides)."""
    c = _delim_ctx("auto", delim_line_max=1 << 20)
    try:
        objs = {"csv": synth.csv((5 << 20) + 77, seed=12), "vcf": synth.vcf((5 << 20) + 91, seed=13)}
        dens = {k: len(dpref.delim(a, 0, len(a))[0]) * 1024 / len(a) for k, a in objs.items()}
        assert dens["csv"] >= 20 > dens["vcf"], dens
        assert c.delim_form(4 << 20) == 0 and c.delim_form(1 << 20) == 1 and c.last_delim_form() == 0
        assert c.delim_form(4 << 20, out_mode=4) == 1     # the uint8 index: line_kernel at every size
        for name, lim, want in (("vcf", None, 3), ("csv", None, 1), ("csv", None, 1), ("vcf", None, 3),
                                ("vcf", 1 << 20, 1), ("csv", 1 << 20, 1), ("vcf", None, 3)):
            a = objs[name]
            n = len(a) if lim is None else lim
            d = c.workspace("t_" + name, len(a) + 64)
            c.h2d(d.ptr, a)
            r = c.delim_ranges(d.ptr, len(a), 0, [(0, n)], out_mode=1)
            assert np.array_equal(r[0], dpref.delim(a, 0, n)[0]), (name, n)
            assert c.last_delim_form() == want, (name, n, c.last_delim_form())
            r4 = c.delim_ranges(d.ptr, len(a), 0, [(0, n)], out_mode=4)
            assert c.last_delim_form() == 1 and r4[1] == len(r[0]), (name, n)
    finally:
        c.close()


def test_placed_input_buffer_probe():
    """A placed input workspace is probed at allocation (read-while-writing / read-only time of the calibration
    kernels; another candidate while above PLACEMENT_SLOW), reused while large enough, and scans like any other."""
    from dataplug_amd.scan import ScanContext
    from dataplug_amd.scan import device as sdev
    c = ScanContext(0)
    try:
        b = c.workspace("input", sdev.PLACEMENT_MIN + 123, placed=True)
        assert len(c.placements) == 1 and 1 <= len(c.placements[0]) <= sdev.PLACEMENT_TRIES
        assert all(0.5 < r < 3.0 for r in c.placements[0])
        assert len(c.placements[0]) == sdev.PLACEMENT_TRIES or c.placements[0][-1] <= sdev.PLACEMENT_SLOW
        assert c.workspace("input", 1 << 20, placed=True) is b and len(c.placements) == 1
        a = synth.fasta(3 << 20, 5)
        c.h2d(b.ptr, a)
        plan = cpu_ref.chunk_plan(len(a), len(a) // 3 + 1)
        pairs, _, _ = c.fasta_index(b.ptr, len(a), 0, len(a), plan)
        np.testing.assert_array_equal(pairs.astype(np.uint64), dpref.fasta_pairs(a, plan))
        c.workspace("small", 1 << 20, placed=True)        # below PLACEMENT_MIN: not probed
        assert len(c.placements) == 1
        assert sdev.PLACEMENT_MIN <= 4 << 30 <= sdev.PLACEMENT_MAX   # the FASTA headline's 4 GiB input is placed
    finally:
        c.close()
