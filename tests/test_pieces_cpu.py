"""The sub-chunk multi-GPU split of the FASTA index (scan.objects.fasta_pieces / stitch_pieces) on CPU.

Each piece is "scanned" the way one GPU launch scans it — as an independent chunk [a, end) with an empty line
state at a and header ends resolved over the whole object (oracle/cpu_ref.fasta_chunk_pairs, the reference's
per-chunk algorithm, fasta.py:24-56) — and the stitched pairs must equal the reference's pairs of the whole,
uncut chunks.  The GPU side of the same path runs in tests/test_gpu_dropin.py and tools/fuzz_gpu.py."""
import math

import numpy as np
import pytest

from dataplug_amd.scan.objects import fasta_pieces, fasta_split, stitch_pieces
from oracle import cpu_ref


def _soup(rng, size):
    p_gt, p_nl = rng.uniform(0, 0.3), rng.uniform(0, 0.3)
    cls = rng.choice(3, size=size, p=[p_gt, p_nl, 1 - p_gt - p_nl])
    out = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size)].copy()
    out[cls == 0] = 62
    out[cls == 1] = 10
    return out


def _records(rng, size):
    parts, total = [], 0
    hmax = int(rng.choice([3, 40, 2000, 20000]))
    wmax = int(rng.choice([1, 60, 3000]))
    while total < size:
        h = b">" * int(rng.integers(1, 3)) + b"h" * int(rng.integers(0, hmax)) + b"\n"
        body = np.frombuffer(b"ACGT>", np.uint8)[rng.integers(0, 5, int(rng.integers(0, 4 * wmax + 1)))]
        w = max(1, int(rng.integers(1, wmax + 1)))
        rec = h + b"".join(body[i:i + w].tobytes() + b"\n" for i in range(0, len(body), w))
        parts.append(rec)
        total += len(rec)
    return np.frombuffer(b"".join(parts)[:size], np.uint8).copy()


def _plan(rng, size):
    r = rng.random()
    if r < 0.15 and size <= 20000:                       # the cs == num_chunks - 1 quirk (handler.py:36-38)
        cs = int(math.isqrt(size))
        while cs > 1 and size // cs != cs + 1:
            cs -= 1
        if cs >= 1 and size // cs == cs + 1:
            return cpu_ref.chunk_plan(size, cs)
    cs = max(1, math.ceil(size / int(rng.integers(1, 9))))
    return cpu_ref.chunk_plan(size, cs)


def _emulate(obj: bytes, plan, n_groups):
    """What fasta_index_object does with the per-GPU launches replaced by the reference's per-chunk scan."""
    pieces, scan_plan, groups = fasta_split(plan, n_groups, len(obj))
    assert [(p.a, p.end) for p in pieces] == scan_plan
    per_piece, first_nl = [], {}
    for k, p in enumerate(pieces):
        pairs = np.array(cpu_ref.fasta_chunk_pairs(obj, p.a, p.end), np.uint64).reshape(-1, 2)
        per_piece.append(pairs)
        if not p.first:
            nl = obj.find(b"\n", p.a)
            first_nl[k] = nl if 0 <= nl < p.end else None
    return stitch_pieces(pieces, per_piece, first_nl), pieces, groups


def _expected(obj: bytes, plan):
    out = [np.array(cpu_ref.fasta_chunk_pairs(obj, c0, c1), np.uint64).reshape(-1, 2) for c0, c1 in plan]
    return np.concatenate(out) if out else np.zeros((0, 2), np.uint64)


@pytest.mark.parametrize("seed", range(6))
def test_stitched_pieces_equal_whole_chunks(seed):
    rng = np.random.default_rng(seed)
    cases = cuts = 0
    for _ in range(60):
        size = int(math.exp(rng.uniform(math.log(2), math.log(60000))))
        a = _soup(rng, size) if rng.random() < 0.5 else _records(rng, size)
        obj = a.tobytes()
        plan = _plan(rng, size)
        n = int(rng.integers(1, 10))
        got, pieces, groups = _emulate(obj, plan, n)
        assert np.array_equal(got, _expected(obj, plan)), (seed, size, plan, n)
        assert len(groups) <= n
        cases += 1
        cuts += sum(not p.first for p in pieces)
    assert cuts > 50                                       # the stitch path is exercised


def test_canonical_plan_fills_every_gpu():
    """The reference's canonical plan (examples/fasta_example.py:23: chunk_size = ceil(size / 4)) on 8 GPUs:
    8 byte-balanced groups, each chunk cut in two; on 4 GPUs the chunks stay whole."""
    size = 4 << 30
    plan = cpu_ref.chunk_plan(size, math.ceil(size / 4))
    pieces, _, groups = fasta_split(plan, 8, size)
    assert len(groups) == 8 and len(pieces) == 8
    assert all(g.hi - g.lo in (size // 8, size // 8 + 1) for g in groups)
    pieces4, _, groups4 = fasta_split(plan, 4, size)
    assert len(groups4) == 4 and all(p.first and p.end == p.b for p in pieces4)
    assert [(p.a, p.b) for p in pieces4] == list(plan)


def test_pieces_cover_plan_in_order():
    rng = np.random.default_rng(7)
    for _ in range(200):
        size = int(rng.integers(1, 10_000_000))
        plan = _plan(rng, size)
        n = int(rng.integers(1, 17))
        runs = fasta_pieces(plan, n)
        flat = [p for r in runs for p in r]
        assert len(runs) <= n
        for i, (c0, c1) in enumerate(plan):
            ps = [p for p in flat if p.chunk == i]
            assert ps[0].a == c0 and ps[-1].b == c1 and ps[0].first and all(not p.first for p in ps[1:])
            assert all(x.b == y.a for x, y in zip(ps, ps[1:]))
            assert all(p.end == (p.b if p is ps[-1] else p.b + 1) for p in ps)
        assert [p.chunk for p in flat] == sorted(p.chunk for p in flat)
