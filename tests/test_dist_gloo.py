"""N>1 path on CPU: two ranks over gloo (127.0.0.1), driven through bench.py's own Team / FastaSpec.  Ranks
get disjoint byte-balanced groups of one object from the product split (scan.objects.fasta_split, a chunk
cut where the group boundary falls inside it); the per-rank outputs gathered in rank order and stitched
(scan.objects.stitch_pieces) equal the single-process index."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from dataplug_amd.dist import rank_byte_range, split_groups

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_split_groups_cover_and_disjoint():
    for n in range(0, 40):
        for g in range(1, 10):
            gr = split_groups(n, g)
            flat = [i for a, b in gr for i in range(a, b)]
            assert flat == list(range(n))
            sizes = [b - a for a, b in gr]
            assert max(sizes) - min(sizes) <= 1
    assert split_groups(2, 4) == [(0, 1), (1, 2)]


def test_rank_byte_ranges_concatenate_to_whole_index():
    """bench.py --workload vcf: the per-rank newline indexes of the body parts concatenate to the whole."""
    from dataplug_amd import synth
    from oracle import cpu_ref
    t = synth.tiled_vcf(2_000_003, seed=4, block=300_007)
    a = t.bytes_range(0, t.size)
    bo = len(t.head)
    whole = cpu_ref.delim_index(a, bo, t.size)
    for world in (1, 2, 3, 8, 13):
        parts = [rank_byte_range(bo, t.size, r, world) for r in range(world)]
        assert parts[0][0] == bo and parts[-1][1] == t.size
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        got = np.concatenate([cpu_ref.delim_index(a, lo, hi) for lo, hi in parts])
        assert np.array_equal(got, whole)
    assert rank_byte_range(5, 5, 0, 4) == (5, 5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = textwrap.dedent("""
    import json, os, sys
    import numpy as np
    sys.path.insert(0, {repo!r})
    import torch.distributed as dist
    import bench
    from oracle import dpref
    from dataplug_amd.dist import rank_byte_range
    from dataplug_amd import synth
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    team = bench.Team(1, dist)                      # what bench.py builds under torch.distributed.run
    # bench.py's strong point: ONE object with the caller's plan (chunk_size = size/4) over the ranks by the
    # product split (scan.objects.fasta_split); this rank materializes only its group + halo, as a bench
    # rank does.  The GPU scan of each launch chunk stands in as the oracle over the same bytes (no GPU here)
    spec = bench.FastaSpec({size}, 4, world, seed=3)
    g = spec.groups[rank]
    host = spec.obj.bytes_range(g.lo, g.buf_hi)
    mine, first_nl = [], {{}}
    for k in range(g.i0, g.i1):
        p = spec.pieces[k]
        mine.append((dpref.fasta_pairs(host, [(p.a - g.lo, p.end - g.lo)]) + np.uint64(g.lo)).tolist())
        if not p.first:
            nl = np.flatnonzero(host[p.a - g.lo:p.end - g.lo] == 10)
            first_nl[k] = int(p.a + nl[0]) if len(nl) else None
    team.barrier()
    tv = synth.tiled_vcf(1_000_003, seed=4, block=200_003)
    lo, hi = rank_byte_range(len(tv.head), tv.size, rank, world)
    nl = np.concatenate(list(tv.delims_range(lo, hi))).tolist()
    allres = team.gather([{{"rank": rank, "group": [g.i0, g.i1, g.lo, g.hi, g.buf_hi], "pairs": mine,
                            "first_nl": first_nl, "nl": nl}}])
    if allres is not None:
        with open(os.path.join({tmp!r}, "gathered.json"), "w") as f:
            json.dump(allres, f)
    dist.destroy_process_group()
""")


def test_two_rank_gloo(tmp_path):
    """Two ranks over gloo, as bench.py runs under torch.distributed.run: each takes its group of ONE object
    from the product's split (the caller's 3-chunk plan over 2 ranks: the middle chunk is cut), the gather
    reaches rank 0 in rank order, and the groups' pieces stitch to the whole object's index."""
    import json
    from oracle import cpu_ref, dpref
    from dataplug_amd import synth
    size = (3 << 20) + 12345
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(repo=REPO, tmp=str(tmp_path), size=size))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, cwd=REPO))
    for p in procs:
        assert p.wait(timeout=240) == 0
    from dataplug_amd.scan.objects import fasta_split, stitch_pieces
    res = json.load(open(tmp_path / "gathered.json"))
    assert [r["rank"] for r in res] == [0, 1]
    g0, g1 = res[0]["group"], res[1]["group"]
    obj = synth.TiledFasta(size, seed=3).bytes_range(0, size)
    plan = cpu_ref.chunk_plan(size, -(-size // 4))         # 3 chunks: the tail past 3 * cs is never scanned
    pieces, _, _ = fasta_split(plan, 2, size)
    assert len(pieces) == 4 and sum(not p.first for p in pieces) == 1
    assert g0[0] == 0 and g0[1] == g1[0] and g1[1] == len(pieces) and g0[3] in (g1[2], g1[2] + 1)
    per_piece = [np.asarray(x, np.uint64).reshape(-1, 2) for r in res for x in r["pairs"]]
    first_nl = {int(k): v for r in res for k, v in r["first_nl"].items()}
    whole = dpref.fasta_pairs(obj, plan)
    assert np.array_equal(stitch_pieces(pieces, per_piece, first_nl), whole)
    tv = synth.tiled_vcf(1_000_003, seed=4, block=200_003)
    body_nl = cpu_ref.delim_index(tv.bytes_range(0, tv.size), len(tv.head), tv.size).tolist()
    assert res[0]["nl"] + res[1]["nl"] == body_nl


def test_line_parts_cover_in_order():
    from dataplug_amd.scan.objects import line_parts, page_ranges
    for begin, end, g, pb in [(0, 100, 3, 1000), (1337, 64 << 30, 8, 16 << 30), (5, 5, 4, 10), (0, 7, 8, 100)]:
        parts = line_parts(begin, end, g, pb)
        if end > begin:
            assert parts[0][0] == begin and parts[-1][1] == end
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert all(hi - lo <= pb for lo, hi in parts)
        else:
            assert parts == []
    G = 1 << 30
    assert page_ranges(3 * G, 9 * G) == [(3 * G, 4 * G), (4 * G, 8 * G), (8 * G, 9 * G)]
    assert page_ranges(4 * G, 8 * G) == [(4 * G, 8 * G)]


@pytest.mark.parametrize("fmt", ["u8s", "u16b", "u32p"])
def test_line_index_parts_merge(monkeypatch, fmt):
    """line_index_object's merge of per-part GPU outputs (parts at unaligned cuts, one per 'device'),
    with each part's scan replaced by what the kernel returns for it (host logic only): the merged index
    rebuilds every offset, across 64 KiB blocks and 4 GiB pages."""
    from types import SimpleNamespace
    from dataplug_amd.scan import objects
    G = 1 << 30
    rng = np.random.default_rng(7)
    begin, end = 3 * G + 4321, 13 * G + 77
    off = np.unique(rng.integers(begin, end, 200_000).astype(np.uint64))

    def fake_group(dev, co, lo, hi, delim, every_k, emit_add, fmt="u64"):
        sel = off[(off >= lo) & (off < hi)]
        if fmt == "u8s":
            from test_partition_golden import byte_offsets
            bo = byte_offsets(sel, lo, hi)
            return bo.low, bo.table, bo.sub
        if fmt == "u32p":
            rg = objects.page_ranges(lo, hi)
            counts = np.cumsum([int(((sel >= a) & (sel < b)).sum()) for a, b in rg])
            return sel.astype(np.uint32), [(r, int(c)) for r, c in zip(rg, counts)]
        j0 = lo >> 16
        nt = ((hi - 1) >> 16) - j0 + 1
        tab = np.searchsorted(sel, (np.arange(j0, j0 + nt, dtype=np.uint64) << np.uint64(16))).astype(np.uint64)
        if lo & 0xFFFF:
            tab[0] = 0
        return (sel & np.uint64(0xFFFF)).astype(np.uint16), tab

    monkeypatch.setattr(objects, "_delim_group", fake_group)
    monkeypatch.setenv("DATAPLUG_AMD_DEVICES", "0,0,0")
    co = SimpleNamespace(size=end)
    res = objects.line_index_object(co, begin=begin, end=end, fmt=fmt, part_bytes=3 * G + 5)
    assert len(res) == len(off) and np.array_equal(res.to_u64(), off)
