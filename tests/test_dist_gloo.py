"""N>1 path on CPU: two ranks over gloo (127.0.0.1).  Ranks get disjoint contiguous chunk groups that
cover the plan, the per-rank outputs concatenated in rank order equal the single-process index, and the
bench's barrier / max / sum reductions behave."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

from dataplug_amd.dist import rank_byte_range, rank_chunks, split_groups

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_split_groups_cover_and_disjoint():
    for n in range(0, 40):
        for g in range(1, 10):
            gr = split_groups(n, g)
            flat = [i for a, b in gr for i in range(a, b)]
            assert flat == list(range(n))
            sizes = [b - a for a, b in gr]
            assert max(sizes) - min(sizes) <= 1
    assert rank_chunks(2, 3, 4) == (2, 2)


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
    from dataplug_amd.dist import Dist, rank_byte_range, rank_chunks
    from dataplug_amd import synth
    from oracle import cpu_ref
    d = Dist.from_env(backend="gloo")
    data = bytes(synth.fasta(1 << 20, 3))
    plan = cpu_ref.chunk_plan(len(data), (1 << 20) // 7)
    i0, i1 = rank_chunks(len(plan), d.rank, d.world)
    mine = [cpu_ref.fasta_chunk_pairs(data, c0, c1) for c0, c1 in plan[i0:i1]]
    d.barrier()
    tv = synth.tiled_vcf(1_000_003, seed=4, block=200_003)
    lo, hi = rank_byte_range(len(tv.head), tv.size, d.rank, d.world)
    nl = np.concatenate(list(tv.delims_range(lo, hi))).tolist()
    mx = d.max(float(d.rank + 1))
    sm = d.sum(float(sum(len(m) for m in mine)))
    out = {{"rank": d.rank, "range": [i0, i1], "pairs": [p for m in mine for p in m], "max": mx, "sum": sm, "nl": nl}}
    with open(os.path.join({tmp!r}, f"r{{d.rank}}.json"), "w") as f:
        json.dump(out, f)
    d.close()
""")


def test_two_rank_gloo(tmp_path):
    import json
    from oracle import cpu_ref
    from dataplug_amd import synth
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(repo=REPO, tmp=str(tmp_path)))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, cwd=REPO))
    for p in procs:
        assert p.wait(timeout=240) == 0
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    data = bytes(synth.fasta(1 << 20, 3))
    idx, n = cpu_ref.fasta_index(data, (1 << 20) // 7)
    whole = np.frombuffer(idx, np.uint32).reshape(-1, 2).tolist()
    assert res[0]["range"][1] == res[1]["range"][0] and res[1]["range"][1] == 7
    assert res[0]["pairs"] + res[1]["pairs"] == whole
    assert res[0]["max"] == res[1]["max"] == 2.0
    assert res[0]["sum"] == res[1]["sum"] == float(n)
    tv = synth.tiled_vcf(1_000_003, seed=4, block=200_003)
    body_nl = cpu_ref.delim_index(tv.bytes_range(0, tv.size), len(tv.head), tv.size).tolist()
    assert res[0]["nl"] + res[1]["nl"] == body_nl
