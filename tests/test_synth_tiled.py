"""synth.TiledText (the bench's configs[2]/[3] objects): ranged bytes and analytic newline offsets agree with
the oracle's newline index over the materialized object."""
import numpy as np
import pytest

from dataplug_amd import synth
from oracle import cpu_ref


@pytest.mark.parametrize("make", [synth.tiled_csv, synth.tiled_vcf])
def test_tiled_ranges_match_oracle(make):
    t = make(3_000_017, seed=5, block=400_009)
    a = t.bytes_range(0, t.size)
    assert len(a) == t.size
    assert bytes(a[:len(t.head)]) == bytes(t.head)
    stage = np.empty(1 << 20, np.uint8)
    for s, e in [(0, t.size), (1, 17), (len(t.head) - 3, 900_000), (400_000, 2_000_001), (t.size - 5, t.size)]:
        exp = cpu_ref.delim_index(a, s, e)
        got = np.concatenate(list(t.delims_range(s, e)) + [np.empty(0, np.uint64)])
        assert np.array_equal(got, exp), (s, e)
        assert t.count_range(s, e) == len(exp)
        assert np.array_equal(t.bytes_range(s, e), a[s:e])
        if e - s <= len(stage):
            assert np.array_equal(t.bytes_range(s, e, out=stage), a[s:e])


@pytest.mark.parametrize("size", [1_000, 3_000_017, 2_400_031])
def test_tiled_fasta_ranges_equal_host_object(size):
    """synth.TiledFasta (bench.py's N x 4 GiB object, built per chunk group) is tiled_fasta_host byte for byte,
    including the object-level tail fix, for any range."""
    block = 400_009
    whole = synth.tiled_fasta_host(size, seed=2, block=block)
    t = synth.TiledFasta(size, seed=2, block=block)
    assert np.array_equal(t.bytes_range(0, size), whole)
    for s, e in [(0, min(size, 17)), (size // 3, size // 2), (max(0, size - 70_000), size), (size - 1, size)]:
        assert np.array_equal(t.bytes_range(s, e), whole[s:e]), (s, e)


def test_tiled_fasta_tail_fix_applies_only_at_object_end():
    # this size ends inside a header line: the object-level fix rewrites that tail ('N'), and only there
    size = 2_000_007
    t = synth.TiledFasta(size, seed=6, block=1_000_003)
    assert t.tail_fix
    whole = synth.tiled_fasta_host(size, seed=6, block=1_000_003)
    assert np.array_equal(t.bytes_range(0, size), whole)
    assert (whole[t.tail0:] == ord("N")).all() and whole[t.tail0 - 1] == 10
    assert np.array_equal(t.bytes_range(t.tail0 - 50, size), whole[t.tail0 - 50:])
    # the same bytes one block earlier are untouched
    b = t.tail0 - 1_000_003
    assert (t.bytes_range(b, b + (size - t.tail0)) == ord(">")).any()
