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
