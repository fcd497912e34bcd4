"""bench.py host logic on the CPU: leg selection, the cgroup-derived CPU-baseline pool, and the every-offset check
of a uint16 + 64 KiB block-table index (fed with a correct index built in numpy, then with corrupted ones)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from dataplug_amd import synth  # noqa: E402


def test_legs():
    assert bench.parse([]).legs == ["fasta", "csv", "vcf"]
    assert bench.parse(["--workload", "csv"]).legs == ["csv"]
    assert bench.parse(["--workload", "vcf", "--legs", "fasta,vcf"]).legs == ["vcf", "fasta"]
    assert bench.parse(["--legs", "fasta"]).legs == ["fasta"]
    with pytest.raises(SystemExit):
        bench.parse(["--legs", "fasta,gff"])


def test_pool_plan_reports_its_basis():
    n, host = bench.pool_plan()
    assert n == host["pool_processes"] >= 1
    assert n <= host["affinity_cpus"]
    q = host["cgroup_quota_cpus"]
    if q is not None:
        assert host["pool_basis"] == "cgroup CPU quota" and n <= max(1, int(q))
    assert "cgroup_cpu" in host and host["os_cpu_count"] == os.cpu_count()


def _blocked_index(obj, begin, end):
    exp = np.concatenate(list(obj.delims_range(begin, end)))
    j0, j1 = begin >> 16, (end - 1) >> 16
    tab = np.searchsorted(exp, np.arange(j0, j1 + 1, dtype=np.uint64) << np.uint64(16)).astype(np.uint64)
    return (exp & np.uint64(0xFFFF)).astype(np.uint16), tab


@pytest.mark.parametrize("begin,end", [(0, 3 << 20), (777, (3 << 20) - 5), (65536, 65536 * 40 + 1), (100, 9000)])
def test_verify_blocked(begin, end):
    obj = synth.tiled_csv(3 << 20, seed=5, block=(100 << 10) - 7)
    got, tab = _blocked_index(obj, begin, end)
    n = len(got)
    assert bench._verify_blocked(obj, begin, end, got, tab, n)
    assert not bench._verify_blocked(obj, begin, end, got[:-1], tab, n - 1)          # one entry short
    g2 = got.copy()
    g2[n // 2] ^= 1
    assert not bench._verify_blocked(obj, begin, end, g2, tab, n)                   # a wrong low word
    for j in range(len(tab)):                                                      # any wrong table entry
        t2 = tab.copy()
        t2[j] += np.uint64(1)
        assert not bench._verify_blocked(obj, begin, end, got, t2, n), j


def _byte_index(obj, begin, end):
    from test_partition_golden import byte_offsets
    exp = np.concatenate(list(obj.delims_range(begin, end)))
    bo = byte_offsets(exp, begin, end)
    return bo.low, bo.sub, bo.table


@pytest.mark.parametrize("begin,end", [(0, 3 << 20), (777, (3 << 20) - 5), (65536, 65536 * 40 + 1), (100, 9000),
                                       (256 * 7, 256 * 700)])
def test_verify_bytes(begin, end):
    obj = synth.tiled_csv(3 << 20, seed=5, block=(100 << 10) - 7)
    got, sub, tab = _byte_index(obj, begin, end)
    n = len(got)
    assert bench._verify_bytes(obj, begin, end, got, sub, tab, n)
    assert not bench._verify_bytes(obj, begin, end, got[:-1], sub, tab, n - 1)      # one entry short
    g2 = got.copy()
    g2[n // 2] ^= 1
    assert not bench._verify_bytes(obj, begin, end, g2, sub, tab, n)               # a wrong low byte
    for j in range(0, len(sub), max(1, len(sub) // 50)):                          # wrong 256-byte entries
        s2 = sub.copy()
        s2[j] += np.uint16(1)
        assert not bench._verify_bytes(obj, begin, end, got, s2, tab, n), j
    for j in range(len(tab)):                                                      # any wrong table entry
        t2 = tab.copy()
        t2[j] += np.uint64(1)
        assert not bench._verify_bytes(obj, begin, end, got, sub, t2, n), j
