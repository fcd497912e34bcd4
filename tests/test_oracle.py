"""The CPU oracle pinned against the reference: golden vectors made by running the reference itself
(tests/golden/make_golden.py), the sample's .fai, and the C restatement (oracle/dpref.c) cross-checked."""
import os

import numpy as np
import pytest

from oracle import cpu_ref, dpref
from dataplug_amd import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cases(fasta_cases):
    z = fasta_cases
    for i in range(len(z["chunk_size"])):
        data = bytes(z["data"][z["data_off"][i]:z["data_off"][i + 1]])
        exp = z["expected"][z["expected_off"][i]:z["expected_off"][i + 1]]
        yield i, str(z["kind"][i]), data, int(z["chunk_size"][i]), exp, int(z["num_sequences"][i])


def test_python_oracle_matches_reference_golden(fasta_cases):
    n = 0
    for i, kind, data, cs, exp, nseq in _cases(fasta_cases):
        idx, got_n = cpu_ref.fasta_index(data, cs)
        assert np.array_equal(np.frombuffer(idx, np.uint32), exp), (i, kind, cs)
        assert got_n == nseq
        n += 1
    assert n > 1000


def test_sample_matches_fai(fasta_cases):
    z = fasta_cases
    i = list(z["kind"]).index("sample")
    data = bytes(z["data"][z["data_off"][i]:z["data_off"][i + 1]])
    idx = np.frombuffer(cpu_ref.fasta_index(data, -(-len(data) // 4))[0], np.uint32).reshape(-1, 2)
    assert idx.tolist() == [[0, 60], [236, 296], [473, 533], [709, 769], [946, 1006], [1183, 1249],
                            [1426, 1486], [1663, 1721], [1898, 1958]]


def test_c_oracle_matches_python_oracle(fasta_cases):
    for i, kind, data, cs, exp, nseq in _cases(fasta_cases):
        if i % 3:
            continue
        plan = cpu_ref.chunk_plan(len(data), cs)
        got = dpref.fasta_pairs(np.frombuffer(data, np.uint8), plan)
        assert np.array_equal(got.reshape(-1).astype(np.uint32), exp), (i, kind)


def test_synthetic_golden_indexes(fasta_cases):
    z = fasta_cases
    for j in range(len(z["syn_seed"])):
        data = synth.fasta(int(z["syn_size"][j]), int(z["syn_seed"][j]))
        assert synth.sha256(data) == str(z["syn_sha256"][j])
        exp = z["syn_index"][z["syn_index_off"][j]:z["syn_index_off"][j + 1]]
        plan = cpu_ref.chunk_plan(len(data), int(z["syn_chunk_size"][j]))
        got = dpref.fasta_pairs(data, plan)
        assert np.array_equal(got.reshape(-1).astype(np.uint32), exp)


@pytest.mark.parametrize("every_k,emit_add", [(1, 0), (4, 1), (3, 7)])
def test_delim_oracles_agree(every_k, emit_add):
    rng = np.random.default_rng(every_k)
    a = rng.choice(np.frombuffer(b"ACGT\n,", np.uint8), size=100_003)
    for begin, end in [(0, len(a)), (5, 77_777), (1000, 1000)]:
        exp = cpu_ref.delim_index(a, begin, end, 10, every_k, emit_add)
        got, nd = dpref.delim(a, begin, end, 10, every_k, emit_add)
        assert np.array_equal(got, exp)
        assert nd == int((a[begin:end] == 10).sum())
