"""Device-side enumeration of every optimal alignment (nw_table_enumerate_paths, the reference's parallel-traceback future work,
README:195-200): each alignment is unranked on its own from the device's
path-count table, and the sequence must be exactly the reference's print order
(its depth-first walk, needleman-wunsch.c:209-331), restated over the oracle's
codes by tests/test_cli_host.py's unrank()."""
import numpy as np
import pytest

import nw_amd
import oracle_lib as O
from test_cli_host import path_counts, unrank

pytestmark = pytest.mark.gpu

CASES = [
    (b"GCATGCU", b"GATTACA", 1, 1, 1),
    (b"AAAAAAAAAA", b"AAAA", 1, 1, 0),          # many ties: C(10,4) alignments
    (b"ACGTAC", b"TGCAT", 0, 0, 0),              # every path is optimal: C(11, 5) = 462
    (b"A", b"", 1, 1, 1), (b"", b"ACG", 1, 1, 1), (b"", b"", 1, 1, 1),
]


@pytest.mark.parametrize("s1,s2,m,k,d", CASES)
def test_enumeration_is_the_reference_order(s1, s2, m, k, d):
    _, D, _ = O.fill(s1, s2, m, k, d)
    C = path_counts(D)
    total = C[len(s1)][len(s2)] if (s1 or s2) else 0
    with nw_amd.Table(max(len(s1), 1), max(len(s2), 1)) as t:
        t.set_sequences(s1, s2)
        t.fill(m, k, d, nw_amd.NW_OUT_ALL)
        got, tot = t.enumerate_paths(0, total + 3)
        assert tot == total
        assert len(got) == total
        for p, mv in enumerate(got):
            assert mv.tolist() == unrank(D, C, p)
        if total:
            assert got[0].tolist()[::-1] == t.first_path().tolist()
            assert t.count_alignments() == total % 2**32
        # any window of the order
        if total > 5:
            win, _ = t.enumerate_paths(3, 2)
            assert [w.tolist() for w in win] == [unrank(D, C, 3), unrank(D, C, 4)]


def test_enumeration_of_a_larger_table():
    """1000 x 800 with ties: the first 5000 alignments against the oracle's order,
    and the last ones, across batches."""
    s1, s2 = O.gen_dna(5, 1000), O.gen_dna(6, 800)
    _, D, _ = O.fill(s1, s2, 1, 1, 1)
    C = path_counts(D)
    total = C[1000][800]
    with nw_amd.Table(1000, 800) as t:
        t.set_sequences(s1, s2)
        t.fill(1, 1, 1, nw_amd.NW_OUT_ALL)
        got, tot = t.enumerate_paths(0, 5000)
        assert tot == min(total, 2**62)
        for p in list(range(0, len(got), 97)) + [len(got) - 1]:
            assert got[p].tolist() == unrank(D, C, p)
        if total < 2**62:
            tail, _ = t.enumerate_paths(total - 3, 10)
            assert [x.tolist() for x in tail] == [unrank(D, C, q) for q in range(total - 3, total)]
