"""GPU parity of the walk services (include/nw_fill.h nw_table_count_alignments,
nw_table_first_path) against the reference's own walk output
(tests/golden/walk_kats.json, from its CLI) and the CPU oracle (path-count
DP and greedy diag > left > up walk, needleman-wunsch.c:209-331).  Integer
work: bit-exact.  At 100k x 100k: the restatement's fixture
(tests/golden/big_walk.json) plus size-independent properties (the path is
a monotone staircase from (0,0) to (L1,L2) whose score is the corner).
"""
import json
import os

import numpy as np
import pytest

import nw_amd
import oracle_lib as O

pytestmark = pytest.mark.gpu

@pytest.fixture(params=["scan", "skew", "pair", "quad"], autouse=True)
def fill_kernel(request, monkeypatch):
    """Every test runs on every fill kernel (nw_fill.hip's column scan,
    nw_skew.hip's skewed stripes, nw_pair.hip's two-row scan, nw_quad.hip's
    skewed 16-row groups; a fill with stats that asks for the last runs the
    first), whose device layouts differ."""
    monkeypatch.setenv("NW_KERNEL", request.param)
    return request.param


DIRS = nw_amd.NW_OUT_DIRS


def _walk(s1, s2, m, k, d, mask=DIRS, max_L1=None, max_L2=None):
    L1, L2 = len(s1), len(s2)
    with nw_amd.Table(max_L1 or L1, max_L2 or L2, mask) as t:
        t.set_sequences(s1, s2)
        t.fill(m, k, d, mask)
        return t.count_alignments(), t.first_path(), t.stats().corner


def _path_score(s1, s2, moves, m, k, d):
    i = j = 0
    sc = 0
    for mv in moves.tolist():
        if mv == 1:
            sc += m if s1[i] == s2[j] else -k
            i += 1
            j += 1
        elif mv == 4:
            sc -= d
            i += 1
        else:
            sc -= d
            j += 1
    return sc, i, j


def test_reference_walk_kats(walk_kats):
    for case in walk_kats:
        s1, s2 = O.kat_inputs(case)
        count, mv, corner = _walk(s1, s2, case["m"], case["k"], case["d"])
        assert corner == case["score"], case
        assert count == case["count"], case
        top, side = nw_amd.render_path(s1, s2, mv)
        assert (top.decode(), side.decode()) == (case["first_top"], case["first_side"]), case


@pytest.mark.parametrize("L1,L2,mkd", [
    (1, 1, (1, 1, 1)), (1, 200, (1, 1, 1)), (200, 1, (1, 1, 1)), (64, 64, (1, 1, 1)), (65, 129, (2, 3, 5)),
    (127, 1000, (1, 1, 1)), (1000, 127, (5, -4, 2)), (513, 1025, (1, 1, 1)), (3000, 1000, (2, 3, 5)),
    (1000, 3000, (0, 0, 0)), (2048, 2048, (1, 1, -1)), (4097, 333, (3, 2, 1)),
])
def test_walk_vs_oracle(L1, L2, mkd):
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    count, mv, corner = _walk(s1, s2, *mkd)
    _, D, st = O.fill(s1, s2, *mkd)
    assert corner == st[0]
    assert count == O.count_paths(D)
    want = O.first_path(D)
    assert len(mv) == len(want) and np.array_equal(mv, want)


def test_walk_ties_everywhere():
    # a single repeated letter: every cell ties, the count is a binomial sum mod 2^32
    for L1, L2 in [(10, 10), (100, 37), (700, 900)]:
        s1, s2 = b"A" * L1, b"A" * L2
        count, mv, _ = _walk(s1, s2, 0, 0, 0)
        _, D, _ = O.fill(s1, s2, 0, 0, 0)
        assert count == O.count_paths(D)
        assert np.array_equal(mv, O.first_path(D))


def test_walk_arbitrary_bytes():
    rng = np.random.default_rng(7)
    s1 = bytes(rng.integers(33, 127, 777, dtype=np.uint8))
    s2 = bytes(rng.integers(33, 127, 555, dtype=np.uint8))
    count, mv, _ = _walk(s1, s2, 3, 2, 1)
    _, D, _ = O.fill(s1, s2, 3, 2, 1)
    assert count == O.count_paths(D)
    assert np.array_equal(mv, O.first_path(D))


def test_walk_empty_and_reuse():
    # empty strings: one path along the seeded row / column; none for two
    # empty strings -- the walk starts on (0,0), whose directions are all done
    # (computation.c:96-99), so the reference counts 0
    for s1, s2 in [(b"", b"ACGT"), (b"ACGT", b""), (b"", b"")]:
        count, mv, _ = _walk(s1, s2, 1, 1, 1, max_L1=8, max_L2=8)
        assert count == (0 if not s1 and not s2 else 1)
        assert mv.tolist() == [2] * len(s2) + [4] * len(s1)
    # one table, several fills of different shapes: the hand-off tags must not leak
    with nw_amd.Table(3000, 3000, DIRS) as t:
        for L1, L2, mkd in [(3000, 3000, (1, 1, 1)), (1000, 2000, (2, 3, 5)), (2999, 129, (1, 1, 1))]:
            s1, s2 = O.gen_dna(3, L1), O.gen_dna(4, L2)
            t.set_sequences(s1, s2)
            t.fill(*mkd, DIRS)
            _, D, _ = O.fill(s1, s2, *mkd)
            assert t.count_alignments() == O.count_paths(D)
            assert np.array_equal(t.first_path(), O.first_path(D))


def test_walk_needs_codes():
    with nw_amd.Table(100, 100, nw_amd.NW_OUT_SCORES) as t:
        t.set_sequences(O.gen_dna(1, 100), O.gen_dna(2, 100))
        t.fill(1, 1, 1, nw_amd.NW_OUT_SCORES)
        with pytest.raises(nw_amd.NWError) as e:
            t.count_alignments()
        assert e.value.rc == nw_amd.NW_ERR_STATE


def test_walk_100k():
    """100k x 100k: count and first path vs the restatement's fixture; the
    path's own score must be the corner (size-independent)."""
    path = os.path.join(os.path.dirname(__file__), "golden", "big_walk.json")
    case = json.load(open(path))[0]
    L1, L2, m, k, d = case["L1"], case["L2"], case["m"], case["k"], case["d"]
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    with nw_amd.Table(L1, L2, DIRS) as t:
        t.set_sequences(s1, s2)
        t.fill(m, k, d, DIRS)
        corner = t.stats().corner
        count = t.count_alignments()
        mv = t.first_path()
        cms, pms = t.walk_elapsed_ms()
    print(f"100k walk: count {cms:.1f} ms, first path {pms:.1f} ms")
    assert corner == case["corner"]
    sc, i, j = _path_score(s1, s2, mv, m, k, d)
    assert (i, j) == (L1, L2) and sc == corner
    assert len(mv) == case["path_len"]
    assert "%016x" % nw_amd.fnv1a64(mv.tobytes()) == case["path_fnv"]
    assert count == case["count"]


@pytest.mark.parametrize("L1,L2,mkd,band", [
    (3000, 1000, (2, 3, 5), 64), (1000, 3000, (1, 1, 1), 128), (513, 1025, (1, 1, 1), 192),
    (4097, 333, (3, 2, 1), 64), (2048, 2048, (1, 1, -1), 1024), (1000, 3000, (0, 0, 0), 256),
    (200, 1, (1, 1, 1), 64), (1, 200, (1, 1, 1), 64), (300, 640, (5, -4, 2), 64), (700, 500, (1, 1, 1), 4096),
])
def test_banded_first_path_vs_oracle(L1, L2, mkd, band):
    """nw_first_path_banded (checkpointed bands, no full table) == the
    reference's first printed alignment (oracle greedy walk)."""
    s1, s2 = O.gen_dna(5, L1), O.gen_dna(6, L2)
    mv = nw_amd.first_path_banded(s1, s2, *mkd, band_rows=band)
    _, D, _ = O.fill(s1, s2, *mkd)
    want = O.first_path(D)
    assert len(mv) == len(want) and np.array_equal(mv, want)


def test_banded_first_path_ties_bytes_and_edges():
    s1, s2 = b"A" * 700, b"A" * 900            # every cell ties
    _, D, _ = O.fill(s1, s2, 0, 0, 0)
    assert np.array_equal(nw_amd.first_path_banded(s1, s2, 0, 0, 0, band_rows=64), O.first_path(D))
    rng = np.random.default_rng(11)
    s1 = bytes(rng.integers(33, 127, 777, dtype=np.uint8))
    s2 = bytes(rng.integers(33, 127, 555, dtype=np.uint8))
    _, D, _ = O.fill(s1, s2, 3, 2, 1)
    assert np.array_equal(nw_amd.first_path_banded(s1, s2, 3, 2, 1, band_rows=128), O.first_path(D))
    for a, b in [(b"", b"ACGT"), (b"ACGT", b""), (b"", b"")]:
        assert nw_amd.first_path_banded(a, b, 1, 1, 1, band_rows=64).tolist() == [2] * len(b) + [4] * len(a)
    with pytest.raises(nw_amd.NWError) as e:
        nw_amd.first_path_banded(b"ACGT", b"ACGT", 1, 1, 1, band_rows=100)
    assert e.value.rc == nw_amd.NW_ERR_ARG


def test_banded_first_path_100k():
    """100k x 100k through 13 bands of 8192 rows (0.4 GB of codes instead of
    5 GB): the restatement's first-path fixture."""
    path = os.path.join(os.path.dirname(__file__), "golden", "big_walk.json")
    case = json.load(open(path))[0]
    L1, L2, m, k, d = case["L1"], case["L2"], case["m"], case["k"], case["d"]
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    mv = nw_amd.first_path_banded(s1, s2, m, k, d, band_rows=8192)
    sc, i, j = _path_score(s1, s2, mv, m, k, d)
    assert (i, j) == (L1, L2) and sc == case["corner"]
    assert len(mv) == case["path_len"]
    assert "%016x" % nw_amd.fnv1a64(mv.tobytes()) == case["path_fnv"]
