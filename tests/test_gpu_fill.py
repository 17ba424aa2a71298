"""GPU parity: the HIP fill (through the C ABI) against the reference goldens
and the CPU oracle.  Bit-exact on every cell (integer work).

Runs on an MI355X only (`pytest -m gpu`).
"""
import os

import numpy as np
import pytest

import nw_amd
import oracle_lib as O

pytestmark = pytest.mark.gpu

@pytest.fixture(params=["scan", "skew", "pair"], autouse=True)
def fill_kernel(request, monkeypatch):
    """Every test runs on every fill kernel (nw_fill.hip's column scan,
    nw_skew.hip's skewed stripes, nw_pair.hip's two-row scan), whose device layouts differ."""
    monkeypatch.setenv("NW_KERNEL", request.param)
    return request.param


ALL = nw_amd.NW_OUT_ALL


@pytest.fixture
def waves(monkeypatch):
    """Force the workgroup height (waves per WG) the library picks."""
    def _set(w):
        if w is None:
            monkeypatch.delenv("NW_WAVES", raising=False)
        else:
            monkeypatch.setenv("NW_WAVES", str(w))
    yield _set
    monkeypatch.delenv("NW_WAVES", raising=False)


def _check_against_oracle(s1, s2, m, k, d):
    H, D, st = nw_amd.fill(s1, s2, m, k, d)
    Ho, Do, sto = O.fill(s1, s2, m, k, d)
    assert H.shape == Ho.shape
    if not np.array_equal(H, Ho):
        bad = np.argwhere(H != Ho)
        raise AssertionError(f"score mismatch at {len(bad)} cells, first {bad[:5].tolist()} "
                             f"got {H[tuple(bad[0])]} want {Ho[tuple(bad[0])]}")
    if not np.array_equal(D, Do):
        bad = np.argwhere(D != Do)
        raise AssertionError(f"code mismatch at {len(bad)} cells, first {bad[:5].tolist()}")
    assert (st.corner, st.greatest_abs_interior, st.branch_count) == sto


def test_reference_kats(ref_kats):
    """Every KAT of the compiled reference: stats + full-table hashes."""
    for case in ref_kats:
        s1, s2 = O.kat_inputs(case)
        H, D, st = nw_amd.fill(s1, s2, case["m"], case["k"], case["d"])
        assert (st.corner, st.greatest_abs_interior, st.branch_count) == \
            (case["corner"], case["gav"], case["branch_count"]), case
        assert "%016x" % O.fnv(H) == case["hH"], case
        assert "%016x" % O.fnv(D) == case["hD"], case
        if "H" in case:
            assert H.ravel().tolist() == case["H"]
            assert D.ravel().tolist() == case["codes"]


@pytest.mark.parametrize("L1,L2", [(1, 1), (1, 64), (64, 1), (8, 63), (9, 65), (17, 128), (16, 129),
                                   (255, 257), (513, 1025), (1000, 3000), (3000, 1000)])
def test_shapes_vs_oracle(L1, L2):
    _check_against_oracle(O.gen_dna(11, L1), O.gen_dna(12, L2), 1, 1, 1)


@pytest.mark.parametrize("m,k,d", [(1, 1, 1), (2, 3, 5), (5, -4, 2), (1, 1, -1), (0, 0, 0),
                                   (-3, 2, 1), (7, 7, 0), (100, 1000, 37), (1, 1, 20000)])
def test_params_vs_oracle(m, k, d):
    _check_against_oracle(O.gen_dna(3, 700), O.gen_dna(4, 900), m, k, d)


@pytest.mark.parametrize("w", [1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 15])
def test_every_workgroup_height(waves, w):
    """Each WG height; L2 spans many WG-stripes so the granule hand-off runs."""
    waves(w)
    _check_against_oracle(O.gen_dna(5, 1234), O.gen_dna(6, 64 * w * 5 + 17), 2, 3, 5)


@pytest.mark.parametrize("L1,L2", [(300, 64 * 300 + 5), (200, 64 * 1000 + 3), (130, 100_000), (61, 64 * 256 * 3)])
def test_balanced_stripe_plan(L1, L2):
    """More stripes than CUs: one WG-stripe per CU holding SQ or SQ+1 stripes."""
    _check_against_oracle(O.gen_dna(15, L1), O.gen_dna(16, L2), 2, 3, 5)


def test_many_workgroup_stripes_handoff(waves):
    """W=1: 157 WG-stripes, every boundary through the granule hand-off."""
    waves(1)
    _check_against_oracle(O.gen_dna(7, 2000), O.gen_dna(8, 10000), 1, 1, 1)


def test_arbitrary_bytes_and_ties():
    rng = np.random.default_rng(0)
    s1 = bytes(rng.integers(1, 256, 1500, dtype=np.uint8))
    s2 = bytes(rng.integers(1, 256, 1300, dtype=np.uint8))
    _check_against_oracle(s1, s2, 3, 2, 1)
    _check_against_oracle(b"A" * 900, b"A" * 700, 1, 1, 1)        # all matches
    _check_against_oracle(b"A" * 900, b"C" * 700, 0, 0, 0)        # every cell ties 3 ways
    _check_against_oracle(b"ACGT" * 300, b"TGCA" * 200, 1, 2, 1)


@pytest.mark.parametrize("s1,s2", [(b"", b""), (b"", b"ACGT"), (b"ACGT", b""), (b"A", b"")])
def test_empty_sequences(s1, s2):
    _check_against_oracle(s1, s2, 1, 1, 1)


def test_overflow_is_rejected():
    with pytest.raises(nw_amd.NWError) as e:
        nw_amd.fill(b"ACGT" * 1000, b"ACGT" * 1000, 1, 1, 1 << 20)
    assert e.value.rc == nw_amd.NW_ERR_RANGE


def test_table_api_slices_hash_and_score_only():
    s1, s2 = O.gen_dna(21, 3001), O.gen_dna(22, 2003)
    Ho, Do, sto = O.fill(s1, s2, 2, 3, 5)
    with nw_amd.Table(4000, 4000) as t:
        t.set_sequences(s1, s2)
        t.fill(2, 3, 5, ALL)
        st = t.stats()
        assert (st.corner, st.greatest_abs_interior, st.branch_count) == sto
        assert np.array_equal(t.scores(100, 357), Ho[100:357])
        assert np.array_equal(t.codes(2990, 3002), Do[2990:3002])
        assert np.array_equal(t.last_column(), Ho[-1])
        h, e, _ = O.colchain(s1, s2, 2, 3, 5)
        assert t.hash() == (h, e)
        kms, cms = t.elapsed_ms()
        assert 0 < kms <= cms
        # refill is idempotent
        t.fill(2, 3, 5, ALL)
        assert t.hash() == (h, e)
        # score-only: corner and last column without the table
        t.fill(2, 3, 5, nw_amd.NW_OUT_STATS)
        st2 = t.stats()
        assert (st2.corner, st2.greatest_abs_interior, st2.branch_count) == sto
        assert np.array_equal(t.last_column(), Ho[-1])
        # dirs-only
        t.fill(2, 3, 5, nw_amd.NW_OUT_DIRS)
        assert np.array_equal(t.codes(0, 40), Do[0:40])


def test_score_only_table_without_score_storage():
    s1, s2 = O.gen_dna(31, 5000), O.gen_dna(32, 4000)
    c, hl = O.score_only(s1, s2, 1, 1, 1)
    with nw_amd.Table(5000, 4000, nw_amd.NW_OUT_STATS) as t:
        t.set_sequences(s1, s2)
        t.fill(1, 1, 1, 0)
        assert t.stats().corner == c
        assert O.fnv(t.last_column()) == hl
        with pytest.raises(nw_amd.NWError):
            t.fill(1, 1, 1, nw_amd.NW_OUT_SCORES)


def test_10k_config_c2(ref_kats):
    """configs[1]: 10k x 10k random DNA, 1 1 1 -- full tables vs the reference."""
    case = next(c for c in ref_kats if c["kind"] == "gen" and c["L1"] == 10000 and c["L2"] == 10000)
    s1, s2 = O.kat_inputs(case)
    with nw_amd.Table(10000, 10000) as t:
        t.set_sequences(s1, s2)
        t.fill(1, 1, 1, ALL)
        st = t.stats()
        assert (st.corner, st.greatest_abs_interior, st.branch_count) == \
            (case["corner"], case["gav"], case["branch_count"])
        H = t.scores()
        D = t.codes()
    assert "%016x" % O.fnv(H) == case["hH"]
    assert "%016x" % O.fnv(D) == case["hD"]


def test_100k_config_c3_colchain():
    """configs[2]: 100k x 100k, full table in HBM.  The reference cannot run it
    (1.36 TB); parity is transitive through the oracle-generated
    tests/golden/big_colchain.json (the oracle is pinned to the reference up to
    10k x 10k by tests/test_oracle_golden.py).  Also the size-independent
    properties: score-only corner/last column == full-table ones, refill
    idempotent."""
    from conftest import load_golden
    g = load_golden("big_colchain.json")[0]
    s1, s2 = nw_amd.gen_dna(1, g["L1"]), nw_amd.gen_dna(2, g["L2"])
    with nw_amd.Table(g["L1"], g["L2"]) as t:
        t.set_sequences(s1, s2)
        t.fill(g["m"], g["k"], g["d"], ALL)
        st = t.stats()
        assert (st.corner, st.greatest_abs_interior, st.branch_count) == \
            (g["corner"], g["gav"], g["branch_count"])
        hH, hD = t.hash()
        assert ("%016x" % hH, "%016x" % hD) == (g["hH2"], g["hD2"])
        last = t.last_column()
        t.fill(g["m"], g["k"], g["d"], nw_amd.NW_OUT_STATS)      # score-only
        st2 = t.stats()
        assert (st2.corner, st2.greatest_abs_interior, st2.branch_count) == \
            (g["corner"], g["gav"], g["branch_count"])
        assert np.array_equal(t.last_column(), last)


def test_100k_score_only_last_column_matches_full_fill():
    """Size-independent check of the score-only path at 100k x 100k: the last
    column H[L1][*] of a score-only fill (no table stored) equals the last
    column of the full fill, whose table hashes to the 100k fixture above."""
    L1 = L2 = 100_000
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    SD = nw_amd.NW_OUT_SCORES | nw_amd.NW_OUT_DIRS
    with nw_amd.Table(L1, L2, SD) as t:
        t.set_sequences(s1, s2)
        t.fill(1, 1, 1, SD)
        full = t.last_column()
        t.fill(1, 1, 1, 0)
        so = t.last_column()
        corner = t.stats().corner
    assert np.array_equal(full, so)
    assert corner == full[-1]


def test_1m_score_only_pinned():
    """configs[4]: 1M x 1M score-only (no table; 4 TB would not fit).  Corner
    and the FNV of the last row H[L1][0..L2] against tests/golden/big_scoreonly.json,
    written by the oracle's multithreaded restatement (make_big_scoreonly.py)."""
    from conftest import load_golden
    g = load_golden("big_scoreonly.json")[0]
    s1, s2 = nw_amd.gen_dna(1, g["L1"]), nw_amd.gen_dna(2, g["L2"])
    with nw_amd.Table(g["L1"], g["L2"], nw_amd.NW_OUT_STATS) as t:
        t.set_sequences(s1, s2)
        t.fill(g["m"], g["k"], g["d"], nw_amd.NW_OUT_STATS)
        assert t.stats().corner == g["corner"]
        assert "%016x" % O.fnv(t.last_column()) == g["lastcol_fnv"]
