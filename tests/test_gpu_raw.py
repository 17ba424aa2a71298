"""GPU parity of the fill variant the benchmark times: scores + direction
codes WITHOUT stats (NW_OUT_SCORES | NW_OUT_DIRS).

With that mask the pair kernel keeps its tiles in the kernel's own shifted
domain (G' = H + r*d + (i - base)*d, the "raw" tiles of nw_pair.hip) and uses
a separately generated 8-column block; every reader subtracts the affine
offset, which depends on the fill's WG-stripe plan and on the cell's
4096-column super-chunk.  Every fill test elsewhere asks for stats too and so
never takes that path; these tests do, on all four kernels, cell by cell
against the CPU oracle (needleman-wunsch.c:418-510 scores, :485-503 flags),
and at 100k x 100k against the whole-table hashes of
tests/golden/big_colchain.json.

Runs on an MI355X only (`pytest -m gpu`).
"""
import numpy as np
import pytest

import nw_amd
import oracle_lib as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

SD = nw_amd.NW_OUT_SCORES | nw_amd.NW_OUT_DIRS


@pytest.fixture(params=["scan", "skew", "pair", "quad"])
def fill_kernel(request, monkeypatch):
    monkeypatch.setenv("NW_KERNEL", request.param)
    monkeypatch.delenv("NW_WAVES", raising=False)
    return request.param


@pytest.fixture
def pair_kernel(monkeypatch):
    monkeypatch.setenv("NW_KERNEL", "pair")
    monkeypatch.delenv("NW_WAVES", raising=False)


@pytest.fixture
def auto_kernel(monkeypatch):
    monkeypatch.delenv("NW_KERNEL", raising=False)
    monkeypatch.delenv("NW_WAVES", raising=False)


def _check_sd(s1, s2, m, k, d, refills=1):
    """Fill with scores + codes and no stats; every cell, every code, the
    corner, the last column and the device hash against the oracle."""
    Ho, Do, sto = O.fill(s1, s2, m, k, d)
    with nw_amd.Table(len(s1), len(s2), SD) as t:
        t.set_sequences(s1, s2)
        for _ in range(refills):
            t.fill(m, k, d, SD)
        H = t.scores()
        D = t.codes()
        st = t.stats()
        last = t.last_column()
        hh = t.hash()
    if not np.array_equal(H, Ho):
        bad = np.argwhere(H != Ho)
        raise AssertionError(f"score mismatch at {len(bad)} cells, first {bad[:5].tolist()} "
                             f"got {H[tuple(bad[0])]} want {Ho[tuple(bad[0])]}")
    if not np.array_equal(D, Do):
        bad = np.argwhere(D != Do)
        raise AssertionError(f"code mismatch at {len(bad)} cells, first {bad[:5].tolist()}")
    assert st.corner == sto[0]
    assert (st.greatest_abs_interior, st.branch_count) == (0, 0)      # not asked for
    assert np.array_equal(last, Ho[-1])
    h, e, _ = O.colchain(s1, s2, m, k, d)
    assert hh == (h, e)


@pytest.mark.parametrize("L1,L2", [(1, 1), (1, 64), (64, 1), (8, 63), (9, 65), (17, 128), (16, 129),
                                   (255, 257), (513, 1025), (1000, 3000), (3000, 1000)])
def test_sd_shapes_vs_oracle(fill_kernel, L1, L2):
    _check_sd(O.gen_dna(11, L1), O.gen_dna(12, L2), 1, 1, 1)


@pytest.mark.parametrize("m,k,d", [(1, 1, 1), (2, 3, 5), (5, -4, 2), (1, 1, -1), (0, 0, 0),
                                   (-3, 2, 1), (7, 7, 0), (100, 1000, 37), (1, 1, 20000)])
def test_sd_params_vs_oracle(fill_kernel, m, k, d):
    _check_sd(O.gen_dna(3, 700), O.gen_dna(4, 900), m, k, d)


@pytest.mark.parametrize("w", [1, 2, 3, 4, 5, 6, 7, 8, 10, 12])
def test_sd_every_workgroup_height(fill_kernel, monkeypatch, w):
    """$NW_WAVES plans: the raw offset's row term follows the plan's SQ / SR."""
    monkeypatch.setenv("NW_WAVES", str(w))
    _check_sd(O.gen_dna(5, 1234), O.gen_dna(6, 128 * w * 3 + 17), 2, 3, 5)


@pytest.mark.parametrize("L1,L2", [(300, 128 * 10), (300, 128 * 11 + 5), (130, 100_000), (70, 150_000),
                                   (61, 64 * 256 * 3)])
def test_sd_uneven_stripe_plans(fill_kernel, L1, L2):
    """Plans whose first SR WG-stripes hold one stripe more (SR > 0), packed
    (<= 4 stripes per workgroup) and one-WG-stripe-per-CU alike."""
    _check_sd(O.gen_dna(15, L1), O.gen_dna(16, L2), 2, 3, 5)


@pytest.mark.parametrize("L1,L2,mkd", [(8200, 700, (1, 1, 1)), (4097, 1300, (2, 3, 5)), (12300, 400, (1, 2, -1)),
                                       (4096, 260, (3, 1, 2))])
def test_sd_crosses_super_chunks(fill_kernel, L1, L2, mkd):
    """L1 > 4096: the kernel's column base moves every 4096 columns, and the
    raw offset's column term with it."""
    _check_sd(O.gen_dna(25, L1), O.gen_dna(26, L2), *mkd)


def test_sd_arbitrary_bytes_and_ties(fill_kernel):
    rng = np.random.default_rng(1)
    s1 = bytes(rng.integers(1, 256, 1500, dtype=np.uint8))       # no profile lookups: byte compares
    s2 = bytes(rng.integers(1, 256, 1300, dtype=np.uint8))
    _check_sd(s1, s2, 3, 2, 1)
    _check_sd(b"A" * 900, b"C" * 700, 0, 0, 0)
    _check_sd(b"ACGT" * 300, b"TGCA" * 200, 1, 2, 1)


@pytest.mark.parametrize("mask", [nw_amd.NW_OUT_SCORES, nw_amd.NW_OUT_DIRS, 0])
@pytest.mark.parametrize("L1,L2", [(3, 70), (8, 64), (21, 200), (1000, 777), (5001, 64 * 9 + 1)])
def test_partial_masks_vs_oracle(fill_kernel, mask, L1, L2):
    """Scores only, codes only, score-only (last column): each its own kernel variant."""
    s1, s2 = O.gen_dna(41, L1), O.gen_dna(42, L2)
    Ho, Do, sto = O.fill(s1, s2, 2, 3, 5)
    with nw_amd.Table(L1, L2, SD) as t:
        t.set_sequences(s1, s2)
        t.fill(2, 3, 5, mask)
        assert t.stats().corner == sto[0]
        assert np.array_equal(t.last_column(), Ho[-1])
        if mask & nw_amd.NW_OUT_SCORES:
            assert np.array_equal(t.scores(), Ho)
        if mask & nw_amd.NW_OUT_DIRS:
            assert np.array_equal(t.codes(), Do)


def test_sd_refill_and_mask_changes(pair_kernel):
    """Raw and plain fills alternate on one table: each reader follows the
    last fill's encoding."""
    s1, s2 = O.gen_dna(21, 5001), O.gen_dna(22, 2003)
    Ho, Do, sto = O.fill(s1, s2, 2, 3, 5)
    h, e, _ = O.colchain(s1, s2, 2, 3, 5)
    with nw_amd.Table(6000, 3000) as t:
        t.set_sequences(s1, s2)
        for mask in (SD, nw_amd.NW_OUT_ALL, SD, nw_amd.NW_OUT_SCORES, SD):
            t.fill(2, 3, 5, mask)
            assert t.stats().corner == sto[0]
            assert np.array_equal(t.scores(4090, 4100), Ho[4090:4100])
            if mask & nw_amd.NW_OUT_DIRS:
                assert t.hash() == (h, e)
                assert np.array_equal(t.codes(4990, 5002), Do[4990:5002])
            else:
                assert t.hash()[0] == h


def test_sd_10k_config_c2(auto_kernel, ref_kats):
    """configs[1] with the benchmark's mask: full tables vs the compiled reference's hashes."""
    case = next(c for c in ref_kats if c["kind"] == "gen" and c["L1"] == 10000 and c["L2"] == 10000)
    s1, s2 = O.kat_inputs(case)
    with nw_amd.Table(10000, 10000, SD) as t:
        t.set_sequences(s1, s2)
        t.fill(1, 1, 1, SD)
        assert t.stats().corner == case["corner"]
        H = t.scores()
        D = t.codes()
    assert "%016x" % O.fnv(H) == case["hH"]
    assert "%016x" % O.fnv(D) == case["hD"]


@pytest.mark.parametrize("kernel", ["auto", "pair", "scan", "quad"])
def test_sd_100k_config_c3_hashes(monkeypatch, kernel):
    """configs[2] exactly as bench.py times it (scores + codes, no stats): the
    45 GB table hashes, on the device, to the fixture's whole-table hashes."""
    monkeypatch.delenv("NW_WAVES", raising=False)
    if kernel == "auto":
        monkeypatch.delenv("NW_KERNEL", raising=False)
    else:
        monkeypatch.setenv("NW_KERNEL", kernel)
    g = load_golden("big_colchain.json")[0]
    s1, s2 = nw_amd.gen_dna(1, g["L1"]), nw_amd.gen_dna(2, g["L2"])
    with nw_amd.Table(g["L1"], g["L2"], SD) as t:
        t.set_sequences(s1, s2)
        for _ in range(2):
            t.fill(g["m"], g["k"], g["d"], SD)
        assert t.stats().corner == g["corner"]
        hH, hD = t.hash()
    assert ("%016x" % hH, "%016x" % hD) == (g["hH2"], g["hD2"])


@pytest.mark.parametrize("L1,L2,mkd,mask", [(4500, 128 * 11 + 5, (2, 3, 5), SD), (700, 900, (1, 1, 1), SD),
                                            (4100, 128 * 7, (1, 2, -1), nw_amd.NW_OUT_ALL)])
def test_header_layout_formulas_decode_the_device_buffers(fill_kernel, L1, L2, mkd, mask):
    """A zero-copy consumer: the raw device buffers, decoded with nothing but
    the layout formulas of include/nw_fill.h and nw_table_layout(), are the
    oracle's tables -- for every kernel's variant, raw tiles included."""
    import hip_mem
    s1, s2 = O.gen_dna(31, L1), O.gen_dna(32, L2)
    Ho, Do, _ = O.fill(s1, s2, *mkd)
    with nw_amd.Table(L1, L2, nw_amd.NW_OUT_ALL) as t:
        t.set_sequences(s1, s2)
        t.fill(*mkd, mask)
        lay = t.layout()
        assert lay.has_scores and lay.has_dirs
        stats = bool(mask & nw_amd.NW_OUT_STATS)       # (the quad kernel has no stats variant: the scan kernel runs)
        assert lay.raw == (0 if stats else {"pair": 1, "quad": 2}.get(fill_kernel, 0))
        assert lay.skew == (1 if fill_kernel == "skew" else 2 if fill_kernel == "quad" and not stats else 0)
        assert lay.score_pitch == t.score_pitch
        hp, dp = t.device_buffers()
        NG, NC = (L2 + 63) // 64, (L1 + 7) // 8
        tiles = hip_mem.copy_from_device(hp, np.int32, (NG + 1) * (NC + 8) * 512)     # as allocated
        words = hip_mem.copy_from_device(dp, np.uint32, (NG + 1) * (NC + 9) * 64)
    H, C = nw_amd.decode_tiles(tiles, words, L1, L2, mkd[2], lay)
    np.testing.assert_array_equal(H, Ho)
    np.testing.assert_array_equal(C, Do)


# ------------------------------------------------------------------ panels
def _check_sd_panels(n, L1, L2, mkd):
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    H, D, st = O.fill(s1, s2, *mkd)
    h, e, _ = O.colchain(s1, s2, *mkd)
    panels = nw_amd.Panel.group([0] * n, L1, L2, SD)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        for _ in range(2):
            nw_amd.Panel.group_fill(panels, *mkd, SD)
        for p in panels:
            base, rows = p.rows()
            if rows == 0:
                continue
            t = p.table
            np.testing.assert_array_equal(t.scores(), H[:, base:base + rows + 1],
                                          err_msg=f"panel {p.rank} scores (rows {base}..{base + rows})")
            np.testing.assert_array_equal(t.codes()[:, 1:], D[:, base + 1:base + rows + 1],
                                          err_msg=f"panel {p.rank} codes")
        assert panels[0].stats().corner == st[0]
        state = nw_amd.hash_states(L1)
        for p in panels:
            p.hash_columns(state)
        assert nw_amd.hash_fold(state) == (h, e)
    finally:
        for p in panels:
            p.close()


@pytest.mark.parametrize("n", [2, 3, 4])
@pytest.mark.parametrize("L1,L2,mkd", [(300, 517, (2, 3, 5)), (4500, 1300, (1, 1, 1)), (2049, 128 * 9, (3, 1, 2))])
def test_sd_group_panels_match_oracle(fill_kernel, n, L1, L2, mkd):
    """Raw panels (row_base > 0): the offset's row term is local to the panel."""
    _check_sd_panels(n, L1, L2, mkd)


@pytest.mark.parametrize("n", [2, 4])
def test_sd_group_panels_100k_match_fixture(auto_kernel, n):
    """C4 with the benchmark's mask: the chained whole-table hashes."""
    g = load_golden("big_colchain.json")[0]
    L1, L2 = g["L1"], g["L2"]
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * n, L1, L2, SD)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, g["m"], g["k"], g["d"], SD)
        assert panels[-1].stats().corner == g["corner"]
        state = nw_amd.hash_states(L1)
        for p in panels:
            p.hash_columns(state)
        hH, hD = nw_amd.hash_fold(state)
        assert ("%016x" % hH, "%016x" % hD) == (g["hH2"], g["hD2"])
    finally:
        for p in panels:
            p.close()
