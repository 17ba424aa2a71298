"""Configs C4 and C5 on the GPU as their multi-GPU splits: the 100k x 100k
table filled as 2, 4 and 8 row panels (include/nw_panel.h) and checked
against the restatement's fixture (tests/golden/big_colchain.json: corner,
greatest |H|, branch count and the whole-table column-chained hashes of
scores and direction codes), and the 1M x 1M score-only fill as 8 panels
against tests/golden/big_scoreonly.json (corner, FNV of the last column).

The panels are an in-process group on device 0 (45 GB in all), so the
hand-off between panels is the very kernel-to-kernel boundary-row transport
the one-process-per-GPU IPC path uses, minus the xGMI hop.  The per-column
FNV states travel from panel to panel (nw_panel_hash_columns), so the folded
hashes are those of one whole table.  With the default kernel choice
(`auto`) a panel of 100k x 50k rows or fewer has no more 64-row stripes than
the chip has SIMDs and runs the one-row column-scan kernel; NW_KERNEL=pair
forces the two-rows-per-lane kernel, so its panel hand-off (credit wait in
the publisher wave, row-above snapshot, whole 128-row stripes) runs against
the fixture at scale as well.
"""
import numpy as np
import pytest

import nw_amd
from conftest import load_golden

pytestmark = pytest.mark.gpu

BIG = load_golden("big_colchain.json")[0]


@pytest.fixture(autouse=True)
def default_kernel(monkeypatch):
    monkeypatch.delenv("NW_KERNEL", raising=False)
    monkeypatch.delenv("NW_WAVES", raising=False)


@pytest.mark.parametrize("n,kernel", [(2, "auto"), (4, "auto"), (8, "auto"), (2, "pair"), (8, "pair")])
def test_group_panels_100k_match_fixture(monkeypatch, n, kernel):
    if kernel != "auto":
        monkeypatch.setenv("NW_KERNEL", kernel)
    L1, L2 = BIG["L1"], BIG["L2"]
    m, k, d = BIG["m"], BIG["k"], BIG["d"]
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * n, L1, L2, nw_amd.NW_OUT_ALL)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        rows = [p.rows() for p in panels]
        assert sum(r for _, r in rows) == L2
        assert all(r % 128 == 0 for _, r in rows[:-1])
        for _ in range(2):   # a second fill over the first one's granules and credits
            nw_amd.Panel.group_fill(panels, m, k, d, nw_amd.NW_OUT_ALL)
        st = panels[-1].stats()
        assert (st.corner, st.greatest_abs_interior, st.branch_count) == (BIG["corner"], BIG["gav"],
                                                                           BIG["branch_count"])
        # the last panel's last column ends in the corner
        assert int(panels[-1].table.last_column()[-1]) == BIG["corner"]
        state = nw_amd.hash_states(L1)
        for p in panels:
            p.hash_columns(state)
        hH, hD = nw_amd.hash_fold(state)
        assert ("%016x" % hH, "%016x" % hD) == (BIG["hH2"], BIG["hD2"])
    finally:
        for p in panels:
            p.close()


def test_group_panels_1m_score_only_8_panels_match_fixture():
    """configs[4] in its 8-GPU split: 1M x 1M score-only as 8 row panels (here
    on one device): the corner and the FNV of the whole last column
    H[L1][0..L2], stitched from the panels' own rows, against the fixture the
    oracle's multithreaded restatement wrote."""
    g = load_golden("big_scoreonly.json")[0]
    L1, L2 = g["L1"], g["L2"]
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * 8, L1, L2, nw_amd.NW_OUT_STATS)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        rows = [p.rows() for p in panels]
        assert sum(r for _, r in rows) == L2 and all(r > 0 for _, r in rows)
        for _ in range(2):
            nw_amd.Panel.group_fill(panels, g["m"], g["k"], g["d"], 0)
        assert panels[0].stats().corner == g["corner"]
        parts = []
        for p in panels:
            base, _ = p.rows()
            col = p.table.last_column()
            parts.append(col if base == 0 else col[1:])      # a panel's row 0 is the panel above's last row
        last = np.concatenate(parts)
        assert last.shape == (L2 + 1,)
        assert int(last[-1]) == g["corner"]
        import oracle_lib as O
        assert "%016x" % O.fnv(last) == g["lastcol_fnv"]
    finally:
        for p in panels:
            p.close()


def test_hash_columns_chain_equals_whole_table_hash():
    """Chaining per-column states over row panels == nw_table_hash of one table."""
    L1, L2 = 5000, 3001
    s1, s2 = nw_amd.gen_dna(7, L1), nw_amd.gen_dna(8, L2)
    with nw_amd.Table(L1, L2) as t:
        t.set_sequences(s1, s2)
        t.fill(2, 3, 5, nw_amd.NW_OUT_ALL)
        whole = t.hash()
        state = nw_amd.hash_states(L1)
        t.hash_columns(0, state)
        assert nw_amd.hash_fold(state) == whole
    panels = nw_amd.Panel.group([0, 0, 0], L1, L2, nw_amd.NW_OUT_ALL)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, 2, 3, 5, nw_amd.NW_OUT_ALL)
        state = nw_amd.hash_states(L1)
        for p in panels:
            p.hash_columns(state)
        assert nw_amd.hash_fold(state) == whole
    finally:
        for p in panels:
            p.close()
