"""Config C4 on the GPU: the 100k x 100k table filled as 2 and 4 row panels
(include/nw_panel.h) and checked against the restatement's fixture
(tests/golden/big_colchain.json: corner, greatest |H|, branch count and the
whole-table column-chained hashes of scores and direction codes).

The panels are an in-process group on device 0 (45 GB in all), so the
hand-off between panels is the very kernel-to-kernel boundary-row transport
the one-process-per-GPU IPC path uses, minus the xGMI hop.  The per-column
FNV states travel from panel to panel (nw_panel_hash_columns), so the folded
hashes are those of one whole table.  The kernel is the default (`auto`:
the two-rows-per-lane pair kernel at this size).
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


@pytest.mark.parametrize("n", [2, 4])
def test_group_panels_100k_match_fixture(n):
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
