"""Row panels on the GPU (include/nw_panel.h) against the CPU oracle.

An in-process group of 2-3 panels on device 0 runs the very hand-off the
multi-GPU path uses (the producer's kernel stores its bottom row into the
consumer's boundary buffer, the consumer's loader wave polls the tags); a
2-process run on device 0 exercises the hipIpc transport between processes.
Every panel's local rows must equal the matching rows of one full oracle
fill, bit for bit, and the reduced stats the full table's stats.
"""
import os
import socket
import subprocess
import sys

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

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _check_panels(panels, s1, s2, m, k, d, scores=True, codes=True):
    H, D, st = O.fill(s1, s2, m, k, d)
    L1 = len(s1)
    for p in panels:
        base, rows = p.rows()
        if rows == 0:
            continue
        t = p.table
        if scores:
            np.testing.assert_array_equal(t.scores(), H[:, base:base + rows + 1],
                                          err_msg=f"panel {p.rank} scores (rows {base}..{base + rows})")
        if codes:
            np.testing.assert_array_equal(t.codes()[:, 1:], D[:, base + 1:base + rows + 1],
                                          err_msg=f"panel {p.rank} codes")
        np.testing.assert_array_equal(t.last_column(), H[L1, base:base + rows + 1])
    got = panels[0].stats()
    assert (got.corner, got.greatest_abs_interior, got.branch_count) == st


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("L1,L2,mkd", [(300, 517, (2, 3, 5)), (1000, 700, (1, 1, 1)), (9, 200, (1, 2, 1)),
                                       (2049, 1300, (3, 1, 2))])
def test_group_panels_match_oracle(n, L1, L2, mkd):
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * n, L1, L2)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        for _ in range(2):   # a second fill: new epoch over stale boundary granules
            nw_amd.Panel.group_fill(panels, *mkd, nw_amd.NW_OUT_ALL)
        _check_panels(panels, s1, s2, *mkd)
    finally:
        for p in panels:
            p.close()


@pytest.mark.parametrize("L1,L2,n", [(100, 70, 3), (50, 64, 2), (0, 300, 2), (300, 0, 2), (1, 1, 3)])
def test_group_panels_edges(L1, L2, n):
    """Fewer stripes than panels (empty panels), empty sequences."""
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * n, max(L1, 1), max(L2, 1))
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, 1, 1, 1, nw_amd.NW_OUT_ALL)
        _check_panels(panels, s1, s2, 1, 1, 1)
    finally:
        for p in panels:
            p.close()


@pytest.mark.parametrize("waves", ["1", "2", "8", "15"])
def test_group_panels_every_wave_count(waves, monkeypatch):
    monkeypatch.setenv("NW_WAVES", waves)
    s1, s2 = O.gen_dna(1, 777), O.gen_dna(2, 1500)
    panels = nw_amd.Panel.group([0, 0], 777, 1500)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, 2, 3, 5, nw_amd.NW_OUT_ALL)
        _check_panels(panels, s1, s2, 2, 3, 5)
    finally:
        for p in panels:
            p.close()


def test_group_panels_score_only():
    L1, L2 = 3000, 2000
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    H, _, st = O.fill(s1, s2, 1, 1, 1, codes=False)
    panels = nw_amd.Panel.group([0, 0, 0], L1, L2, nw_amd.NW_OUT_STATS)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, 1, 1, 1, nw_amd.NW_OUT_STATS)
        for p in panels:
            base, rows = p.rows()
            np.testing.assert_array_equal(p.table.last_column(), H[L1, base:base + rows + 1])
        got = panels[1].stats()
        assert (got.corner, got.greatest_abs_interior, got.branch_count) == st
    finally:
        for p in panels:
            p.close()


def test_group_panels_10k():
    """10k x 10k in 3 panels: per-panel scores/codes vs one oracle fill."""
    L1 = L2 = 10_000
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0, 0, 0], L1, L2)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        nw_amd.Panel.group_fill(panels, 1, 1, 1, nw_amd.NW_OUT_ALL)
        _check_panels(panels, s1, s2, 1, 1, 1)
    finally:
        for p in panels:
            p.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ipc(tmp_path, L1, L2, mkd, world=2, extra_env=None):
    out = str(tmp_path / "ipc.npz")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "panel_ipc_worker.py"), out,
                                       str(L1), str(L2), *map(str, mkd), "ipc", "0"], env=env))
    rcs = [p.wait(timeout=100) for p in procs]
    assert rcs == [0] * world
    return out


@pytest.mark.parametrize("L1,L2,mkd", [(2000, 1500, (2, 3, 5)), (500, 100, (1, 1, 1))])
def test_ipc_two_processes(tmp_path, L1, L2, mkd):
    """Two processes, one panel each, on device 0, boundary over hipIpc."""
    out = _run_ipc(tmp_path, L1, L2, mkd)
    _check_ipc(out, L1, L2, mkd)


@pytest.mark.parametrize("delay_rank,world", [(1, 2), (2, 3)])
def test_ipc_back_to_back_delayed_consumer(tmp_path, delay_rank, world):
    """Back-to-back fills with different m, k, d while one consumer starts
    every fill 0.4 s late: the panels above run ahead into the next fill and
    must wait for its credit (without back-pressure the producer
    overwrote a boundary row still being read, and the consumer timed out)."""
    L1, L2 = 3000, 1000
    seq = [(2, 3, 5), (1, 1, 1), (3, 1, 2), (1, 2, 1)]
    out = _run_ipc(tmp_path, L1, L2, seq[-1], world,
                   {"NW_TEST_MKD_SEQ": ";".join(",".join(map(str, x)) for x in seq),
                    "NW_TEST_DELAY": f"{delay_rank}:0.4"})
    _check_ipc(out, L1, L2, seq[-1])


def _check_ipc(out, L1, L2, mkd):
    z = np.load(out)
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    H, D, st = O.fill(s1, s2, *mkd)
    assert int(z["rc"]) == 0
    assert tuple(int(x) for x in z["stats"]) == st
    for rank, base, rows, rc in z["meta"]:
        assert rc == 0
        if rows == 0:
            continue
        np.testing.assert_array_equal(z[f"H{rank}"], H[:, base:base + rows + 1])
        np.testing.assert_array_equal(z[f"D{rank}"][:, 1:], D[:, base + 1:base + rows + 1])
