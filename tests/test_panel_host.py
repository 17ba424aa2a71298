"""Row-panel host logic on CPU (include/nw_panel.h; no GPU needed).

* nw_panel_partition / nw_panel_chain / nw_panel_reduce from the product
  library (pure host code, callable without a device);
* the panel protocol itself -- row bands chained by their boundary row --
  run with the CPU oracle as the band filler, in one process and across a
  world_size-2 gloo process group using bench_multi.py's control helpers.
  The assembled table and the reduced stats must equal a single full fill.
"""
import os
import socket

import numpy as np
import pytest

import nw_amd
import oracle_lib as O


def _parts(L2, n):
    return [nw_amd.panel_partition(L2, n, r) for r in range(n)]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("L2", [0, 1, 63, 64, 65, 130, 511, 1000, 4097, 100_000, 1_000_000])
def test_partition_covers_rows(L2, n):
    parts = _parts(L2, n)
    pos = 0
    sizes = []
    for r, (base, rows) in enumerate(parts):
        assert base == pos or rows == 0
        assert base % 128 == 0 or rows == 0
        pos = base + rows if rows else pos
        sizes.append(rows)
    assert pos == L2 and sum(sizes) == L2
    nonempty = [i for i, s in enumerate(sizes) if s]
    for i in nonempty[:-1]:
        assert sizes[i] % 128 == 0, "a feeding panel must hold whole 128-row stripes"
    if nonempty:
        stripes = [-(-sizes[i] // 128) for i in range(n)]
        assert max(stripes) - min(stripes) <= 1


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("L2", [0, 1, 65, 130, 100_000])
def test_chain_is_consistent(L2, n):
    chain = [nw_amd.panel_chain(L2, n, r) for r in range(n)]
    parts = _parts(L2, n)
    live = [r for r in range(n) if parts[r][1] > 0]
    for r, (prev, nxt, pos) in enumerate(chain):
        if r not in live:
            assert (prev, nxt, pos) == (-1, -1, -1)
            continue
        i = live.index(r)
        assert pos == i
        assert prev == (live[i - 1] if i > 0 else -1)
        assert nxt == (live[i + 1] if i + 1 < len(live) else -1)
        if nxt >= 0:
            assert chain[nxt][0] == r
    # two communicators: a rank's send link and receive link differ in parity
    for r in live:
        prev, nxt, pos = chain[r]
        if prev >= 0 and nxt >= 0:
            assert (pos - 1) & 1 != pos & 1


def test_partition_bad_args():
    with pytest.raises(nw_amd.NWError):
        nw_amd.panel_partition(-1, 2, 0)
    with pytest.raises(nw_amd.NWError):
        nw_amd.panel_partition(10, 2, 2)
    with pytest.raises(nw_amd.NWError):
        nw_amd.panel_chain(10, 0, 0)


def _rec(err=0, has_corner=0, corner=0, gav=0, bc=0, seed=0, rows=0):
    return [err, has_corner, corner, gav, bc, seed, rows, 0]


def test_reduce_semantics():
    rc, st = nw_amd.panel_reduce([_rec(gav=5, bc=3, seed=-9, rows=64), _rec(has_corner=1, corner=12, gav=9, bc=4,
                                                                          seed=-9, rows=10)])
    assert rc == 0 and (st.corner, st.greatest_abs_interior, st.branch_count) == (12, 9, 7)
    # no panel holds the corner (L1 == 0 or L2 == 0): the seed corner
    rc, st = nw_amd.panel_reduce([_rec(seed=-17), _rec(seed=-17)])
    assert rc == 0 and st.corner == -17
    # branch_count wraps like the reference's unsigned counter
    rc, st = nw_amd.panel_reduce([_rec(bc=0xFFFFFFFF), _rec(bc=2)])
    assert st.branch_count == 1
    # the root cause wins over the NW_ERR_PEER it caused downstream
    rc, _ = nw_amd.panel_reduce([_rec(), _rec(err=nw_amd.NW_ERR_PEER), _rec(err=nw_amd.NW_ERR_TIMEOUT)])
    assert rc == nw_amd.NW_ERR_TIMEOUT
    rc, _ = nw_amd.panel_reduce([_rec(), _rec(err=nw_amd.NW_ERR_PEER)])
    assert rc == nw_amd.NW_ERR_PEER


def _band_fill(s1, s2, L2, n, r, top, m, k, d):
    base, rows = nw_amd.panel_partition(L2, n, r)
    return base, rows, O.fill_band(s1, s2[base:base + rows], base, top, m, k, d)


def _seed_row(L1, d):
    return (-np.arange(L1 + 1, dtype=np.int64) * d).astype(np.int32)


@pytest.mark.parametrize("L1,L2,n,mkd", [(300, 517, 3, (2, 3, 5)), (97, 130, 2, (1, 1, 1)), (64, 65, 4, (1, 2, 1)),
                                         (200, 1000, 5, (3, 1, 2)), (50, 10, 3, (1, 1, 1))])
def test_band_chain_equals_full_fill(L1, L2, n, mkd):
    m, k, d = mkd
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    H, D, st = O.fill(s1, s2, m, k, d)
    top = _seed_row(L1, d)
    recs = []
    for r in range(n):
        base, rows, (Hb, Db, sb) = _band_fill(s1, s2, L2, n, r, top, m, k, d)
        if rows:
            np.testing.assert_array_equal(Hb, H[:, base:base + rows + 1])
            np.testing.assert_array_equal(Db[:, 1:], D[:, base + 1:base + rows + 1])
            top = Hb[:, -1].copy()
        prev, nxt, _ = nw_amd.panel_chain(L2, n, r)
        recs.append(_rec(has_corner=int(rows > 0 and nxt < 0), corner=sb[0], gav=sb[1], bc=sb[2],
                         seed=-(L1 + L2) * d, rows=rows))
    rc, got = nw_amd.panel_reduce(recs)
    assert rc == 0
    assert (got.corner, got.greatest_abs_interior, got.branch_count) == st


# ------------------------------------------------------- world_size-2 gloo
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, L1, L2, mkd, out_path):
    import torch
    import torch.distributed as dist

    import bench_multi
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, k, d = mkd
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    base, rows = nw_amd.panel_partition(L2, world, rank)
    prev, nxt, _ = nw_amd.panel_chain(L2, world, rank)
    # the boundary row travels rank -> rank+1, as the panels' hand-off does
    top = torch.from_numpy(_seed_row(L1, d))
    if prev >= 0:
        dist.recv(top, src=prev)
    Hb, Db, sb = O.fill_band(s1, s2[base:base + rows], base, top.numpy(), m, k, d)
    if nxt >= 0:
        dist.send(torch.from_numpy(Hb[:, -1].copy()), dst=nxt)
    rec = _rec(has_corner=int(rows > 0 and nxt < 0), corner=sb[0], gav=sb[1], bc=sb[2], seed=-(L1 + L2) * d,
               rows=rows)
    recs = bench_multi.gather_records(rec)
    slowest = bench_multi.max_over_ranks(float(rank + 1))
    tables = bench_multi.exchange_bytes(Hb[:, 1:].tobytes())
    if rank == 0:
        rc, st = nw_amd.panel_reduce(recs)
        full = np.concatenate([np.frombuffer(t, dtype=np.int32).reshape(L1 + 1, -1) for t in tables], axis=1)
        np.savez(out_path, rc=rc, stats=np.array([st.corner, st.greatest_abs_interior, st.branch_count]),
                 slowest=slowest, table=full, nrec=len(recs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("L1,L2", [(300, 517), (120, 64)])
def test_gloo_two_ranks_chain(tmp_path, L1, L2):
    import torch.multiprocessing as mp
    mkd = (2, 3, 5)
    out = str(tmp_path / "r0.npz")
    mp.spawn(_gloo_worker, args=(2, _free_port(), L1, L2, mkd, out), nprocs=2, join=True)
    z = np.load(out)
    H, _, st = O.fill(O.gen_dna(1, L1), O.gen_dna(2, L2), *mkd)
    assert int(z["rc"]) == 0 and int(z["nrec"]) == 2
    assert tuple(int(x) for x in z["stats"]) == st
    assert float(z["slowest"]) == 2.0
    np.testing.assert_array_equal(z["table"], H[:, 1:])
