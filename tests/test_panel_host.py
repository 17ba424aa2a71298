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


def test_credit_comparison_accepts_later_epochs_and_wraps():
    """The producer's back-pressure wait (needleman-wunsch.c:444-452's wait on
    the left neighbour, moved to one boundary row per panel) accepts the
    awaited epoch or a later one: a consumer whose fill failed posts its
    credit from the host, possibly for the epoch after the awaited one."""
    reached = lambda c, w: bool(nw_amd.load().nw_panel_credit_reached(c, w))
    assert reached(0, 0) and reached(5, 5) and reached(6, 5) and reached(1000, 5)
    assert not reached(4, 5) and not reached(0, 1)
    # epochs wrap from 2^31 - 1 to 1 (bit 31 is the poison bit)
    top = 0x7FFFFFFF
    assert reached(top, top) and reached(1, top) and reached(2, top - 1)
    assert not reached(top - 1, top) and not reached(top, 1)


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


class _OraclePanel:
    """Stands in for a Panel on the CPU: continues the per-column FNV-1a-64
    states over a band's own rows exactly as nw_panel_hash_columns does (the
    first panel hashes global row 0 too, the others start at their first own
    row)."""

    def __init__(self, Hb, Db, first):
        self.H, self.D, self.j0 = Hb, Db, 0 if first else 1

    def hash_columns(self, state):
        P = np.uint64(0x100000001B3)
        with np.errstate(over="ignore"):
            for j in range(self.j0, self.H.shape[1]):
                x = self.H[:, j].astype(np.uint32).astype(np.uint64)
                for b in range(4):
                    state[0] = (state[0] ^ ((x >> np.uint64(8 * b)) & np.uint64(0xFF))) * P
                state[1] = (state[1] ^ self.D[:, j].astype(np.uint64)) * P


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
    if rows and base == 0:
        Db[0, 0], Db[1:, 0] = 0, 4                      # the band's row 0 is the table's seeded row 0
    # every rank takes part, a rank without rows passes the states on untouched
    hashes = bench_multi.chain_hash_states(_OraclePanel(Hb[:, :rows + 1 if rows else 0], Db, base == 0), L1, rank,
                                           world)
    if rank == 0:
        rc, st = nw_amd.panel_reduce(recs)
        full = np.concatenate([np.frombuffer(t, dtype=np.int32).reshape(L1 + 1, -1) for t in tables], axis=1)
        np.savez(out_path, rc=rc, stats=np.array([st.corner, st.greatest_abs_interior, st.branch_count]),
                 slowest=slowest, table=full, nrec=len(recs),
                 hashes=np.array(hashes if hashes else (0, 0), dtype=np.uint64))
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
    # the per-column hash states chained rank to rank fold to the whole table's hashes
    h, e, _ = O.colchain(O.gen_dna(1, L1), O.gen_dna(2, L2), *mkd)
    assert tuple(int(x) for x in z["hashes"]) == (h, e)


# ------------------------------------------- RCCL host proxy (sequencing only)
POISON = 0x80000000


def _blocks(L1, xblk):
    step = 8 * xblk
    return [(off, min(step, L1 - off)) for off in range(0, L1, step)]


@pytest.mark.parametrize("L1,xblk", [(1, 1), (64, 1), (65, 1), (1000, 4), (100_000, 512)])
def test_proxy_posts_every_recv_first_then_sends_in_order(L1, xblk):
    log = []
    rc = nw_amd.panel_proxy_run(L1, xblk, True, True, True,
                                recv=lambda o, c: log.append(("recv", o, c)) or 0,
                                flag=lambda b, spin: 1 if spin >= 2 else 0,
                                poison=lambda o, c: log.append(("poison", o, c)) or 0,
                                send=lambda o, c: log.append(("send", o, c)) or 0)
    assert rc == 0
    blocks = _blocks(L1, xblk)
    assert log == [("recv", o, c) for o, c in blocks] + [("send", o, c) for o, c in blocks]


def test_proxy_poisons_what_the_kernel_never_produced():
    L1, xblk, dead = 1000, 2, 5          # the producer kernel ends after block 4
    log = []
    rc = nw_amd.panel_proxy_run(L1, xblk, False, True, True,
                                flag=lambda b, spin: 1 if b < dead else (-1 if spin > 3 else 0),
                                poison=lambda o, c: log.append(("poison", o, c)) or 0,
                                send=lambda o, c: log.append(("send", o, c)) or 0)
    assert rc == 0
    want = []
    for b, (o, c) in enumerate(_blocks(L1, xblk)):
        if b >= dead:
            want.append(("poison", o, c))
        want.append(("send", o, c))
    assert log == want


def test_proxy_unlaunched_kernel_poisons_every_block_without_polling():
    log = []
    rc = nw_amd.panel_proxy_run(100, 1, False, True, False, flag=lambda b, s: pytest.fail("polled"),
                                poison=lambda o, c: log.append("p") or 0, send=lambda o, c: log.append("s") or 0)
    assert rc == 0 and log == ["p", "s"] * len(_blocks(100, 1))


def test_proxy_stops_at_the_first_transport_failure():
    sent = []
    rc = nw_amd.panel_proxy_run(640, 8, False, True, True, flag=lambda b, s: 1, poison=lambda o, c: 0,
                                send=lambda o, c: (sent.append(o), nw_amd.NW_ERR_HIP if o == 128 else 0)[1])
    assert rc == nw_amd.NW_ERR_HIP and sent == [0, 64, 128]
    posted = []
    rc = nw_amd.panel_proxy_run(640, 8, True, True, True,
                                recv=lambda o, c: (posted.append(o), nw_amd.NW_ERR_HIP if o == 64 else 0)[1],
                                flag=lambda b, s: pytest.fail("no send after a failed recv"))
    assert rc == nw_amd.NW_ERR_HIP and posted == [0, 64]
    # a poison failure is reported after its block went out
    log = []
    rc = nw_amd.panel_proxy_run(200, 8, False, True, False, poison=lambda o, c: nw_amd.NW_ERR_HIP,
                                send=lambda o, c: log.append(o) or 0)
    assert rc == nw_amd.NW_ERR_HIP and log == [0]


def test_proxy_rejects_missing_callbacks():
    assert nw_amd.panel_proxy_run(64, 0, False, True, True, flag=lambda b, s: 1) == nw_amd.NW_ERR_ARG
    assert nw_amd.panel_proxy_run(-1, 1, False, False, True) == nw_amd.NW_ERR_ARG


def _proxy_worker(rank, world, port, L1, L2, mkd, dead, out_path):
    """Two ranks exchange one boundary row through nw_panel_proxy_run with
    gloo point-to-point in the role of ncclSend / ncclRecv: granules
    {epoch, H - d} per column, blocks of 8*xblk, receives posted up front."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, k, d = mkd
    epoch, xblk = 7, 3
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    base, rows = nw_amd.panel_partition(L2, world, rank)
    prev, nxt, _ = nw_amd.panel_chain(L2, world, rank)
    works = []
    if rank == 0:
        Hb, _, _ = O.fill_band(s1, s2[base:base + rows], base, _seed_row(L1, d), m, k, d)
        vals = (Hb[1:, -1].astype(np.int64) - d) & 0xFFFFFFFF
        xout = torch.from_numpy(((epoch << 32) | vals).astype(np.int64))

        def poison(o, c):
            xout[o:o + c] = ((epoch | POISON) << 32) - (1 << 64)   # as int64
            return 0
        rc = nw_amd.panel_proxy_run(L1, xblk, prev >= 0, nxt >= 0, True,
                                    flag=lambda b, spin: 1 if b < dead else -1, poison=poison,
                                    send=lambda o, c: works.append(dist.isend(xout[o:o + c].clone(), dst=nxt)) or 0)
    else:
        xin = torch.zeros(L1, dtype=torch.int64)
        slices = []

        def recv(o, c):
            buf = torch.zeros(c, dtype=torch.int64)
            slices.append((o, buf))
            works.append(dist.irecv(buf, src=prev))
            return 0
        rc = nw_amd.panel_proxy_run(L1, xblk, prev >= 0, nxt >= 0, True, recv=recv)
    for w in works:
        w.wait()
    if rank == 1:
        for o, buf in slices:
            xin[o:o + buf.numel()] = buf
        g = xin.numpy().astype(np.uint64)
        np.savez(out_path, rc=rc, tags=(g >> np.uint64(32)).astype(np.int64),
                 vals=(g & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dead", [10**9, 4])
def test_gloo_two_ranks_proxy_moves_the_boundary_row(tmp_path, dead):
    import torch.multiprocessing as mp
    L1, L2, mkd = 500, 300, (2, 3, 5)
    out = str(tmp_path / "r1.npz")
    mp.spawn(_proxy_worker, args=(2, _free_port(), L1, L2, mkd, dead, out), nprocs=2, join=True)
    z = np.load(out)
    assert int(z["rc"]) == 0
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    H, _, _ = O.fill(s1, s2, *mkd)
    base, rows = nw_amd.panel_partition(L2, 2, 1)
    nblk_ok = min(dead, len(_blocks(L1, 3)))
    ok = min(L1, nblk_ok * 24)
    assert (z["tags"][:ok] == 7).all()
    assert (z["tags"][ok:] == (7 | POISON)).all()
    # the delivered granules are the row above panel 1 (H - d), and filling
    # panel 1 from them gives the whole table's rows
    np.testing.assert_array_equal(z["vals"][:ok], H[1:ok + 1, base] - mkd[2])
    if ok == L1:
        top = np.concatenate([[H[0, base]], z["vals"] + mkd[2]]).astype(np.int32)
        Hb, _, _ = O.fill_band(s1, s2[base:], base, top, *mkd)
        np.testing.assert_array_equal(Hb, H[:, base:])
