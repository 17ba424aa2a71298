"""Host I/O of the device-resident table: pinned
sequence upload and streamed slice copies (nw_table_copy_scores /
nw_table_copy_codes through two device staging buffers, DMA straight into
pinned destinations or through pinned bounce buffers), checked against the
CPU oracle and against the device's own per-column hashes."""
import numpy as np
import pytest

import nw_amd
import oracle_lib as O

pytestmark = pytest.mark.gpu


def test_streamed_slices_match_oracle_pinned_and_pageable():
    # 40001 columns x 1000 rows of int32 = 160 MB: three 64 MB staging blocks
    L1, L2 = 40000, 999
    s1, s2 = O.gen_dna(11, L1), O.gen_dna(12, L2)
    Ho, Do, _ = O.fill(s1, s2, 2, 3, 5)
    with nw_amd.Table(L1, L2) as t:
        t.set_sequences(s1, s2)
        t.fill(2, 3, 5, nw_amd.NW_OUT_ALL)
        H = t.scores()
        assert np.array_equal(H, Ho)
        io = t.io_stats()
        assert io["copy_bytes"] == Ho.nbytes and io["copy_ms"] > 0
        with nw_amd.HostBuffer((L1 + 1, L2 + 1), np.int32) as hb:
            t.scores(out=hb.array)
            assert np.array_equal(hb.array, Ho)
        # odd column ranges, both kinds of destination
        for i0, i1 in ((0, 1), (17, 16801), (16776, 33555), (39999, 40001)):
            assert np.array_equal(t.scores(i0, i1), Ho[i0:i1])
            assert np.array_equal(t.codes(i0, i1), Do[i0:i1])
            with nw_amd.HostBuffer((i1 - i0, L2 + 1), np.uint8) as hb:
                t.codes(i0, i1, out=hb.array)
                assert np.array_equal(hb.array, Do[i0:i1])


def test_out_must_fit():
    with nw_amd.Table(10, 10) as t:
        t.set_sequences(b"ACGTACGTAC", b"ACGTACGTAA")
        t.fill(1, 1, 1, nw_amd.NW_OUT_ALL)
        with pytest.raises(ValueError):
            t.scores(out=np.empty((11, 10), dtype=np.int32))
        with pytest.raises(ValueError):
            t.scores(out=np.empty((11, 11), dtype=np.int64))


def test_gigabyte_slice_of_the_100k_table():
    """A 1.08 GB score slice (2700 columns of 100,001 rows) of the 100k x 100k
    table, streamed into pinned and into pageable memory; every column's
    FNV-1a-64 equals the device's own column hash of the same table."""
    L1 = L2 = 100_000
    i0, i1 = 48_650, 51_350
    with nw_amd.Table(L1, L2) as t:
        t.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
        t.fill(1, 1, 1, nw_amd.NW_OUT_ALL)
        state = nw_amd.hash_states(L1)
        t.hash_columns(0, state)
        want = state[0][i0:i1]
        with nw_amd.HostBuffer((i1 - i0, L2 + 1), np.int32) as hb:
            t.scores(i0, i1, out=hb.array)
            io = t.io_stats()
            assert io["copy_bytes"] == hb.array.nbytes > 10**9
            got = [O.fnv(hb.array[c]) for c in range(0, i1 - i0, 97)]
            assert got == [int(x) for x in want[::97]]
            print(f"pinned: {io['copy_bytes'] / io['copy_ms'] / 1e6:.1f} GB/s")
            pageable = t.scores(i0, i1)
            io = t.io_stats()
            print(f"pageable: {io['copy_bytes'] / io['copy_ms'] / 1e6:.1f} GB/s")
            assert np.array_equal(pageable, hb.array)


def test_megabase_upload_then_fill():
    """1M-long top string: pinned upload (coded to 2-bit symbols on the way),
    then a score-only fill whose last column matches the oracle."""
    L1, L2 = 1_000_000, 256
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    with nw_amd.Table(L1, L2, 0) as t:
        t.set_sequences(s1, s2)
        io = t.io_stats()
        assert io["upload_bytes"] == L1 + L2 and io["upload_ms"] > 0
        t.fill(1, 1, 1, 0)
        corner, hlast = O.score_only(s1, s2, 1, 1, 1)
        lastcol = t.last_column()
        assert int(lastcol[-1]) == corner
        assert O.fnv(lastcol) == hlast


def test_host_buffer_views_keep_the_pinned_memory_alive():
    """An array taken out of a HostBuffer outlives it: the pinned memory is
    released with the last view, not with the wrapper."""
    import gc
    a = nw_amd.HostBuffer((1 << 16,), np.int32).array      # the wrapper is gone at once
    gc.collect()
    a[:] = 7
    hb = nw_amd.HostBuffer((4, 4), np.int32)
    v = hb.array[1:]
    hb.close()
    gc.collect()
    v[:] = 3
    churn = [nw_amd.HostBuffer((1 << 16,), np.int32) for _ in range(8)]   # reuse of freed pinned pages would show
    for c in churn:
        c.array[:] = -1
    assert int(a.sum()) == 7 << 16 and int(v.sum()) == 36
