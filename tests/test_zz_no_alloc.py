"""nw_fill_noalloc (include/nw_fill.h): the fill that allocates nothing, on
caller-provided device buffers, against the existing entry point nw_fill()
-- bit-exact scores, direction codes, last column and stats -- on two calls
in a row, the second with a smaller input (the static scratch array keeps the
first call's contents).

Runs on an MI355X only (`pytest -m gpu`); collected last (see the file name):
a failure here must not hide the other tests under `pytest -x`.
"""
import ctypes

import numpy as np
import pytest

import hip_mem
import nw_amd
import oracle_lib as O

pytestmark = pytest.mark.gpu

ALL = nw_amd.NW_OUT_ALL


class Buffers:
    """Device buffers of one caller, sized once for the largest input."""

    def __init__(self, L1, L2):
        self.s1 = hip_mem.DeviceBuffer(L1 + 1)
        self.s2 = hip_mem.DeviceBuffer(L2 + 1)
        self.tiles = hip_mem.DeviceBuffer(4 * nw_amd.noalloc_score_elems(L1, L2), fill=0x5A)
        self.words = hip_mem.DeviceBuffer(4 * nw_amd.noalloc_dir_words(L1, L2), fill=0x5A)
        self.last = hip_mem.DeviceBuffer(4 * (L2 + 1), fill=0x5A)
        self.res = hip_mem.DeviceBuffer(ctypes.sizeof(nw_amd.NoallocResult), fill=0x5A)

    def close(self):
        for b in (self.s1, self.s2, self.tiles, self.words, self.last, self.res):
            b.close()


def _run(buf, s1, s2, mkd, mask, stream=None):
    L1, L2 = len(s1), len(s2)
    buf.s1.upload(s1)
    buf.s2.upload(s2)
    rc = nw_amd.fill_noalloc(0, stream.handle if stream else None, buf.s1.ptr, L1, buf.s2.ptr, L2, *mkd, mask,
                             buf.tiles.ptr if mask & nw_amd.NW_OUT_SCORES else 0,
                             buf.words.ptr if mask & nw_amd.NW_OUT_DIRS else 0, buf.last.ptr, buf.res.ptr)
    assert rc == 0, nw_amd.load().nw_last_error()
    if stream:
        stream.synchronize()
    else:
        hip_mem.device_synchronize()
    res = nw_amd.NoallocResult.from_buffer_copy(buf.res.download(np.uint8, ctypes.sizeof(nw_amd.NoallocResult)))
    last = buf.last.download(np.int32, L2 + 1)
    tiles = buf.tiles.download(np.int32, nw_amd.noalloc_score_elems(L1, L2)) if mask & nw_amd.NW_OUT_SCORES else None
    words = buf.words.download(np.uint32, nw_amd.noalloc_dir_words(L1, L2)) if mask & nw_amd.NW_OUT_DIRS else None
    if tiles is None and words is None:
        return res, last, None, None
    H, C = nw_amd.decode_tiles(tiles, words, L1, L2, mkd[2])
    return res, last, (H if tiles is not None else None), (C if words is not None else None)


def _check(buf, s1, s2, mkd, mask=ALL, stream=None):
    res, last, H, C = _run(buf, s1, s2, mkd, mask, stream)
    # the existing entry point, on the same inputs
    Hx, Cx, stx = nw_amd.fill(s1, s2, *mkd)
    assert res.status == 0
    assert res.stats.corner == stx.corner
    if mask & nw_amd.NW_OUT_STATS:
        assert (res.stats.greatest_abs_interior, res.stats.branch_count) == (stx.greatest_abs_interior, stx.branch_count)
    else:
        assert (res.stats.greatest_abs_interior, res.stats.branch_count) == (0, 0)
    np.testing.assert_array_equal(last, Hx[-1])
    if H is not None:
        np.testing.assert_array_equal(H, Hx)
    if C is not None:
        np.testing.assert_array_equal(C, Cx)
    # and the CPU oracle (the checker)
    Ho, Co, sto = O.fill(s1, s2, *mkd)
    assert res.stats.corner == sto[0]
    if H is not None:
        np.testing.assert_array_equal(H, Ho)
    if C is not None:
        np.testing.assert_array_equal(C, Co)


def test_two_calls_in_a_row_second_smaller():
    buf = Buffers(3001, 2003)
    try:
        _check(buf, O.gen_dna(21, 3001), O.gen_dna(22, 2003), (2, 3, 5))
        _check(buf, O.gen_dna(23, 517), O.gen_dna(24, 300), (1, 1, 1))      # smaller: stale scratch around it
        _check(buf, O.gen_dna(25, 9), O.gen_dna(26, 65), (5, -4, 2))
        _check(buf, O.gen_dna(21, 3001), O.gen_dna(22, 2003), (2, 3, 5))     # and the first again
    finally:
        buf.close()


@pytest.mark.parametrize("mask", [nw_amd.NW_OUT_SCORES | nw_amd.NW_OUT_DIRS, nw_amd.NW_OUT_SCORES,
                                  nw_amd.NW_OUT_DIRS, nw_amd.NW_OUT_STATS, 0])
def test_every_output_mask_on_a_stream(mask):
    buf = Buffers(1500, 1300)
    st = hip_mem.Stream()
    try:
        rng = np.random.default_rng(2)
        s1 = bytes(rng.integers(1, 256, 1500, dtype=np.uint8))     # arbitrary bytes
        s2 = bytes(rng.integers(1, 256, 1300, dtype=np.uint8))
        _check(buf, s1, s2, (3, 2, 1), mask, st)
        _check(buf, O.gen_dna(5, 700), O.gen_dna(6, 64 * 9 + 17), (1, 1, 1), mask, st)
    finally:
        st.close()
        buf.close()


@pytest.mark.parametrize("L1,L2", [(0, 0), (0, 40), (40, 0), (1, 1), (8, 64), (64, 1)])
def test_edges(L1, L2):
    buf = Buffers(64, 64)
    try:
        _check(buf, O.gen_dna(1, L1), O.gen_dna(2, L2), (1, 1, 1))
    finally:
        buf.close()


def test_maximum_size_runs_and_larger_is_rejected():
    L = nw_amd.NW_NOALLOC_MAX_L1
    s1, s2 = O.gen_dna(1, L), O.gen_dna(2, nw_amd.NW_NOALLOC_MAX_L2)
    buf = Buffers(L, nw_amd.NW_NOALLOC_MAX_L2)
    try:
        # score-only at the maximum: corner and last column against the oracle
        res, last, _, _ = _run(buf, s1, s2, (1, 1, 1), 0)
        c, hl = O.score_only(s1, s2, 1, 1, 1)
        assert res.status == 0 and res.stats.corner == c
        assert O.fnv(last) == hl
        for a, b in ((L + 1, 10), (10, nw_amd.NW_NOALLOC_MAX_L2 + 1)):
            rc = nw_amd.fill_noalloc(0, None, buf.s1.ptr, a, buf.s2.ptr, b, 1, 1, 1, 0, 0, 0, buf.last.ptr, buf.res.ptr)
            assert rc == nw_amd.NW_ERR_ARG
            assert b"beyond the scratch array's limit" in nw_amd.load().nw_last_error()
        # a missing output buffer and an overflowing penalty are rejected too
        assert nw_amd.fill_noalloc(0, None, buf.s1.ptr, 10, buf.s2.ptr, 10, 1, 1, 1, nw_amd.NW_OUT_SCORES) == nw_amd.NW_ERR_ARG
        assert nw_amd.fill_noalloc(0, None, buf.s1.ptr, 4000, buf.s2.ptr, 4000, 1, 1, 1 << 20, 0, 0, 0,
                                   buf.last.ptr, buf.res.ptr) == nw_amd.NW_ERR_RANGE
    finally:
        buf.close()
