"""Python binding (ctypes) of the MI355X Needleman-Wunsch fill, include/nw_fill.h
and include/nw_panel.h.

This mirrors the reference's hot-path seam -- ``compute_table_scores(C)``
(needleman-wunsch.c:583-626), called once per alignment by the driver at
needleman-wunsch.c:662 -- as two entry points:

* :func:`fill` -- one-shot fill into host arrays (scores, direction codes,
  stats), what the CLI's traceback/printer consume;
* :class:`Table` -- a device-resident table (the 100k x 100k path: the table
  stays in HBM; hashes, slices and stats are pulled on demand);
* :class:`Panel` -- one row panel of a table split across GPUs (one process
  per GPU over hipIpc or RCCL, or an in-process group).

The library is required: importing works without it (so CPU-only tooling can
inspect the module), but every call raises :class:`NWError` when
``lib/libnwfill.so`` is missing or no gfx950 GPU is visible.  There is no CPU
fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NW_LIB") or os.path.join(HERE, "lib", "libnwfill.so")

NW_OUT_SCORES = 1
NW_OUT_DIRS = 2
NW_OUT_STATS = 4
NW_OUT_ALL = NW_OUT_SCORES | NW_OUT_DIRS | NW_OUT_STATS

NW_OK = 0
NW_ERR_ARG = -1
NW_ERR_NODEVICE = -2
NW_ERR_OOM = -3
NW_ERR_HIP = -4
NW_ERR_RANGE = -5
NW_ERR_TIMEOUT = -6
NW_ERR_STATE = -7
NW_ERR_PEER = -8

NW_PANEL_GROUP = 0
NW_PANEL_IPC = 1
NW_PANEL_RCCL = 2
PANEL_ID_BYTES = 256
PANEL_IPC_BYTES = 64
PANEL_REC = 8

# Exported symbols of include/nw_fill.h (checked by tests/test_abi.py).
EXPORTS = (
    "nw_strerror", "nw_last_error", "nw_fill",
    "nw_table_create", "nw_table_destroy", "nw_table_set_sequences", "nw_table_fill",
    "nw_table_stats", "nw_table_elapsed_ms", "nw_table_hash", "nw_table_copy_scores",
    "nw_table_copy_codes", "nw_table_copy_last_column", "nw_table_score_pitch", "nw_table_waves",
    "nw_table_trace", "nw_table_count_alignments", "nw_table_first_path", "nw_table_walk_elapsed_ms",
    "nw_first_path_banded", "nw_table_hash_columns", "nw_hash_fold",
    "nw_host_alloc", "nw_host_free", "nw_table_io_stats", "nw_table_enumerate_paths",
    "nw_table_layout", "nw_table_device_buffers", "nw_fill_noalloc",
    # include/nw_panel.h
    "nw_panel_partition", "nw_panel_chain", "nw_panel_get_id", "nw_panel_create", "nw_panel_ipc_handle",
    "nw_panel_ipc_connect", "nw_panel_group_create", "nw_panel_destroy", "nw_panel_set_sequences",
    "nw_panel_fill", "nw_panel_group_fill", "nw_panel_stats", "nw_panel_record", "nw_panel_reduce",
    "nw_panel_rows", "nw_panel_table", "nw_panel_elapsed_ms", "nw_panel_hash_columns", "nw_panel_proxy_run",
    "nw_panel_credit_reached",
)


class NWError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"{msg} (rc={rc})")
        self.rc = rc


class Layout(ctypes.Structure):
    """nw_layout (include/nw_fill.h): how the last fill laid the table out in HBM."""
    _fields_ = [("score_pitch", ctypes.c_int64), ("NQ", ctypes.c_int64), ("pair", ctypes.c_int32),
                ("skew", ctypes.c_int32), ("raw", ctypes.c_int32), ("SQ", ctypes.c_int32), ("SR", ctypes.c_int32),
                ("d", ctypes.c_int32), ("has_scores", ctypes.c_int32), ("has_dirs", ctypes.c_int32)]


class _Stats(ctypes.Structure):
    _fields_ = [("corner", ctypes.c_int32), ("greatest_abs_interior", ctypes.c_int32),
                ("branch_count", ctypes.c_uint32)]


class NoallocResult(ctypes.Structure):
    """nw_noalloc_result (include/nw_fill.h)."""
    _fields_ = [("status", ctypes.c_int32), ("stats", _Stats)]


NW_NOALLOC_MAX_L1 = 16384
NW_NOALLOC_MAX_L2 = 16384


def noalloc_score_elems(L1: int, L2: int) -> int:
    """NW_NOALLOC_SCORE_ELEMS: int32 elements of the caller's score-tile buffer."""
    return ((L2 + 63) // 64 + 1) * ((L1 + 7) // 8 + 8) * 512


def noalloc_dir_words(L1: int, L2: int) -> int:
    """NW_NOALLOC_DIR_WORDS: uint32 words of the caller's code-word buffer."""
    return ((L2 + 63) // 64 + 1) * ((L1 + 7) // 8 + 9) * 64


def fill_noalloc(device: int, stream, s1_dev: int, L1: int, s2_dev: int, L2: int, m: int, k: int, d: int,
                 out_mask: int, score_tiles_dev: int = 0, dir_words_dev: int = 0, last_column_dev: int = 0,
                 result_dev: int = 0) -> int:
    """nw_fill_noalloc on raw device addresses; returns the status code (the
    work is only enqueued on `stream`)."""
    return load().nw_fill_noalloc(device, stream, s1_dev or None, L1, s2_dev or None, L2, m, k, d, out_mask,
                                  score_tiles_dev or None, dir_words_dev or None, last_column_dev or None,
                                  result_dev or None)


def decode_tiles(tiles: np.ndarray, words: np.ndarray | None, L1: int, L2: int, d: int, lay=None):
    """Dense (H, codes) from the device layout of include/nw_fill.h -- what a
    zero-copy consumer computes.  tiles / words: the raw device buffers copied
    to the host; lay: a Layout (None = the plain variant)."""
    NQ = int(lay.NQ) if lay is not None else (L1 + 7) // 8
    P = int(lay.score_pitch) if lay is not None else 512 * NQ
    pair, skew, raw = (int(lay.pair), int(lay.skew), int(lay.raw)) if lay is not None else (0, 0, 0)
    H = np.empty((L1 + 1, L2 + 1), dtype=np.int64)
    H[:, 0] = -np.arange(L1 + 1, dtype=np.int64) * d
    H[0, :] = -np.arange(L2 + 1, dtype=np.int64) * d
    C = np.zeros((L1 + 1, L2 + 1), dtype=np.uint8)
    C[1:, 0] = 4
    C[0, 1:] = 2
    if L1 and L2:
        i = np.arange(1, L1 + 1, dtype=np.int64)[:, None]
        j = np.arange(1, L2 + 1, dtype=np.int64)[None, :]
        r, q = j - 1, i - 1
        rr = 64 * (2 * (r // 128) + r % 2) + (r % 128) // 2 if pair else r
        t = q + rr % 64 if skew == 1 else q + (rr % 64) // 16 if skew == 2 else q
        if tiles is not None:
            x = tiles[(rr // 64) * P + ((t // 4) * 64 + rr % 64) * 4 + t % 4].astype(np.int64)
            if raw:
                SQ, SR = int(lay.SQ), int(lay.SR)
                hgt = 64 if raw == 2 else 128            # rows per stripe of the kernel that wrote them
                g = r // hgt
                big = SR * (SQ + 1)
                s = np.where(g < big, g // (SQ + 1), SR + (g - big) // max(SQ, 1))
                rw = r - hgt * (s * SQ + np.minimum(s, SR))
                base = 0 if raw == 2 else ((i - 1) // 4096) * 4096
                x = x - (rw + i - base) * int(lay.d)
            H[1:, 1:] = x
        if words is not None:
            w = words[((rr // 64) * (NQ + 1) + t // 8 + 1) * 64 + rr % 64].astype(np.int64)
            C[1:, 1:] = ((w >> (21 - 3 * (t % 8))) & 7).astype(np.uint8)
    H = ((H + 2**31) % 2**32 - 2**31).astype(np.int32)
    return H, C


@dataclass(frozen=True)
class Stats:
    corner: int
    greatest_abs_interior: int
    branch_count: int


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libnwfill.so (raises NWError if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NWError(NW_ERR_STATE, f"{path} not built (run `make -C needleman-wunsch_amd`)")
    lib = ctypes.CDLL(path)
    c_i64, c_i32, c_u32, c_p = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p
    lib.nw_strerror.restype = ctypes.c_char_p
    lib.nw_strerror.argtypes = [ctypes.c_int]
    lib.nw_last_error.restype = ctypes.c_char_p
    lib.nw_last_error.argtypes = []
    lib.nw_fill.restype = ctypes.c_int
    lib.nw_fill.argtypes = [ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64, c_i32, c_i32, c_i32, c_u32,
                            ctypes.c_int, c_p, c_p, ctypes.POINTER(_Stats)]
    lib.nw_table_create.restype = ctypes.c_int
    lib.nw_table_create.argtypes = [ctypes.c_int, c_i64, c_i64, c_u32, ctypes.POINTER(c_p)]
    lib.nw_table_destroy.restype = None
    lib.nw_table_destroy.argtypes = [c_p]
    lib.nw_table_set_sequences.restype = ctypes.c_int
    lib.nw_table_set_sequences.argtypes = [c_p, ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64]
    lib.nw_table_fill.restype = ctypes.c_int
    lib.nw_table_fill.argtypes = [c_p, c_i32, c_i32, c_i32, c_u32]
    lib.nw_table_stats.restype = ctypes.c_int
    lib.nw_table_stats.argtypes = [c_p, ctypes.POINTER(_Stats)]
    lib.nw_table_elapsed_ms.restype = ctypes.c_int
    lib.nw_table_elapsed_ms.argtypes = [c_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.nw_table_hash.restype = ctypes.c_int
    lib.nw_table_hash.argtypes = [c_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.nw_table_copy_scores.restype = ctypes.c_int
    lib.nw_table_copy_scores.argtypes = [c_p, c_i64, c_i64, c_p]
    lib.nw_table_copy_codes.restype = ctypes.c_int
    lib.nw_table_copy_codes.argtypes = [c_p, c_i64, c_i64, c_p]
    lib.nw_table_copy_last_column.restype = ctypes.c_int
    lib.nw_table_copy_last_column.argtypes = [c_p, c_p]
    lib.nw_table_score_pitch.restype = c_i64
    lib.nw_table_score_pitch.argtypes = [c_p]
    lib.nw_table_trace.restype = c_i64
    lib.nw_table_trace.argtypes = [c_p, c_p, c_i64]
    lib.nw_table_waves.restype = ctypes.c_int
    lib.nw_table_waves.argtypes = [c_p]
    c_int, P = ctypes.c_int, ctypes.POINTER
    sigs = {
        "nw_panel_partition": (c_int, [c_i64, c_int, c_int, P(c_i64), P(c_i64)]),
        "nw_panel_chain": (c_int, [c_i64, c_int, c_int, P(c_int), P(c_int), P(c_int)]),
        "nw_panel_get_id": (c_int, [c_p]),
        "nw_panel_create": (c_int, [c_int, c_int, c_int, c_int, c_p, c_i64, c_i64, c_u32, P(c_p)]),
        "nw_panel_ipc_handle": (c_int, [c_p, c_p]),
        "nw_panel_ipc_connect": (c_int, [c_p, c_p]),
        "nw_panel_group_create": (c_int, [c_int, c_p, c_i64, c_i64, c_u32, c_p]),
        "nw_panel_destroy": (None, [c_p]),
        "nw_panel_set_sequences": (c_int, [c_p, ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64]),
        "nw_panel_fill": (c_int, [c_p, c_i32, c_i32, c_i32, c_u32]),
        "nw_panel_group_fill": (c_int, [c_p, c_int, c_i32, c_i32, c_i32, c_u32]),
        "nw_panel_stats": (c_int, [c_p, P(_Stats)]),
        "nw_panel_record": (c_int, [c_p, c_p]),
        "nw_panel_reduce": (c_int, [c_p, c_int, P(_Stats)]),
        "nw_panel_rows": (c_int, [c_p, P(c_i64), P(c_i64)]),
        "nw_panel_table": (c_p, [c_p]),
        "nw_panel_elapsed_ms": (c_int, [c_p, P(ctypes.c_float), P(ctypes.c_float)]),
        "nw_panel_hash_columns": (c_int, [c_p, c_p, c_p]),
        "nw_panel_credit_reached": (c_int, [c_u32, c_u32]),
        "nw_table_hash_columns": (c_int, [c_p, c_i64, c_p, c_p]),
        "nw_hash_fold": (ctypes.c_uint64, [c_p, c_i64]),
        "nw_table_count_alignments": (c_int, [c_p, P(c_u32)]),
        "nw_table_first_path": (c_int, [c_p, c_p, c_i64, P(c_i64)]),
        "nw_table_walk_elapsed_ms": (c_int, [c_p, P(ctypes.c_float), P(ctypes.c_float)]),
        "nw_first_path_banded": (c_int, [c_int, ctypes.c_char_p, c_i64, ctypes.c_char_p, c_i64, c_i32, c_i32, c_i32,
                                         c_i64, c_p, c_i64, P(c_i64)]),
        "nw_host_alloc": (c_int, [ctypes.c_size_t, P(c_p)]),
        "nw_table_enumerate_paths": (c_int, [c_p, ctypes.c_uint64, ctypes.c_uint64, c_p, c_i64, c_p,
                                             P(ctypes.c_uint64), P(ctypes.c_uint64)]),
        "nw_host_free": (None, [c_p]),
        "nw_fill_noalloc": (c_int, [c_int, c_p, c_p, c_i64, c_p, c_i64, c_i32, c_i32, c_i32, c_u32, c_p, c_p, c_p, c_p]),
        "nw_table_layout": (c_int, [c_p, P(Layout)]),
        "nw_table_device_buffers": (c_int, [c_p, P(c_p), P(c_p)]),
        "nw_table_io_stats": (c_int, [c_p, P(ctypes.c_double), P(c_i64), P(ctypes.c_double), P(c_i64)]),
    }
    for name, (res, args) in sigs.items():
        if os.environ.get("NW_LIB") and not hasattr(lib, name):
            continue        # an older A/B build (tools/ab_libs.sh) may predate an entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != NW_OK:
        lib = load()
        detail = lib.nw_last_error().decode(errors="replace")
        raise NWError(rc, f"{what}: {lib.nw_strerror(rc).decode()}: {detail}")


class HostBuffer:
    """Pinned (page-locked) host memory from nw_host_alloc, viewed as a numpy
    array: slice copies into it are DMA'd straight from the device.

    The memory belongs to the views: `array`, every slice or reshape of it and
    every array a copy call returned for `out=hb.array` keep it alive, and it
    goes back to the runtime when the last of them is gone.  close() only
    drops this object's own view."""

    def __init__(self, shape, dtype):
        import weakref
        lib = load()
        self.array_dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * self.array_dtype.itemsize
        p = ctypes.c_void_p()
        _check(lib.nw_host_alloc(n, ctypes.byref(p)), "nw_host_alloc")
        raw = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
        # numpy keeps `raw` alive as the base of every view; the pinned
        # memory is released when `raw` itself is collected
        weakref.finalize(raw, lib.nw_host_free, ctypes.c_void_p(p.value))
        self.array = np.frombuffer(raw, dtype=np.uint8, count=n).view(self.array_dtype).reshape(shape)

    def close(self) -> None:
        self.array = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _bytes(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def fill(s1, s2, m: int, k: int, d: int, *, scores: bool = True, dirs: bool = True,
         stats: bool = True, device: int = -1):
    """One-shot fill.  Returns (H, codes, Stats).

    H     : int32 array (L1+1, L2+1), H[i, j] = reference cells[i][j].score, or None
    codes : uint8 array (L1+1, L2+1) of direction codes (bit0 diag, bit1 up,
            bit2 left), unpacked from the library's nibble output, or None
    """
    lib = load()
    b1, b2 = _bytes(s1), _bytes(s2)
    L1, L2 = len(b1), len(b2)
    ncell = (L1 + 1) * (L2 + 1)
    H = np.empty((L1 + 1, L2 + 1), dtype=np.int32) if scores else None
    nib = np.empty((ncell + 1) // 2, dtype=np.uint8) if dirs else None
    st = _Stats()
    rc = lib.nw_fill(b1, L1, b2, L2, m, k, d, NW_OUT_STATS if stats else 0, device,
                     H.ctypes.data if H is not None else None,
                     nib.ctypes.data if nib is not None else None, ctypes.byref(st))
    _check(rc, "nw_fill")
    codes = unpack_nibbles(nib, ncell).reshape(L1 + 1, L2 + 1) if dirs else None
    return H, codes, Stats(st.corner, st.greatest_abs_interior, st.branch_count)


def unpack_nibbles(nib: np.ndarray, ncell: int) -> np.ndarray:
    """Dense nibble plane (cell c -> nibble c of the byte stream, low first)."""
    out = np.empty(2 * len(nib), dtype=np.uint8)
    out[0::2] = nib & 0xF
    out[1::2] = nib >> 4
    return out[:ncell]


def _out(out, shape, dtype):
    if out is None:
        return np.empty(shape, dtype=dtype)
    if out.shape != tuple(shape) or out.dtype != np.dtype(dtype) or not out.flags.c_contiguous:
        raise ValueError(f"out must be a C-contiguous {np.dtype(dtype)} array of shape {tuple(shape)}")
    return out


class Table:
    """Device-resident score table (include/nw_fill.h nw_table_*)."""

    def __init__(self, max_L1: int, max_L2: int, out_mask: int = NW_OUT_ALL, device: int = -1):
        self._lib = load()
        self._h = ctypes.c_void_p()
        self._owned = True
        _check(self._lib.nw_table_create(device, max_L1, max_L2, out_mask, ctypes.byref(self._h)),
               "nw_table_create")
        self.L1 = self.L2 = None

    @classmethod
    def _borrow(cls, handle, L1: int, L2: int) -> "Table":
        """A view of a table owned elsewhere (a panel's local rows)."""
        t = cls.__new__(cls)
        t._lib = load()
        t._h = ctypes.c_void_p(handle)
        t._owned = False
        t.L1, t.L2 = L1, L2
        return t

    def close(self) -> None:
        if self._h and self._owned:
            self._lib.nw_table_destroy(self._h)
        self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_sequences(self, s1, s2) -> None:
        b1, b2 = _bytes(s1), _bytes(s2)
        _check(self._lib.nw_table_set_sequences(self._h, b1, len(b1), b2, len(b2)),
               "nw_table_set_sequences")
        self.L1, self.L2 = len(b1), len(b2)

    def fill(self, m: int, k: int, d: int, out_mask: int = NW_OUT_SCORES | NW_OUT_DIRS) -> None:
        _check(self._lib.nw_table_fill(self._h, m, k, d, out_mask), "nw_table_fill")

    def stats(self) -> Stats:
        st = _Stats()
        _check(self._lib.nw_table_stats(self._h, ctypes.byref(st)), "nw_table_stats")
        return Stats(st.corner, st.greatest_abs_interior, st.branch_count)

    def elapsed_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(self._lib.nw_table_elapsed_ms(self._h, ctypes.byref(a), ctypes.byref(b)),
               "nw_table_elapsed_ms")
        return a.value, b.value

    def hash(self):
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._lib.nw_table_hash(self._h, ctypes.byref(a), ctypes.byref(b)), "nw_table_hash")
        return a.value, b.value

    def hash_columns(self, j0: int, state: np.ndarray) -> None:
        """Continue per-column FNV states (2, L1+1) uint64 -- scores, codes -- over rows j0..L2."""
        _check(self._lib.nw_table_hash_columns(self._h, j0, state[0].ctypes.data, state[1].ctypes.data),
               "nw_table_hash_columns")

    def scores(self, i0: int = 0, i1: int | None = None, out: np.ndarray | None = None) -> np.ndarray:
        """Columns [i0, i1) as int32 (i1-i0, L2+1); `out` (C-contiguous, e.g. a
        HostBuffer's array) receives them in place."""
        i1 = self.L1 + 1 if i1 is None else i1
        out = _out(out, (i1 - i0, self.L2 + 1), np.int32)
        _check(self._lib.nw_table_copy_scores(self._h, i0, i1, out.ctypes.data), "nw_table_copy_scores")
        return out

    def codes(self, i0: int = 0, i1: int | None = None, out: np.ndarray | None = None) -> np.ndarray:
        i1 = self.L1 + 1 if i1 is None else i1
        out = _out(out, (i1 - i0, self.L2 + 1), np.uint8)
        _check(self._lib.nw_table_copy_codes(self._h, i0, i1, out.ctypes.data), "nw_table_copy_codes")
        return out

    def enumerate_paths(self, first: int = 0, count: int = 1) -> tuple[list[np.ndarray], int]:
        """Alignments first .. first+count-1 in the reference's print order, each
        as its moves from the corner back to (0,0) (1 diag, 2 up, 4 left), and the
        total number of alignments (nw_table_enumerate_paths)."""
        stride = max(self.L1 + self.L2, 1)
        mv = np.zeros((max(count, 1), stride), dtype=np.uint8)
        ln = np.zeros(max(count, 1), dtype=np.int32)
        n, tot = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._lib.nw_table_enumerate_paths(self._h, first, count, mv.ctypes.data, stride, ln.ctypes.data,
                                                  ctypes.byref(n), ctypes.byref(tot)), "nw_table_enumerate_paths")
        return [mv[p, :ln[p]].copy() for p in range(n.value)], tot.value

    def io_stats(self) -> dict:
        """Last upload / slice copy: wall ms and bytes (nw_table_io_stats)."""
        um, cm = ctypes.c_double(), ctypes.c_double()
        ub, cb = ctypes.c_int64(), ctypes.c_int64()
        _check(self._lib.nw_table_io_stats(self._h, ctypes.byref(um), ctypes.byref(ub), ctypes.byref(cm),
                                           ctypes.byref(cb)), "nw_table_io_stats")
        return {"upload_ms": um.value, "upload_bytes": ub.value, "copy_ms": cm.value, "copy_bytes": cb.value}

    def last_column(self) -> np.ndarray:
        out = np.empty(self.L2 + 1, dtype=np.int32)
        _check(self._lib.nw_table_copy_last_column(self._h, out.ctypes.data), "nw_table_copy_last_column")
        return out

    def trace(self, mid: bool = False) -> np.ndarray:
        """In-kernel timeline (needs $NW_TRACE): rows (dequeue, start, end, block|cu<<32,
        clk_start, clk_end, last wave start, 0) per WG-stripe -- realtime at 100 MHz,
        clk = shader clock.  mid=True: the pair kernel's per-stripe time at the
        middle chunk of the table instead."""
        n = self._lib.nw_table_trace(self._h, None, 0)
        out = np.zeros(max(n, 0), dtype=np.uint64)
        if n > 0:
            self._lib.nw_table_trace(self._h, out.ctypes.data, n)
        if n < 8:
            return out[:0].reshape(-1, 8) if not mid else out[:0]
        nsw, nmid = int(out[0]), int(out[1])
        body = out[8:]
        return body[8 * nsw:8 * nsw + nmid] if mid else body[:8 * nsw].reshape(-1, 8)

    def count_alignments(self) -> int:
        """Number of optimal alignments, mod 2**32 like the reference's counter
        (needs a fill with NW_OUT_DIRS)."""
        c = ctypes.c_uint32()
        _check(self._lib.nw_table_count_alignments(self._h, ctypes.byref(c)), "nw_table_count_alignments")
        return c.value

    def first_path(self) -> np.ndarray:
        """Moves of the first alignment the reference prints (1 diag, 2 up, 4 left),
        forward order."""
        cap = self.L1 + self.L2
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = ctypes.c_int64()
        _check(self._lib.nw_table_first_path(self._h, out.ctypes.data, cap, ctypes.byref(n)),
               "nw_table_first_path")
        return out[:n.value]

    def walk_elapsed_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(self._lib.nw_table_walk_elapsed_ms(self._h, ctypes.byref(a), ctypes.byref(b)),
               "nw_table_walk_elapsed_ms")
        return a.value, b.value

    @property
    def waves(self) -> int:
        return self._lib.nw_table_waves(self._h)

    def layout(self) -> Layout:
        """Device layout of the last fill (nw_table_layout)."""
        l = Layout()
        _check(self._lib.nw_table_layout(self._h, ctypes.byref(l)), "nw_table_layout")
        return l

    def device_buffers(self) -> tuple[int, int]:
        """Device addresses (score tiles, code words) for zero-copy consumers."""
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _check(self._lib.nw_table_device_buffers(self._h, ctypes.byref(a), ctypes.byref(b)),
               "nw_table_device_buffers")
        return a.value or 0, b.value or 0

    @property
    def score_pitch(self) -> int:
        return self._lib.nw_table_score_pitch(self._h)


# ------------------------------------------------------------------ panels
def panel_partition(L2: int, nranks: int, rank: int):
    """(row_base, rows) of `rank`'s panel (include/nw_panel.h)."""
    lib = load()
    b, n = ctypes.c_int64(), ctypes.c_int64()
    _check(lib.nw_panel_partition(L2, nranks, rank, ctypes.byref(b), ctypes.byref(n)), "nw_panel_partition")
    return b.value, n.value


def panel_chain(L2: int, nranks: int, rank: int):
    """(prev, next, pos) of `rank` in the boundary-row chain (-1 = none)."""
    lib = load()
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib.nw_panel_chain(L2, nranks, rank, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
           "nw_panel_chain")
    return a.value, b.value, c.value


_PROXY_RANGE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64)
_PROXY_FLAG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64)


class _ProxyOps(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("recv", _PROXY_RANGE), ("flag", _PROXY_FLAG),
                ("poison", _PROXY_RANGE), ("send", _PROXY_RANGE)]


def panel_proxy_run(L1: int, xblk: int, has_prev: bool, has_next: bool, launched: bool,
                    recv=None, flag=None, poison=None, send=None) -> int:
    """Drive the RCCL transport's host proxy (nw_panel_proxy_run) with Python
    callbacks: recv/poison/send(off, cnt) -> rc, flag(b, spin) -> 1/0/-1.
    Returns the proxy's status code."""
    lib = load()
    fn = lib.nw_panel_proxy_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(_ProxyOps)]

    def guard(f, *a):
        try:
            return int(f(*a))
        except Exception:          # a raising callback is a failed transport step
            return NW_ERR_STATE

    def rng(f):
        return _PROXY_RANGE(lambda _c, off, cnt: guard(f, off, cnt) if f else NW_ERR_ARG)

    ops = _ProxyOps(None, rng(recv), _PROXY_FLAG(lambda _c, b, spin: guard(flag, b, spin) if flag else -1),
                    rng(poison), rng(send))
    return fn(L1, xblk, int(has_prev), int(has_next), int(launched), ctypes.byref(ops))


def panel_get_id() -> bytes:
    """RCCL rendezvous id (rank 0 creates, every rank passes it to Panel)."""
    lib = load()
    buf = (ctypes.c_uint8 * PANEL_ID_BYTES)()
    _check(lib.nw_panel_get_id(buf), "nw_panel_get_id")
    return bytes(buf)


def panel_reduce(records) -> tuple[int, Stats]:
    """Whole-table stats from every rank's record; returns (rc, Stats)."""
    lib = load()
    recs = np.ascontiguousarray(np.asarray(records, dtype=np.int64).reshape(-1, PANEL_REC))
    st = _Stats()
    rc = lib.nw_panel_reduce(recs.ctypes.data, recs.shape[0], ctypes.byref(st))
    return rc, Stats(st.corner, st.greatest_abs_interior, st.branch_count)


class Panel:
    """One row panel of a table split across GPUs (include/nw_panel.h)."""

    def __init__(self, transport: int, rank: int, nranks: int, max_L1: int, max_L2: int,
                 out_mask: int = NW_OUT_ALL, device: int = -1, rdv_id: bytes | None = None, _handle=None):
        self._lib = load()
        self._h = ctypes.c_void_p()
        self.rank, self.nranks = rank, nranks
        self.L1 = self.L2 = None
        if _handle is not None:
            self._h = ctypes.c_void_p(_handle)
            return
        idbuf = None
        if rdv_id is not None:
            idbuf = (ctypes.c_uint8 * PANEL_ID_BYTES).from_buffer_copy(rdv_id)
        _check(self._lib.nw_panel_create(transport, device, rank, nranks, idbuf, max_L1, max_L2, out_mask,
                                         ctypes.byref(self._h)), "nw_panel_create")

    @classmethod
    def group(cls, devices, max_L1: int, max_L2: int, out_mask: int = NW_OUT_ALL) -> list["Panel"]:
        lib = load()
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        _check(lib.nw_panel_group_create(n, devs, max_L1, max_L2, out_mask, hs), "nw_panel_group_create")
        return [cls(NW_PANEL_GROUP, r, n, 0, 0, _handle=hs[r]) for r in range(n)]

    @staticmethod
    def group_fill(panels, m: int, k: int, d: int, out_mask: int = NW_OUT_SCORES | NW_OUT_DIRS) -> None:
        lib = load()
        hs = (ctypes.c_void_p * len(panels))(*[p._h.value for p in panels])
        _check(lib.nw_panel_group_fill(hs, len(panels), m, k, d, out_mask), "nw_panel_group_fill")

    def close(self) -> None:
        if self._h:
            self._lib.nw_panel_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def ipc_handle(self) -> bytes:
        buf = (ctypes.c_uint8 * PANEL_IPC_BYTES)()
        _check(self._lib.nw_panel_ipc_handle(self._h, buf), "nw_panel_ipc_handle")
        return bytes(buf)

    def ipc_connect(self, handles: bytes) -> None:
        assert len(handles) == self.nranks * PANEL_IPC_BYTES
        buf = (ctypes.c_uint8 * len(handles)).from_buffer_copy(handles)
        _check(self._lib.nw_panel_ipc_connect(self._h, buf), "nw_panel_ipc_connect")

    def set_sequences(self, s1, s2) -> None:
        b1, b2 = _bytes(s1), _bytes(s2)
        _check(self._lib.nw_panel_set_sequences(self._h, b1, len(b1), b2, len(b2)), "nw_panel_set_sequences")
        self.L1, self.L2 = len(b1), len(b2)

    def fill(self, m: int, k: int, d: int, out_mask: int = NW_OUT_SCORES | NW_OUT_DIRS) -> None:
        _check(self._lib.nw_panel_fill(self._h, m, k, d, out_mask), "nw_panel_fill")

    def fill_rc(self, m: int, k: int, d: int, out_mask: int = NW_OUT_SCORES | NW_OUT_DIRS) -> int:
        return self._lib.nw_panel_fill(self._h, m, k, d, out_mask)

    def record(self) -> np.ndarray:
        rec = np.zeros(PANEL_REC, dtype=np.int64)
        _check(self._lib.nw_panel_record(self._h, rec.ctypes.data), "nw_panel_record")
        return rec

    def stats(self) -> Stats:
        st = _Stats()
        _check(self._lib.nw_panel_stats(self._h, ctypes.byref(st)), "nw_panel_stats")
        return Stats(st.corner, st.greatest_abs_interior, st.branch_count)

    def rows(self):
        b, n = ctypes.c_int64(), ctypes.c_int64()
        _check(self._lib.nw_panel_rows(self._h, ctypes.byref(b), ctypes.byref(n)), "nw_panel_rows")
        return b.value, n.value

    @property
    def table(self) -> Table:
        """The panel's local rows (local row j = global row row_base + j)."""
        _, rows = self.rows()
        return Table._borrow(self._lib.nw_panel_table(self._h), self.L1, rows)

    def elapsed_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(self._lib.nw_panel_elapsed_ms(self._h, ctypes.byref(a), ctypes.byref(b)), "nw_panel_elapsed_ms")
        return a.value, b.value

    def hash_columns(self, state: np.ndarray) -> None:
        """Continue the whole table's per-column FNV states (see hash_states) over this panel's rows."""
        _check(self._lib.nw_panel_hash_columns(self._h, state[0].ctypes.data, state[1].ctypes.data),
               "nw_panel_hash_columns")


def hash_states(L1: int) -> np.ndarray:
    """Fresh per-column FNV-1a-64 states for a table of L1+1 columns: row 0 = scores, row 1 = codes."""
    return np.full((2, L1 + 1), 0xCBF29CE484222325, dtype=np.uint64)


def hash_fold(state: np.ndarray) -> tuple[int, int]:
    """(hH, hD) of nw_table_hash from chained per-column states (Panel.hash_columns)."""
    lib = load()
    st = np.ascontiguousarray(state, dtype=np.uint64)
    return int(lib.nw_hash_fold(st[0].ctypes.data, st.shape[1])), int(lib.nw_hash_fold(st[1].ctypes.data, st.shape[1]))


def render_path(s1, s2, moves) -> tuple[bytes, bytes]:
    """Aligned (top, side) strings of a move sequence from Table.first_path()
    (what the reference prints for that alignment, needleman-wunsch.c:296-322
    with print_aligned_strings_and_counts, before colouring)."""
    b1, b2 = _bytes(s1), _bytes(s2)
    mv = np.asarray(moves, dtype=np.uint8)
    top = np.full(len(mv), ord("-"), dtype=np.uint8)
    side = np.full(len(mv), ord("-"), dtype=np.uint8)
    a1 = (mv & 5) != 0            # diag or left consume s1
    a2 = (mv & 3) != 0            # diag or up consume s2
    if a1.sum() != len(b1) or a2.sum() != len(b2):
        raise ValueError("moves do not span the two sequences")
    top[a1] = np.frombuffer(b1, dtype=np.uint8)
    side[a2] = np.frombuffer(b2, dtype=np.uint8)
    return top.tobytes(), side.tobytes()


def walk(s1, s2, m: int, k: int, d: int, device: int = -1):
    """Fill (direction codes only) and walk on the device: returns
    (optimal score, number of optimal alignments mod 2**32, (top, side) of the
    first alignment the reference prints)."""
    b1, b2 = _bytes(s1), _bytes(s2)
    with Table(len(b1), len(b2), NW_OUT_DIRS, device) as t:
        t.set_sequences(b1, b2)
        t.fill(m, k, d, NW_OUT_DIRS)
        return t.stats().corner, t.count_alignments(), render_path(b1, b2, t.first_path())


# ----------------------------------------------------------------- inputs
def first_path_banded(s1, s2, m: int, k: int, d: int, band_rows: int = 65536, device: int = -1) -> np.ndarray:
    """Moves of the reference's first printed alignment (1 diag, 2 up, 4 left,
    forward order) without the full table: nw_first_path_banded (checkpointed
    bands of `band_rows` rows, a multiple of 64)."""
    lib = load()
    b1, b2 = _bytes(s1), _bytes(s2)
    cap = len(b1) + len(b2)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    n = ctypes.c_int64()
    _check(lib.nw_first_path_banded(device, b1, len(b1), b2, len(b2), m, k, d, band_rows, out.ctypes.data, cap,
                                    ctypes.byref(n)), "nw_first_path_banded")
    return out[:n.value]


def gen_dna(seed: int, n: int) -> bytes:
    """splitmix64 i.i.d. DNA: base = "ACGT"[z >> 62]."""
    if n == 0:
        return b""
    with np.errstate(over="ignore"):
        st = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = st
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return np.frombuffer(b"ACGT", dtype=np.uint8)[(z >> np.uint64(62)).astype(np.intp)].tobytes()


def fnv1a64(data, h: int = 0xCBF29CE484222325) -> int:
    """FNV-1a-64 (host side, for small buffers and the column-chain fold)."""
    mv = memoryview(bytes(data))
    for b in mv:
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h
