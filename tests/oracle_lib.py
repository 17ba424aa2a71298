"""ctypes binding of oracle/libnworacle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the clean-room CPU restatement of the reference fill
(oracle/nw_oracle.c); tests use it strictly as the checker.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ORACLE_SO = os.path.join(ROOT, "oracle", "libnworacle.so")
FNV_INIT = 0xCBF29CE484222325


class Stats(ctypes.Structure):
    _fields_ = [("corner", ctypes.c_int32), ("gav", ctypes.c_int32), ("bc", ctypes.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
        L = ctypes.CDLL(ORACLE_SO)
        i64, i32, p = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.nwo_fnv1a.restype = ctypes.c_uint64
        L.nwo_fnv1a.argtypes = [ctypes.c_uint64, p, i64]
        L.nwo_fill.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i32, i32, i32, p, p,
                               ctypes.POINTER(Stats)]
        L.nwo_fill_hash.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i32, i32, i32,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(Stats)]
        L.nwo_fill_colchain.argtypes = L.nwo_fill_hash.argtypes
        L.nwo_score_only.restype = ctypes.c_int32
        L.nwo_score_only.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i32, i32, i32,
                                     ctypes.POINTER(ctypes.c_uint64)]
        L.nwo_score_only_mt.restype = ctypes.c_int32
        L.nwo_score_only_mt.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i32, i32, i32, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_uint64)]
        L.nwo_fill_mt.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i32, i32, i32, p, p,
                                  ctypes.POINTER(Stats), ctypes.c_int]
        L.nwo_gen_dna.argtypes = [ctypes.c_uint64, i64, ctypes.c_char_p]
        L.nwo_fill_band.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64, i64, p, i32, i32, i32, p, p,
                                    ctypes.POINTER(Stats)]
        L.nwo_count_paths.restype = ctypes.c_uint32
        L.nwo_count_paths.argtypes = [p, i64, i64]
        L.nwo_first_path.restype = i64
        L.nwo_first_path.argtypes = [p, i64, i64, p]
        _lib = L
    return _lib


def gen_dna(seed, n):
    b = ctypes.create_string_buffer(n + 1)
    lib().nwo_gen_dna(seed, n, b)
    return b.raw[:n]


def fnv(arr, h=FNV_INIT):
    a = np.ascontiguousarray(arr)
    return lib().nwo_fnv1a(h, a.ctypes.data, a.nbytes)


def fill(s1, s2, m, k, d, codes=True):
    """Full tables: (H int32 (L1+1, L2+1), codes uint8 or None, (corner, gav, bc))."""
    L1, L2 = len(s1), len(s2)
    H = np.empty((L1 + 1, L2 + 1), dtype=np.int32)
    D = np.empty((L1 + 1, L2 + 1), dtype=np.uint8) if codes else None
    st = Stats()
    lib().nwo_fill(s1, L1, s2, L2, m, k, d, H.ctypes.data, D.ctypes.data if codes else None,
                   ctypes.byref(st))
    return H, D, (st.corner, st.gav, st.bc)


def fill_band(s1, s2_band, row_base, top, m, k, d):
    """Row band given the row above it (top: L1+1 int32 of global row row_base).
    Returns (H (L1+1, rows+1) with row 0 = top, codes (row 0 = 0), (corner, gav, bc))."""
    L1, rows = len(s1), len(s2_band)
    top = np.ascontiguousarray(top, dtype=np.int32)
    assert top.shape == (L1 + 1,)
    H = np.empty((L1 + 1, rows + 1), dtype=np.int32)
    D = np.empty((L1 + 1, rows + 1), dtype=np.uint8)
    st = Stats()
    lib().nwo_fill_band(s1, L1, s2_band, rows, row_base, top.ctypes.data, m, k, d, H.ctypes.data, D.ctypes.data,
                        ctypes.byref(st))
    return H, D, (st.corner, st.gav, st.bc)


def colchain(s1, s2, m, k, d):
    a, b, st = ctypes.c_uint64(), ctypes.c_uint64(), Stats()
    lib().nwo_fill_colchain(s1, len(s1), s2, len(s2), m, k, d, ctypes.byref(a), ctypes.byref(b),
                            ctypes.byref(st))
    return a.value, b.value, (st.corner, st.gav, st.bc)


def score_only(s1, s2, m, k, d):
    h = ctypes.c_uint64()
    c = lib().nwo_score_only(s1, len(s1), s2, len(s2), m, k, d, ctypes.byref(h))
    return c, h.value


def score_only_mt(s1, s2, m, k, d, threads):
    """score_only on `threads` row bands: (corner, FNV of the last column)."""
    h = ctypes.c_uint64()
    c = lib().nwo_score_only_mt(s1, len(s1), s2, len(s2), m, k, d, threads, ctypes.byref(h))
    return c, h.value


def fnv_bytes(buf) -> int:
    """FNV-1a-64 of a bytes-like buffer (the oracle's nwo_fnv1a)."""
    b = bytes(buf)
    return lib().nwo_fnv1a(0xCBF29CE484222325, b, len(b))


def kat_inputs(case):
    if case["kind"] == "str":
        return case["s1"].encode(), case["s2"].encode()
    return gen_dna(1, case["L1"]), gen_dna(2, case["L2"])


def count_paths(D):
    """The reference's optimal-alignment count from a code table (L1+1, L2+1)."""
    D = np.ascontiguousarray(D, dtype=np.uint8)
    return lib().nwo_count_paths(D.ctypes.data, D.shape[0] - 1, D.shape[1] - 1)


def first_path(D):
    """Moves (1 diag, 2 up, 4 left) of the first alignment the reference prints."""
    D = np.ascontiguousarray(D, dtype=np.uint8)
    L1, L2 = D.shape[0] - 1, D.shape[1] - 1
    mv = np.zeros(L1 + L2 + 1, dtype=np.uint8)
    n = lib().nwo_first_path(D.ctypes.data, L1, L2, mv.ctypes.data)
    assert n >= 0
    return mv[:n]


def render_path(s1, s2, moves):
    """Aligned (top, side) byte strings of a move sequence."""
    X, Y = bytearray(), bytearray()
    i = j = 0
    for mv in moves.tolist():
        if mv == 1:
            X.append(s1[i]); Y.append(s2[j]); i += 1; j += 1
        elif mv == 4:
            X.append(s1[i]); Y.append(ord("-")); i += 1
        else:
            X.append(ord("-")); Y.append(s2[j]); j += 1
    assert i == len(s1) and j == len(s2)
    return bytes(X), bytes(Y)
