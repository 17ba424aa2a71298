"""The C ABI (include/nw_fill.h, include/nw_panel.h) -- CPU checks: the library loads, exports
every declared entry point, reports errors without exit()ing, and the
Python binding mirrors it.  No GPU compute here."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "needleman-wunsch_amd")
LIB = os.path.join(PKG, "lib", "libnwfill.so")
HEADERS = [os.path.join(ROOT, "include", h) for h in ("nw_fill.h", "nw_panel.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(nw_[a-z_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", PKG, "lib"])
    return ctypes.CDLL(LIB)


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert len(names) >= 33
    for n in names:
        assert hasattr(lib, n), n


def test_python_binding_lists_every_export():
    import nw_amd
    assert sorted(nw_amd.EXPORTS) == declared_functions()


def test_strerror_covers_codes(lib):
    lib.nw_strerror.restype = ctypes.c_char_p
    for rc in range(0, -9, -1):
        assert lib.nw_strerror(rc) and lib.nw_strerror(rc) != b"unknown error"
    assert lib.nw_strerror(-99) == b"unknown error"


def test_bad_arguments_return_error_codes(lib):
    # argument validation happens before any device call
    lib.nw_table_create.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32,
                                    ctypes.POINTER(ctypes.c_void_p)]
    assert lib.nw_table_create(0, -1, 5, 1, None) == -1
    lib.nw_table_fill.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32]
    assert lib.nw_table_fill(None, 1, 1, 1, 1) == -1
    P = ctypes.POINTER
    lib.nw_panel_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, P(ctypes.c_void_p)]
    h = ctypes.c_void_p()
    assert lib.nw_panel_create(7, 0, 0, 2, None, 10, 10, 1, ctypes.byref(h)) == -1     # unknown transport
    assert lib.nw_panel_create(2, 0, 0, 2, None, 10, 10, 1, ctypes.byref(h)) == -1     # RCCL needs an id
    assert lib.nw_panel_create(1, 0, 2, 2, None, 10, 10, 1, ctypes.byref(h)) == -1     # rank >= nranks
    lib.nw_panel_fill.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32]
    assert lib.nw_panel_fill(None, 1, 1, 1, 1) == -1
    lib.nw_panel_group_create.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_uint32, ctypes.c_void_p]
    assert lib.nw_panel_group_create(0, None, 10, 10, 1, None) == -1
    lib.nw_panel_table.restype = ctypes.c_void_p
    assert lib.nw_panel_table(None) is None


def test_device_code_is_gfx950_only():
    """The embedded offload bundle carries exactly one device target: gfx950."""
    data = open(LIB, "rb").read()
    starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", data)]
    assert starts
    for i in starts:   # one bundle per HIP source
        targets = re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data[i:i + 4096])
        assert targets == [b"gfx950"]
