"""Host side of the CLI on CPU (no GPU): argument/reader error paths of the
real binary, and the traceback/summary/table renderer (libnwhost.so) fed with
oracle tables, both byte-compared with the reference's own output
(tests/golden/cli_cases.json, produced by oracle/_ref/needleman-wunsch)."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as O
from conftest import ROOT, load_golden

PKG = os.path.join(ROOT, "needleman-wunsch_amd")
CLI = os.path.join(PKG, "bin", "needleman-wunsch")
HOSTLIB = os.path.join(PKG, "lib", "libnwhost.so")
CASES = load_golden("cli_cases.json")


def _built():
    if not (os.path.exists(CLI) and os.path.exists(HOSTLIB)):
        subprocess.check_call(["make", "-s", "-C", PKG, "cli", "hostlib"])


def run_cli(case, binary=None):
    """Run the CLI as `needleman-wunsch` (argv[0] matters, dbg.c:7-15)."""
    if binary is None:
        _built()
    args, stdin, tmp = list(case["args"]), case["stdin"], None
    if "{FILE}" in args:
        tmp = tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False)
        tmp.write(stdin)
        tmp.close()
        args = [tmp.name if a == "{FILE}" else a for a in args]
        stdin = ""
    try:
        p = subprocess.run(["needleman-wunsch"] + args, executable=binary or CLI, input=stdin.encode(),
                           capture_output=True, timeout=300)
    finally:
        if tmp:
            os.unlink(tmp.name)
    return p.returncode, p.stdout.decode("utf-8", "replace"), p.stderr.decode("utf-8", "replace")


class Flags(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("cflag", "lflag", "qflag", "sflag", "tflag", "uflag")]


def parse_args(args):
    """getopt "cf:hlp:qstu" for the success cases of the golden set."""
    f, ops, i = Flags(), [], 0
    while i < len(args):
        a = args[i]
        if a == "--":
            ops += args[i + 1:]
            break
        if a.startswith("-") and len(a) > 1 and not ops:
            for ch in a[1:]:
                if ch in "cqlstu":
                    setattr(f, ch + "flag", 1)
                elif ch in "fp":
                    i += 1
                    break
            i += 1
            continue
        ops.append(a)
        i += 1
    return f, [int(x) for x in ops]


def read_two(text):
    """read-sequences.c:43-122 semantics for the success cases."""
    b = text.encode()
    ws = b" \t\n\v\f\r"
    i = 0
    while i < len(b) and b[i] not in ws:
        i += 1
    s1 = b[:i]
    i += 1
    while i < len(b) and b[i] in ws:
        i += 1
    j = i
    while j < len(b) and b[j] not in ws:
        j += 1
    # the reference handles the tokens as C strings (strlen, computation.c:158-160)
    return s1.split(b"\0")[0], b[i:j].split(b"\0")[0]


def render(case):
    lib = ctypes.CDLL(HOSTLIB)
    f, (m, k, d) = parse_args(case["args"])
    s1, s2 = read_two(case["stdin"])
    H, D, (corner, gav, bc) = O.fill(s1, s2, m, k, d)
    out, err = ctypes.c_char_p(), ctypes.c_char_p()
    on, en = ctypes.c_size_t(), ctypes.c_size_t()
    lib.nwh_render_to_buffers.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Flags),
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t)]
    H = np.ascontiguousarray(H)
    D = np.ascontiguousarray(D)
    rc = lib.nwh_render_to_buffers(s1, s2, ctypes.byref(f), H.ctypes.data, D.ctypes.data, corner, gav,
                                   ctypes.byref(out), ctypes.byref(on), ctypes.byref(err), ctypes.byref(en))
    assert rc == 0
    o = ctypes.string_at(out, on.value).decode("utf-8")
    e = ctypes.string_at(err, en.value).decode("utf-8")
    return o, e


@pytest.mark.parametrize("case", [c for c in CASES if c["rc"] != 0], ids=lambda c: c["name"])
def test_cli_error_paths_match_reference(case):
    assert run_cli(case) == (case["rc"], case["stdout"], case["stderr"])


@pytest.mark.parametrize("case", [c for c in CASES if c["rc"] == 0], ids=lambda c: c["name"])
def test_renderer_matches_reference(case):
    _built()
    o, e = render(case)
    assert o == case["stdout"]
    assert e == case["stderr"]


def test_golden_set_covers_readme_examples():
    names = {c["name"] for c in CASES}
    for n in ("readme_table_q_s_t", "gat_gta", "gat_gta_s", "gat_gta_l", "gt_gt", "gt_ga"):
        assert n in names
    readme = next(c for c in CASES if c["name"] == "readme_table_q_s_t")
    assert readme["stderr"] == "3 optimal alignments\nOptimal score is 0\n"


# --------------------------------------- renderer fed with unranked paths
# The CLI prints alignments that the device enumerates one by one
# (nw_table_enumerate_paths, nwh_render_paths).  Here the same unranking runs
# in Python over the oracle's codes and feeds the same renderer, which must
# reproduce the reference's bytes -- order, -l counts, -s, -t marks included.
NEXT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                        ctypes.POINTER(ctypes.c_int64))


def path_counts(D):
    """C(i, j): code paths from (i, j) to (0, 0)."""
    L1, L2 = D.shape[0] - 1, D.shape[1] - 1
    C = [[0] * (L2 + 1) for _ in range(L1 + 1)]
    for i in range(L1 + 1):
        for j in range(L2 + 1):
            if i == 0 or j == 0:
                C[i][j] = 1
                continue
            c = int(D[i, j])
            C[i][j] = ((C[i - 1][j - 1] if c & 1 else 0) + (C[i - 1][j] if c & 4 else 0) +
                       (C[i][j - 1] if c & 2 else 0))
    return C


def unrank(D, C, k):
    """Alignment k of the reference's order: moves from the corner back to (0, 0)."""
    i, j, out = D.shape[0] - 1, D.shape[1] - 1, []
    while i > 0 or j > 0:
        c = 2 if i == 0 else 4 if j == 0 else int(D[i, j])
        mv = 2
        if c & 1:
            if k < C[i - 1][j - 1]:
                mv = 1
            else:
                k -= C[i - 1][j - 1]
        if mv != 1 and c & 4:
            if k < C[i - 1][j]:
                mv = 4
            else:
                k -= C[i - 1][j]
        out.append(mv)
        j -= mv != 4
        i -= mv != 2
    return out


def render_paths(case):
    lib = ctypes.CDLL(HOSTLIB)
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    f, (m, k, d) = parse_args(case["args"])
    s1, s2 = read_two(case["stdin"])
    H, D, (corner, gav, bc) = O.fill(s1, s2, m, k, d)
    C = path_counts(D)
    total = C[len(s1)][len(s2)] if (s1 or s2) else 0
    state = {"k": 0, "buf": None}

    def nxt(_ctx, mv, n):
        if state["k"] >= total:
            return 0
        p = unrank(D, C, state["k"])
        state["k"] += 1
        state["buf"] = (ctypes.c_uint8 * max(len(p), 1))(*p)
        mv[0] = ctypes.cast(state["buf"], ctypes.c_void_p)
        n[0] = len(p)
        return 1
    cb = NEXT(nxt)
    lib.nwh_render_paths.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Flags), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint, NEXT,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    H = np.ascontiguousarray(H)
    D8 = np.ascontiguousarray(D)
    with tempfile.TemporaryDirectory() as tmp:
        po, pe = os.path.join(tmp, "o"), os.path.join(tmp, "e")
        fo, fe = libc.fopen(po.encode(), b"w"), libc.fopen(pe.encode(), b"w")
        rc = lib.nwh_render_paths(s1, s2, ctypes.byref(f), H.ctypes.data, D8.ctypes.data, corner, gav,
                                  total % 2**32, cb, None, fo, fe)
        libc.fclose(fo)
        libc.fclose(fe)
        assert rc == 0
        return open(po, encoding="utf-8").read(), open(pe, encoding="utf-8").read()


@pytest.mark.parametrize("case", [c for c in CASES if c["rc"] == 0], ids=lambda c: c["name"])
def test_unranked_paths_render_like_the_reference(case):
    _built()
    o, e = render_paths(case)
    assert o == case["stdout"]
    assert e == case["stderr"]
