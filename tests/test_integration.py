"""The reference-side drop-in, built for real (CPU side).

oracle/Makefile links the reference program from its own objects (compiled
from /root/reference, never copied) with integration/nw_gpu_shim.c and
-lnwfill: the reference's compute_table_scores is weakened in its object, so
the call at needleman-wunsch.c:662 lands in the shim, which fills through
include/nw_fill.h.  Here (no GPU) that binary must link, bind the call to the
shim, and fail loudly the reference's way when no device is present -- the
fill has no CPU fallback.  tests/test_gpu_integration.py runs the CLI goldens
through it on the MI355X.
"""
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "oracle", "_ref", "needleman-wunsch-gpu")
SHIM = os.path.join(ROOT, "integration", "nw_gpu_shim.c")

pytestmark = pytest.mark.skipif(not os.path.exists(BIN),
                                reason="oracle/_ref/needleman-wunsch-gpu not built (needs /root/reference)")


def test_shim_takes_the_call_at_662():
    nm = subprocess.run(["nm", BIN], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1]: ln.split()[-2] for ln in nm.splitlines() if len(ln.split()) >= 2}
    assert syms.get("compute_table_scores") == "T"
    assert syms.get("compute_table_scores_gpu") == "T"
    dis = subprocess.run(["objdump", "-d", BIN], capture_output=True, text=True, check=True).stdout
    # the strong compute_table_scores is the shim's: a jump/call into compute_table_scores_gpu
    body = dis.split("<compute_table_scores>:", 1)[1].split("\n\n", 1)[0]
    assert "compute_table_scores_gpu" in body
    ldd = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "libnwfill.so" in ldd and "not found" not in ldd


def test_without_gpu_it_fails_like_the_reference(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; tests/test_gpu_integration.py covers the success path")
    p = subprocess.run(["needleman-wunsch", "-s", "1", "1", "1"], executable=BIN, input=b"GAT GTA\n",
                       capture_output=True, timeout=60)
    assert p.returncode == 1
    err = p.stderr.decode()
    assert err.startswith("needleman-wunsch: error: GPU fill failed: "), err   # dbg.h:67-77 format
    assert p.stdout == b""


def test_shim_documented_in_integration_md():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    assert "integration/nw_gpu_shim.c" in doc and "needleman-wunsch-gpu" in doc
    with open(SHIM) as f:
        assert "compute_table_scores_gpu" in f.read()
