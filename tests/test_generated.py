"""The hand-scheduled blocks under csrc/ are generated files: each must be
exactly what its generator in tools/ writes today, or the library was built
from a schedule nobody can regenerate.  The generators also check their own
schedules (two wait states before every DPP read), so running them is a test
of the schedule rules too."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CSRC = os.path.join(ROOT, "needleman-wunsch_amd", "csrc")


@pytest.mark.parametrize("gen,inc", [("gen_pair_asm.py", "nw_pair_chunk.inc"), ("gen_quad_asm.py", "nw_quad_chunk.inc"),
                                     ("gen_chunk_asm.py", "nw_chunk.inc"), ("gen_skew_asm.py", "nw_skew_chunk.inc")])
def test_generated_block_is_current(tmp_path, gen, inc):
    out = tmp_path / inc
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", gen), "--out", str(out)], check=True,
                   capture_output=True, timeout=120)
    with open(os.path.join(CSRC, inc)) as f:
        assert out.read_text() == f.read(), f"{inc} is stale: run tools/{gen}"
