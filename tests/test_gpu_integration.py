"""The drop-in on the MI355X: the reference program itself
(oracle/_ref/needleman-wunsch-gpu -- its own objects, compiled from its
sources in the build container) with the call at needleman-wunsch.c:662
served by integration/nw_gpu_shim.c -> nw_fill() -> libnwfill.so.  Every CLI
golden of the reference (tests/golden/cli_cases.json) must come out byte for
byte: this exercises the C ABI against the real computation_t
(computation.h:44-75), score_table_t and walk_table_t, not our own CLI.
"""
import os

import pytest

from conftest import ROOT, load_golden
from test_cli_host import run_cli

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "oracle", "_ref", "needleman-wunsch-gpu")
CASES = load_golden("cli_cases.json")


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/needleman-wunsch-gpu not built")
@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_reference_program_with_gpu_fill_matches_goldens(case):
    assert run_cli(case, binary=BIN) == (case["rc"], case["stdout"], case["stderr"])
