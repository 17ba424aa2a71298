"""End-to-end CLI on the GPU: every golden case of the reference CLI
(tests/golden/cli_cases.json) must be reproduced byte for byte (stdout,
stderr, exit status) by needleman-wunsch_amd/bin/needleman-wunsch, whose fill
runs through libnwfill.so on the MI355X."""
import pytest

from conftest import load_golden
from test_cli_host import run_cli

pytestmark = pytest.mark.gpu
CASES = load_golden("cli_cases.json")


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_cli_matches_reference(case):
    assert run_cli(case) == (case["rc"], case["stdout"], case["stderr"])


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_cli_host_walk_fallback_matches_reference(case, monkeypatch):
    """When the device's path-count table (8 bytes per cell) does not fit, the
    CLI walks the codes on the host (needleman-wunsch.c:209-331) instead of
    failing; $NW_ENUM_MAX_BYTES = 0 forces that path for every golden."""
    monkeypatch.setenv("NW_ENUM_MAX_BYTES", "0")
    assert run_cli(case) == (case["rc"], case["stdout"], case["stderr"])


def test_enumerate_paths_reports_missing_memory(monkeypatch):
    import nw_amd
    monkeypatch.setenv("NW_ENUM_MAX_BYTES", "1000")
    with nw_amd.Table(300, 200) as t:
        t.set_sequences(b"ACGT" * 75, b"TGCA" * 50)
        t.fill(1, 1, 1, nw_amd.NW_OUT_ALL)
        with pytest.raises(nw_amd.NWError) as e:
            t.enumerate_paths(0, 1)
        assert e.value.rc == nw_amd.NW_ERR_OOM and "8 per cell" in str(e.value)
        monkeypatch.delenv("NW_ENUM_MAX_BYTES")
        paths, total = t.enumerate_paths(0, 1)
        assert len(paths) == 1 and total >= 1


def test_cli_large_summary_and_quiet():
    """CLI on longer inputs.  -q alone skips the traceback (needleman-wunsch.c:667);
    -s runs it, so use a near-identical pair whose optimum is a single alignment
    (random pairs have exponentially many co-optimal alignments -- the
    reference's enumeration would not finish either, README:195-200)."""
    import oracle_lib as O
    s1 = bytearray(O.gen_dna(41, 3000))
    s2 = bytearray(s1)
    for p in (17, 1234, 2999):
        s2[p] = ord("A") if s2[p] != ord("A") else ord("C")
    s1, s2 = bytes(s1), bytes(s2)
    H, D, st = O.fill(s1, s2, 1, 1, 1)
    rc, out, err = run_cli({"args": ["-q", "1", "1", "1"], "stdin": (s1 + b" " + s2 + b"\n").decode()})
    assert (rc, out, err) == (0, "", "")
    rc, out, err = run_cli({"args": ["-q", "-s", "1", "1", "1"], "stdin": (s1 + b" " + s2 + b"\n").decode()})
    assert rc == 0 and out == ""
    assert err == f"1 optimal alignment\nOptimal score is {st[0]}\n"


@pytest.mark.parametrize("L1,L2,mkd", [(2000, 1500, (1, 1, 1)), (300, 250, (3, 5, 7)), (12000, 9000, (2, 3, 5))])
def test_cli_quiet_summary_counts_random_pairs(L1, L2, mkd):
    """`-q -s` on random pairs with exponentially many alignments: the count
    (mod 2^32, the reference's unsigned counter) comes from the device walk
    service; checked against the oracle's path-count DP, which
    tests/golden/walk_kats.json pins to the reference's own enumeration."""
    import oracle_lib as O
    s1, s2 = O.gen_dna(5, L1), O.gen_dna(6, L2)
    H, D, st = O.fill(s1, s2, *mkd)
    n = O.count_paths(D)
    n_signed = n - (1 << 32) if n >= 1 << 31 else n
    rc, out, err = run_cli({"args": ["-q", "-s", "--"] + [str(x) for x in mkd],
                            "stdin": (s1 + b" " + s2 + b"\n").decode()})
    assert (rc, out) == (0, "")
    assert err == f"{n_signed} optimal alignment{'s' if n > 1 else ''}\nOptimal score is {st[0]}\n"
