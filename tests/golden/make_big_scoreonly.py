"""Pin the 1M x 1M score-only fill (BASELINE.json configs[4]) with the CPU restatement.

    python tests/golden/make_big_scoreonly.py [threads]

Writes tests/golden/big_scoreonly.json: the corner H[L1][L2] and the FNV-1a-64
of the last column H[L1][0..L2] (int32 LE), from oracle/nw_oracle.c's
nwo_score_only_mt (row bands on `threads` cores; equal to the serial
nwo_score_only at every size tested, tests/test_oracle_golden.py).  Inputs:
splitmix64 DNA seeds 1 and 2, m = k = d = 1.  The oracle is
test infrastructure; this script only produces the fixture.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import oracle_lib as O  # noqa: E402


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    L1 = L2 = 1_000_000
    m = k = d = 1
    s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
    t0 = time.time()
    corner, hlast = O.score_only_mt(s1, s2, m, k, d, threads)
    dt = time.time() - t0
    out = [{"L1": L1, "L2": L2, "m": m, "k": k, "d": d, "corner": corner, "lastcol_fnv": "%016x" % hlast,
            "source": f"oracle nwo_score_only_mt, {threads} threads, {dt:.0f} s"}]
    with open(os.path.join(HERE, "big_scoreonly.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
