"""Debug probe: run each output-mask variant of the fill on a small table, each
in its own process so a fault in one does not hide the others."""
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
code = r'''
import sys, os
sys.path[:0] = [os.path.join(%r, "needleman-wunsch_amd"), os.path.join(%r, "tests")]
import numpy as np, nw_amd, oracle_lib as O
mask, L1, L2, W = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
if W != "0": os.environ["NW_WAVES"] = W
s1, s2 = O.gen_dna(21, L1), O.gen_dna(22, L2)
Ho, Do, sto = O.fill(s1, s2, 2, 3, 5)
with nw_amd.Table(L1, L2, nw_amd.NW_OUT_ALL) as t:
    t.set_sequences(s1, s2)
    t.fill(2, 3, 5, mask)
    st = t.stats()
    ok = st.corner == sto[0]
    if mask & 4: ok = ok and (st.greatest_abs_interior, st.branch_count) == sto[1:]
    lc = np.array_equal(t.last_column(), Ho[-1])
    print("mask", mask, "L1", L1, "L2", L2, "W", W, "stats_ok", ok, "lastcol_ok", lc, flush=True)
''' % (ROOT, ROOT)
for args in [("7", "3001", "2003", "0"), ("4", "3001", "2003", "0"), ("0", "3001", "2003", "0"),
             ("2", "3001", "2003", "0"), ("1", "3001", "2003", "0"), ("4", "3000", "2003", "0"),
             ("4", "3001", "64", "1"), ("0", "17", "70", "1"), ("4", "8", "64", "1")]:
    r = subprocess.run([sys.executable, "-c", code, *args], capture_output=True, text=True, timeout=120)
    print(args, "rc", r.returncode, r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
