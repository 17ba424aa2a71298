"""Debug: pair kernel vs oracle at small shapes with a forced wave count."""
import os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "needleman-wunsch_amd"), os.path.join(ROOT, "tests")]
import nw_amd
import oracle_lib as O
os.environ["NW_KERNEL"] = "pair"
for W, L1, L2, mkd in [(2, 100, 256, (2, 3, 5)), (2, 1234, 256, (2, 3, 5)), (2, 1234, 657, (2, 3, 5)),
                       (3, 200, 384, (1, 1, 1)), (1, 200, 384, (1, 1, 1))]:
    os.environ["NW_WAVES"] = str(W)
    s1, s2 = O.gen_dna(5, L1), O.gen_dna(6, L2)
    H, D, st = nw_amd.fill(s1, s2, *mkd)
    Ho, Do, sto = O.fill(s1, s2, *mkd)
    bad = np.argwhere(H != Ho)
    print(W, L1, L2, "bad cells", len(bad), "first", bad[:3].tolist(), "codes bad", int((D != Do).sum()))
    if len(bad):
        i, j = bad[0]
        print("  col", i, "rows", j, "..: got", H[i, j:j + 4].tolist(), "want", Ho[i, j:j + 4].tolist())
        cols = sorted(set(bad[:, 0].tolist()))
        rows = sorted(set(bad[:, 1].tolist()))
        print("  bad cols", cols[:10], "... n", len(cols), " bad rows", rows[:10], "... n", len(rows))
