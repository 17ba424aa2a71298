"""Record and summarize the in-kernel timeline of one fill ($NW_TRACE)."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "needleman-wunsch_amd"))
os.environ["NW_TRACE"] = "1"
import nw_amd
L1, L2 = int(sys.argv[1]), int(sys.argv[2])
mask = {"sd": 3, "": 0, "s": 1, "d": 2}[sys.argv[3] if len(sys.argv) > 3 else "sd"]
t = nw_amd.Table(L1, L2, mask | 4)
t.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
t.fill(1, 1, 1, mask); t.fill(1, 1, 1, mask)
tr = t.trace().astype(np.int64)
k = t.elapsed_ms()[0]
t0 = tr[:, 0].min()
deq, st, en = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0   # us
dur = en - st
n = len(tr)
print(f"L1={L1} L2={L2} mask={mask} waves={t.waves} stripes={n} kernel_ms={k:.3f}")
idx = sorted(set(min(n - 1, i) for i in [0, 1, 2, n // 4, n // 2, 3 * n // 4, n - 1]))
print(f"start of stripe i (us): " + " ".join(f"{st[i]:.1f}" for i in idx))
print(f"end   of stripe i (us): " + " ".join(f"{en[i]:.1f}" for i in idx))
clk = (tr[:, 5] - tr[:, 4]).astype(np.float64)
mhz = clk / np.maximum(dur, 1e-9)
print(f"shader clock over stripe i (MHz): " + " ".join(f"{mhz[i]:.0f}" for i in idx))
lag = np.diff(st) if n > 1 else np.zeros(1)
print(f"start lag per stripe: mean {lag.mean():.2f} us  median {np.median(lag):.2f}  p90 {np.percentile(lag, 90):.2f}  max {lag.max():.2f}")
print(f"stripe duration: first {dur[0]:.1f} us  median {np.median(dur):.1f}  last {dur[-1]:.1f}  max {dur.max():.1f}")
lastw = (tr[:, 6] - t0) / 100.0
nwv = max(t.waves - 1, 1)
intra = (lastw - st) / nwv
print(f"intra-WG lag per stripe (first -> last wave start)/(W-1): median {np.median(intra):.3f} us  p90 {np.percentile(intra, 90):.3f}")
if n > 1:
    hand = st[1:] - lastw[:-1]
    print(f"WG-stripe hand-off (last wave start -> next WG first wave start): median {np.median(hand):.3f} us  p90 {np.percentile(hand, 90):.3f}  max {hand.max():.3f}")
cu = (tr[:, 3] >> 32) & 0xffffffff
print(f"distinct CU ids used: {len(set(cu.tolist()))}")
