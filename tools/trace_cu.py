#!/usr/bin/env python3
"""Where the pair kernel's WG-stripes ran: CU sharing and per-WG-stripe pace.

    python tools/trace_cu.py [L1 L2]

Fills with $NW_TRACE (the default library; no NW_TRACE_EXT build needed) and
reads the per-WG-stripe timeline: the CU id (__smid) each WG-stripe ran on,
how many WG-stripes shared a CU, and the start / end of the WG-stripes that
did against those that did not.  Two workgroups on one CU put two compute
waves on a SIMD, which runs each at roughly the two-wave rate, and the whole
stripe chain behind them at that pace.
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "needleman-wunsch_amd"))
os.environ["NW_TRACE"] = "1"
import nw_amd  # noqa: E402

L1 = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
L2 = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
with nw_amd.Table(L1, L2, 3) as t:
    t.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
    for _ in range(3):
        t.fill(1, 1, 1, 3)
    wg = t.trace().astype(np.int64)
    k = t.elapsed_ms()[0]
    W = t.waves
t0 = wg[:, 0].min()
start = (wg[:, 1] - t0) / 100.0       # us (s_memrealtime, 100 MHz)
end = (wg[:, 2] - t0) / 100.0
cu = wg[:, 3] >> 32
blk = wg[:, 3] & 0xffffffff
cnt = collections.Counter(cu.tolist())
shared = np.array([cnt[c] > 1 for c in cu.tolist()])
print(f"L1={L1} L2={L2} W={W} NSW={len(wg)} kernel_ms={k:.3f}")
print(f"distinct CUs {len(cnt)} for {len(wg)} WG-stripes; WG-stripes per CU: "
      f"{dict(sorted(collections.Counter(cnt.values()).items()))}")
print(f"WG-stripes on a shared CU: {int(shared.sum())}"
      + (f" (indices {np.nonzero(shared)[0][:24].tolist()}{' ...' if shared.sum() > 24 else ''})" if shared.any() else ""))
dur = end - start
for name, sel in (("shared CU", shared), ("own CU", ~shared)):
    if sel.any():
        print(f"  {name:9s}: run time mean {dur[sel].mean():8.1f} us  min {dur[sel].min():8.1f}  max {dur[sel].max():8.1f}")
# pace along the chain: end of WG-stripe s minus end of s-1
de = np.diff(end)
print(f"end-to-end hop per WG-stripe: mean {de.mean():.2f} us, median {np.median(de):.2f}, p90 {np.percentile(de, 90):.2f}")
q = len(wg) // 4
for a_, b_ in ((0, q), (q, 2 * q), (2 * q, 3 * q), (3 * q, len(wg))):
    print(f"  WG-stripes {a_:4d}..{b_ - 1:4d}: run time mean {dur[a_:b_].mean():8.1f} us, "
          f"shared {int(shared[a_:b_].sum())}")
