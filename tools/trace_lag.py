#!/usr/bin/env python3
"""Where the pair kernel's pipeline lag goes: per-stripe lag at mid-table.

    python tools/trace_lag.py L1 L2 [sd|'']

Needs a library built with -DNW_TRACE_EXT=1 (bash tools/ab_build.sh trace
-DNW_TRACE_EXT=1, then NW_LIB=lib_ab/libnwfill_trace.so).  $NW_TRACE makes
the pair kernel stamp, per 128-row stripe, the time its
compute wave reaches the middle chunk of the table (trace words 8*NSW + g).
The lag of stripe g+1 behind stripe g there is the steady-state pipeline lag;
it is split into hops inside a workgroup (LDS ring) and hops between
workgroups (granules through L2).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "needleman-wunsch_amd"))
os.environ["NW_TRACE"] = "1"
os.environ.setdefault("NW_KERNEL", "pair")
import nw_amd  # noqa: E402

L1, L2 = int(sys.argv[1]), int(sys.argv[2])
mask = {"sd": 3, "": 0, "s": 1, "d": 2}[sys.argv[3] if len(sys.argv) > 3 else "sd"]
NG = (L2 + 127) // 128
with nw_amd.Table(L1, L2, mask | 4) as t:
    t.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
    for _ in range(3):
        t.fill(1, 1, 1, mask)
    wg = t.trace().astype(np.int64)
    mid = t.trace(mid=True).astype(np.int64)
    k = t.elapsed_ms()[0]
    W = t.waves
NSW = len(wg)
ext = mid
mid, pub, lod = ext[:NG], ext[NG:NG + NSW], ext[NG + NSW:NG + 2 * NSW]
lin, lcr = ext[NG + 2 * NSW:NG + 3 * NSW], ext[NG + 3 * NSW:NG + 4 * NSW]
if os.environ.get("NW_WAVES"):
    SQ, SR = W, 0
else:
    SQ, SR = NG // NSW, NG % NSW
owner = np.empty(NG, dtype=np.int64)
for s in range(NSW):
    g0 = s * SQ + min(s, SR)
    n = min(SQ + (1 if s < SR else 0), NG - g0)
    owner[g0:g0 + n] = s
t0 = wg[:, 0].min()
end = (wg[:, 2] - t0) / 100.0
midus = (mid - t0) / 100.0
lag = np.diff(midus)
cross = owner[1:] != owner[:-1]
print(f"L1={L1} L2={L2} mask={mask} W={W} NSW={NSW} NG={NG} kernel_ms={k:.3f}")
print(f"WG-stripe end: first {end[0]:.1f} us, last {end[-1]:.1f} us")
print(f"mid-table time: stripe 0 {midus[0]:.1f} us, last {midus[-1]:.1f} us -> total lag {midus[-1] - midus[0]:.1f} us")
for name, sel in (("in-WG (LDS ring)", ~cross), ("cross-WG (granules)", cross)):
    x = lag[sel]
    if len(x):
        print(f"  {name:22s} hops {len(x):4d}: mean {x.mean():6.2f} us  median {np.median(x):6.2f}  "
              f"p10 {np.percentile(x, 10):6.2f}  p90 {np.percentile(x, 90):6.2f}  sum {x.sum():8.1f} us")
pos = np.arange(NG - 1) - np.array([0 if s == 0 else 0 for s in range(NG - 1)])
# lag by wave position inside its WG (0 = first wave of the WG, whose input comes from granules)
first = np.array([owner[g] * SQ + min(owner[g], SR) for g in range(NG)])
posw = np.arange(NG) - first
for p in range(W):
    sel = posw[1:] == p
    if sel.any():
        print(f"  lag into wave position {p}: mean {lag[sel].mean():6.2f} us  (n={sel.sum()})")

# one cross-WG hop at the middle chunk cm, split: the producer WG's last wave
# starts cm (mid) -> its publisher has stored cm's granules (pub) -> the next
# WG's loader has them in ring 0 (load) -> that WG's first wave starts cm (mid)
lastg = np.array([s * SQ + min(s, SR) + min(SQ + (1 if s < SR else 0), NG - (s * SQ + min(s, SR))) - 1
                  for s in range(NSW)])
firstg = np.array([s * SQ + min(s, SR) for s in range(NSW)])
a1 = (pub[:-1] - mid[lastg[:-1]]) / 100.0
a2 = (lod[1:] - pub[:-1]) / 100.0
a3 = (mid[firstg[1:]] - lod[1:]) / 100.0
for name, x in (("last wave starts cm -> granules stored", a1), ("granules stored -> loader has them", a2),
                ("loader has them -> next WG's wave 0 starts cm", a3)):
    print(f"  {name:46s}: mean {x.mean():6.2f} us  median {np.median(x):6.2f}  p90 {np.percentile(x, 90):6.2f}")

xcc = wg[:, 7]
same = xcc[1:] == xcc[:-1]
print(f"  XCDs seen: {sorted(set(xcc.tolist()))}; consecutive WG-stripes on one XCD: {same.sum()} of {len(same)}")
hop = np.array([(mid[firstg[s + 1]] - mid[lastg[s]]) / 100.0 for s in range(NSW - 1)])
for name, sel in (("same-XCD", same), ("cross-XCD", ~same)):
    if sel.any():
        print(f"  cross-WG hop, {name:9s}: mean {hop[sel].mean():6.2f} us  median {np.median(hop[sel]):6.2f}  "
              f"visibility mean {a2[sel].mean():6.2f} median {np.median(a2[sel]):6.2f}  (n={sel.sum()})")

b1 = (lcr[1:] - lin[1:]) / 100.0
b2 = (lod[1:] - lcr[1:]) / 100.0
b0 = (lin[1:] - pub[:-1]) / 100.0
print(f"  loader reaches cm - granules stored: mean {b0.mean():6.2f} median {np.median(b0):6.2f} us (negative: loader was early)")
print(f"  loader ring-credit wait at cm      : mean {b1.mean():6.2f} median {np.median(b1):6.2f} us")
print(f"  loader granule wait at cm          : mean {b2.mean():6.2f} median {np.median(b2):6.2f} us")
