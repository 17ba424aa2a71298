#!/usr/bin/env python3
"""What row panels cost beyond sharing one GPU (run via gpurun).

A one-GPU rehearsal of N panels mixes two things: the panels' workgroups share
the chip (a CU that hosts workgroups of two panels runs two compute waves per
SIMD, and the whole stripe chain moves at that pace), and the hand-off itself
(the producer's boundary stores, the consumer's polls, the credit wait).  This
tool separates them: it fills tables small enough that all panels together
keep one compute wave per SIMD (rows <= 64 * 4 * CUs), un-split and as 2 / 4 /
8 panels of an in-process group on one device, so the difference is the
hand-off alone; then the 100k x 100k table the same way, where the difference
also contains the sharing.  With $NW_TRACE the kernels stamp each workgroup
stripe's start and end on the GPU's realtime clock (one clock for all panels
of the device), which gives each panel's start lag behind the panel above.

    python tools/panel_cost.py [--L1 100000] [--rows 25600,51200,100000] [--panels 2,4,8] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "needleman-wunsch_amd"))
os.environ.setdefault("NW_TRACE", "1")

import nw_amd  # noqa: E402

SD = nw_amd.NW_OUT_SCORES | nw_amd.NW_OUT_DIRS


def span(tr):
    """(first wave start, last wave end) of one kernel's WG-stripes, in us of the realtime clock."""
    tr = tr[tr[:, 1] > 0]
    return float(tr[:, 1].min()) / 100.0, float(tr[:, 2].max()) / 100.0


def unsplit(L1, L2, reps):
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    with nw_amd.Table(L1, L2, SD) as t:
        t.set_sequences(s1, s2)
        ms = []
        for _ in range(reps + 1):
            t.fill(1, 1, 1, SD)
            ms.append(t.elapsed_ms()[0])
        a, b = span(t.trace())
        return {"kernel_ms": round(min(ms[1:]), 4), "span_ms": round((b - a) / 1e3, 4), "waves": t.waves}


def split(L1, L2, n, reps):
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    panels = nw_amd.Panel.group([0] * n, L1, L2, SD)
    try:
        for p in panels:
            p.set_sequences(s1, s2)
        best = None
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            nw_amd.Panel.group_fill(panels, 1, 1, 1, SD)
            wall = (time.perf_counter() - t0) * 1e3
            traces = [p.table.trace() for p in panels if p.rows()[1] > 0]
            spans = [span(t) for t in traces]
            cus = [set((t[t[:, 1] > 0][:, 3] >> np.uint64(32)).tolist()) for t in traces]
            tot = (max(b for _, b in spans) - min(a for a, _ in spans)) / 1e3
            rec = {"span_ms": round(tot, 4), "wall_ms": round(wall, 3),
                   "panel_kernel_ms": [round(p.elapsed_ms()[0], 3) for p in panels],
                   "panel_span_ms": [round((b - a) / 1e3, 3) for a, b in spans],
                   # a panel's first wave starts this long after the first wave of the panel above
                   "start_lag_us": [round(spans[i][0] - spans[i - 1][0], 1) for i in range(1, len(spans))],
                   # and ends this long after it (the pipeline's skew at the end of the table)
                   "end_lag_us": [round(spans[i][1] - spans[i - 1][1], 1) for i in range(1, len(spans))],
                   # hardware CUs (HW_ID) a panel's workgroups ran on that the panel above used too
                   "cus": [len(c) for c in cus],
                   "cus_shared_with_panel_above": [len(cus[i] & cus[i - 1]) for i in range(1, len(cus))],
                   "waves": [p.table.waves for p in panels]}
            if best is None or rec["span_ms"] < best["span_ms"]:
                best = rec
        return best
    finally:
        for p in panels:
            p.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L1", type=int, default=100_000)
    ap.add_argument("--rows", default="25600,51200,100000")
    ap.add_argument("--panels", default="2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for L2 in (int(x) for x in a.rows.split(",")):
        u = unsplit(a.L1, L2, a.reps)
        print(json.dumps({"L1": a.L1, "L2": L2, "panels": 1, **u}), flush=True)
        for n in (int(x) for x in a.panels.split(",")):
            r = split(a.L1, L2, n, a.reps)
            r["extra_ms_vs_unsplit"] = round(r["span_ms"] - u["span_ms"], 4)
            r["extra_us_per_boundary"] = round(1e3 * (r["span_ms"] - u["span_ms"]) / (n - 1), 1)
            print(json.dumps({"L1": a.L1, "L2": L2, "panels": n, **r}), flush=True)


if __name__ == "__main__":
    main()
