#!/usr/bin/env python3
"""Host I/O throughput of the device-resident table .

    python tools/io_bench.py > profiles/<round>_io_stream.json

- upload: nw_table_set_sequences of two 1,000,000-base sequences (symbol
  coding into pinned staging + H2D), wall ms;
- slices: a 1.08 GB score slice (2700 columns) and a 270 MB code slice of the
  filled 100k x 100k table streamed into pinned (nw_host_alloc) and into
  pageable memory, GB/s on the host clock (nw_table_io_stats).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "needleman-wunsch_amd"))
import nw_amd  # noqa: E402


def rate(io):
    return round(io["copy_bytes"] / io["copy_ms"] / 1e6, 2)


out = {}
with nw_amd.Table(1_000_000, 1_000_000, 0) as t:
    s1, s2 = nw_amd.gen_dna(1, 1_000_000), nw_amd.gen_dna(2, 1_000_000)
    ups = []
    for _ in range(3):
        t.set_sequences(s1, s2)
        ups.append(t.io_stats()["upload_ms"])
    out["upload_1M_plus_1M"] = {"bytes": 2_000_000, "ms_best": round(min(ups), 3), "ms_all": [round(x, 3) for x in ups]}

L = 100_000
i0, i1 = 48_650, 51_350
with nw_amd.Table(L, L) as t:
    t.set_sequences(nw_amd.gen_dna(1, L), nw_amd.gen_dna(2, L))
    t.fill(1, 1, 1, nw_amd.NW_OUT_ALL)
    res = {}
    with nw_amd.HostBuffer((i1 - i0, L + 1), np.int32) as hb:
        for rep in range(2):
            t.scores(i0, i1, out=hb.array)
            res.setdefault("scores_pinned_GBps", []).append(rate(t.io_stats()))
        pg = np.empty((i1 - i0, L + 1), dtype=np.int32)
        for rep in range(2):
            t.scores(i0, i1, out=pg)
            res.setdefault("scores_pageable_GBps", []).append(rate(t.io_stats()))
        assert np.array_equal(pg, hb.array)
    with nw_amd.HostBuffer((i1 - i0, L + 1), np.uint8) as hb:
        for rep in range(2):
            t.codes(i0, i1, out=hb.array)
            res.setdefault("codes_pinned_GBps", []).append(rate(t.io_stats()))
        pg = t.codes(i0, i1)
        res["codes_pageable_GBps"] = [rate(t.io_stats())]
        assert np.array_equal(pg, hb.array)
    out["slice_100k_table"] = {"columns": [i0, i1], "score_bytes": (i1 - i0) * (L + 1) * 4,
                               "code_bytes": (i1 - i0) * (L + 1), **res}
print(json.dumps(out))
