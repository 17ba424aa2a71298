#!/usr/bin/env python3
"""A/B of library variants over a few fill shapes on one box: a lone wave
(L2 = 64), one 8-wave workgroup (NW_WAVES=8, L2 = 512) and the full 100k^2
table, for the given output modes.  Each run is a fresh bench.py process
with NW_LIB pointing at lib_ab/libnwfill_<name>.so.

    python tools/ab_shapes.py [--rounds 2] [--outputs sd,none] [--only v4,v3]
"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--outputs", default="sd")
ap.add_argument("--only", default="")
ap.add_argument("--shapes", default="lone,wg8,full")
a = ap.parse_args()
SHAPES = {"lone": (["--L2", "64"], {}), "wg8": (["--L2", "512"], {"NW_WAVES": "8"}),
          "full": ([], {})}
libs = sorted(glob.glob(os.path.join(ROOT, "lib_ab", "libnwfill_*.so")))
if a.only:
    keep = a.only.split(",")
    libs = [l for l in libs if os.path.basename(l)[10:-3] in keep]
res = {}
for r in range(a.rounds):
    for shape in a.shapes.split(","):
        sargs, senv = SHAPES[shape]
        for outs in a.outputs.split(","):
            for lib in libs:
                name = os.path.basename(lib)[10:-3]
                env = dict(os.environ, NW_LIB=lib, **senv)
                cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--steps", "3",
                       "--warmup", "1", "--outputs", outs, *sargs]
                out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
                try:
                    ms = json.loads(out.stdout.strip().splitlines()[-1])["roofline"]["kernel_ms"]
                except Exception:
                    print(out.stdout[-500:], out.stderr[-1500:], flush=True)
                    raise
                res.setdefault((shape, outs, name), []).append(ms)
                print(f"round {r} {shape:5s} {outs:5s} {name:12s} {ms:8.3f} ms", flush=True)
print("--- min over rounds (kernel ms)")
for (shape, outs, name), v in sorted(res.items()):
    print(f"{shape:5s} {outs:5s} {name:12s} {min(v):8.3f}")
