#!/usr/bin/env python3
"""A/B timing of library variants on one box: alternate lib_ab/libnwfill_*.so
(run `bash tools/ab_build.sh NAME ...` first) over several rounds, each run a
fresh process of bench.py, and print per-variant kernel ms.

    python tools/ab_bench.py [--rounds 3] [bench.py args...]
"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
rounds = 3
args = sys.argv[1:]
if args[:1] == ["--rounds"]:
    rounds, args = int(args[1]), args[2:]
libs = sorted(glob.glob(os.path.join(ROOT, "lib_ab", "libnwfill_*.so")))
res = {os.path.basename(l): [] for l in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, NW_LIB=lib)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--steps", "4",
                              "--warmup", "1", *args], env=env, capture_output=True, text=True, timeout=300)
        j = json.loads(out.stdout.strip().splitlines()[-1])
        res[os.path.basename(lib)].append(j["roofline"]["kernel_ms"])
        print(f"round {r} {os.path.basename(lib):32s} kernel_ms {j['roofline']['kernel_ms']:.3f}", flush=True)
for k, v in res.items():
    print(f"{k:32s} min {min(v):.3f}  mean {sum(v) / len(v):.3f}")
