#!/usr/bin/env python3
"""A/B timing sweeps of the fill on one GPU box (run via gpurun from the repo
root).  One tool for every comparison this repository records under
profiles/: library variants, environment knobs, kernels, waves per workgroup,
table shapes and output modes.  Every cell of the cross product is a fresh
bench.py process; the kernel time comes from HIP events on the library's
stream.

    python tools/ab_run.py [--libs 'lib_ab/*.so'] [--env NW_KERNEL=scan,pair]
        [--env NW_WAVES=4,8] [--shapes 100000x100000,10000x10000]
        [--outputs sd,s,none] [--reps 2] [--steps 10] [--warmup 2]

  --libs     glob of alternate builds (tools/ab_build.sh); default: the
             in-tree library only
  --env      VAR=v1,v2,...  (repeatable; '-' as a value leaves VAR unset)
  --shapes   L1xL2 list
  --outputs  what the fill writes: sd | s | d | t | none (score-only)

Prints one line per run and the minimum per cell at the end.
"""
import argparse
import glob
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--shapes", default="100000x100000")
    ap.add_argument("--outputs", default="sd")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    libs = sorted(glob.glob(os.path.join(ROOT, a.libs))) if a.libs else [None]
    if not libs:
        sys.exit(f"no library matches {a.libs}")
    knobs = []
    for e in a.env:
        var, vals = e.split("=", 1)
        knobs.append([(var, v) for v in vals.split(",")])
    shapes = [tuple(int(x) for x in s.split("x")) for s in a.shapes.split(",")]
    res = {}
    for rep in range(a.reps):
        for shape, outs, lib, *kv in itertools.product(shapes, a.outputs.split(","), libs, *knobs):
            env = dict(os.environ)
            if lib:
                env["NW_LIB"] = lib
            for var, v in kv:
                env.pop(var, None)
                if v != "-":
                    env[var] = v
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-c2", "--no-hash",
                   "--steps", str(a.steps), "--warmup", str(a.warmup), "--L1", str(shape[0]), "--L2", str(shape[1]),
                   "--outputs", outs]
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
            try:
                j = json.loads(out.stdout.strip().splitlines()[-1])
            except Exception:
                print(out.stdout[-500:], out.stderr[-1500:], flush=True)
                raise
            ms = j["roofline"]["kernel_ms"]
            key = (f"{shape[0]}x{shape[1]}", outs, os.path.basename(lib) if lib else "in-tree",
                   " ".join(f"{var}={v}" for var, v in kv))
            res.setdefault(key, []).append(ms)
            print(f"rep {rep} {key[0]:15s} {key[1]:5s} {key[2]:34s} {key[3]:24s} {ms:9.4f} ms "
                  f"{j['value']:9.2f} GCUPS W={j['config'].get('waves_per_wg')} parity={j.get('parity', {}).get('ok')}",
                  flush=True)
    print("--- min / mean over reps (kernel ms)")
    for key, v in res.items():
        print(f"{key[0]:15s} {key[1]:5s} {key[2]:34s} {key[3]:24s} {min(v):9.4f} {sum(v) / len(v):9.4f}")


if __name__ == "__main__":
    main()
