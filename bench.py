#!/usr/bin/env python3
"""Benchmark: GCUPS of the 100k x 100k Needleman-Wunsch score-table fill.

BASELINE.json metric: "GCUPS (cell updates/s) + achieved HBM GB/s, 100k x 100k
fill at 1/2/4/8 GPUs".  One *step* = one complete fill of the 100,000 x
100,000 table (configs[2]: random DNA, m=k=d=1) -- int32 scores plus packed
direction codes for all (L1+1)(L2+1) cells -- with the sequences already
resident in HBM.  value = L1*L2 / (ms_per_step) in GCUPS (whole job).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: launched by torch.distributed.run, one rank per GPU; the table is
         split into row panels across ranks (strong scaling, bench_multi.py,
         DESIGN.md "Multi-GPU").

Extra JSON fields:
  roofline     -- fill kernel's algorithmic bytes (4.5 B/cell: 4 B score +
                  4 bits of direction code) / its average device time (HIP
                  events on the library's own stream), vs 8 TB/s HBM3E.
  cpu_baseline -- the reference itself (oracle/_ref/ref_harness, serial
                  compute_table_scores) timed on this host on a bounded sample.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "needleman-wunsch_amd"))

import nw_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
BYTES_PER_CELL = 4.5             # int32 score + 4-bit code


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--L1", type=int, default=100_000)
    ap.add_argument("--L2", type=int, default=100_000)
    ap.add_argument("--mkd", type=int, nargs=3, default=(1, 1, 1))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--outputs", default="sd",
                    help="what the fill writes: s = scores, d = direction codes, t = stats "
                         "('' = score-only); the metric's workload is 'sd'")
    ap.add_argument("--cpu-sample", type=int, default=14142,
                    help="side of the square sample the CPU reference fills (~2e8 cells)")
    ap.add_argument("--transport", choices=("ipc", "rccl"), default="ipc",
                    help="N > 1: how a panel's bottom row reaches the next GPU (bench_multi.py)")
    ap.add_argument("--pg-backend", default="nccl",
                    help="N > 1: torch.distributed backend for barriers (gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--device", type=int, default=None,
                    help="N > 1: force every rank onto this device (rehearsal on one GPU)")
    return ap.parse_args()


def cpu_baseline(n):
    """Time the reference's own serial fill on an n x n sample on this host."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    cores = 1
    if os.path.exists(harness):
        out = subprocess.run([harness, "gen", str(n), str(n), "1", "1", "1", "1"],
                             capture_output=True, text=True, timeout=600)
        if out.returncode == 0:
            r = json.loads(out.stdout)
            res = {"value": round(n * n / r["fill_s"] / 1e9, 5), "unit": "GCUPS", "cores": cores,
                   "kind": "reference",
                   "sample": f"{n}x{n} random DNA, m=k=d=1: reference compute_table_scores "
                             f"(needleman-wunsch.c:583, serial, -O3 -DNDEBUG) fill phase "
                             f"{r['fill_s']:.2f} s, tables calloc'd cold as in the reference"}
            # The reference's -p path (per-cell mutex/cond hand-off, needleman-wunsch.c:444-475)
            # on this host's share of cores, on a smaller sample: it is slower than serial.
            T = min(16, os.cpu_count() or 1)
            npar = max(256, n // 4)
            outp = subprocess.run([harness, "gen", str(npar), str(npar), "1", "1", "1", str(T)],
                                  capture_output=True, text=True, timeout=600)
            if outp.returncode == 0:
                rp = json.loads(outp.stdout)
                res["pthread"] = {"value": round(npar * npar / rp["fill_s"] / 1e9, 5), "unit": "GCUPS",
                                  "threads": T, "sample": f"{npar}x{npar}, -p {T}: fill phase {rp['fill_s']:.2f} s"}
            return res
    # Fallback: the clean-room restatement (same algorithm, dense layout).
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O  # checker/baseline only
    s1, s2 = O.gen_dna(1, n), O.gen_dna(2, n)
    t0 = time.perf_counter()
    O.fill(s1, s2, 1, 1, 1)
    dt = time.perf_counter() - t0
    return {"value": round(n * n / dt / 1e9, 5), "unit": "GCUPS", "cores": cores, "kind": "port",
            "sample": f"{n}x{n} random DNA, m=k=d=1: oracle/nw_oracle.c serial fill {dt:.2f} s"}


def latest_traffic(L1, L2):
    """HBM bytes per fill launch from the newest committed rocprofv3 PMC summary."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(p) as f:
                j = json.load(f)
        except Exception:
            continue
        if j.get("L1") == L1 and j.get("L2") == L2 and "hbm_bytes_per_launch" in j:
            best = j
    return best


def run_single(a):
    m, k, d = a.mkd
    L1, L2 = a.L1, a.L2
    s1, s2 = nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2)
    mask = ((nw_amd.NW_OUT_SCORES if "s" in a.outputs else 0) | (nw_amd.NW_OUT_DIRS if "d" in a.outputs else 0)
            | (nw_amd.NW_OUT_STATS if "t" in a.outputs else 0))
    t = nw_amd.Table(L1, L2, mask | nw_amd.NW_OUT_STATS)
    t.set_sequences(s1, s2)
    for _ in range(a.warmup):
        t.fill(m, k, d, mask)
    kern = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.fill(m, k, d, mask)           # synchronous: memsets + seed + fill kernel
        kern.append(t.elapsed_ms()[0])
    dt = time.perf_counter() - t0
    waves = t.waves
    corner = t.stats().corner
    t.close()
    return dt, kern, waves, corner


def main():
    a = parse()
    if a.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import bench_multi  # row-panel strong scaling (N > 1)
        return bench_multi.main(a)
    L1, L2 = a.L1, a.L2
    dt, kern, waves, corner = run_single(a)
    ms = dt / a.steps * 1e3
    cells = L1 * L2
    value = cells / (ms * 1e-3) / 1e9
    kern_ms = sum(kern) / len(kern)
    bpc = (4.0 if "s" in a.outputs else 0.0) + (0.5 if "d" in a.outputs else 0.0)
    alg_bytes = bpc * (L1 + 1) * (L2 + 1)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    tr = latest_traffic(L1, L2)
    out = {
        "metric": "GCUPS (cell updates/s), 100k x 100k NW score-table fill",
        "value": round(value, 2), "unit": "GCUPS", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int32", "data": "synthetic (splitmix64 DNA, seeds 1/2)",
        "config": {"workload": f"{L1}x{L2} " + ("full-table fill (scores+direction codes)" if a.outputs == "sd"
                                                 else f"fill writing '{a.outputs}'") +
                               f", m,k,d={a.mkd[0]},{a.mkd[1]},{a.mkd[2]}",
                   "L1": L1, "L2": L2, "parallelism": "single GPU", "waves_per_wg": waves,
                   "corner": corner},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_cell": bpc,
                     "traffic": tr["hbm_bytes_per_launch"] if tr else None,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes,
                     "kernel_gcups": round(cells / (kern_ms * 1e-3) / 1e9, 2)},
        "cpu_baseline": None if a.no_cpu_baseline else cpu_baseline(a.cpu_sample),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
