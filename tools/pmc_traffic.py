#!/usr/bin/env python3
"""Summarise rocprofv3 output of tools/profile_round.sh into profiles/.

    python tools/pmc_traffic.py ROUND OUTDIR L1 L2 [WARMUP]

OUTDIR holds three rocprofv3 runs of `bench.py` (same workload):
  kt/   --kernel-trace --stats        -> per-kernel average duration; the
        steady-state average skips the first WARMUP fill launches (bench.py's
        untimed warm-up), which is what bench.py's HIP-event kernel_ms covers;
        kt.log holds the bench line printed under the profiler
  wr/   --pmc WRITE_SIZE              -> HBM write bytes per fill launch
  rd/   --pmc FETCH_SIZE              -> HBM read bytes per fill launch
Counters come from separate passes (TCC slots: FETCH_SIZE costs 3,
WRITE_SIZE 2, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Both are KiB
(x1024).  gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reads
half the bytes of a wide coalesced stream, so it is doubled; WRITE_SIZE is
exact for 16-B/lane streaming stores (the score tiles).

Writes OUTDIR/<ROUND>_kernel_stats.csv (copy of the stats summary) and
OUTDIR/<ROUND>_pmc_traffic.json; commit both under profiles/ (bench.py reads
profiles/*pmc*.json for roofline.traffic).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
FILL_KERNELS = ("nw_fill_kernel", "nw_skew_kernel", "nw_pair_kernel")   # whichever fill ran


def is_fill(name):
    return any(k in name for k in FILL_KERNELS)


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[-1]


def counter_per_launch(d, name):
    path = find(d, "*counter_collection.csv")
    per = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if not is_fill(r["Kernel_Name"]) or r["Counter_Name"] != name:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"{name}: no fill-kernel rows in {path}")
    vals = list(per.values())
    return sum(vals) / len(vals), len(vals), os.path.relpath(path, ROOT)


def main():
    rnd, out, L1, L2 = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    stats = find(os.path.join(out, "kt"), "*kernel_stats.csv")
    dst = os.path.join(out, f"{rnd}_kernel_stats.csv")
    shutil.copy(stats, dst)
    avg_ns = None
    with open(stats) as f:
        for r in csv.DictReader(f):
            if is_fill(r["Name"]):
                avg_ns = float(r["AverageNs"])
                name = r["Name"]
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    durs = []
    with open(find(os.path.join(out, "kt"), "*kernel_trace.csv")) as f:
        rows = [r for r in csv.DictReader(f) if is_fill(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows]
    steady = durs[warm:] if len(durs) > warm else durs
    steady_ns = sum(steady) / len(steady)
    bench_line = None
    try:
        with open(os.path.join(out, "kt.log")) as f:
            for ln in f:
                if ln.startswith("{") and '"metric"' in ln:
                    bench_line = json.loads(ln)
    except OSError:
        pass
    wr_kib, nw, wsrc = counter_per_launch(os.path.join(out, "wr"), "WRITE_SIZE")
    rd_kib, nr, rsrc = counter_per_launch(os.path.join(out, "rd"), "FETCH_SIZE")
    # the raw per-dispatch counter rows and the kernel trace travel with the summary
    shutil.copy(find(os.path.join(out, "wr"), "*counter_collection.csv"), os.path.join(out, f"{rnd}_pmc_write_size.csv"))
    shutil.copy(find(os.path.join(out, "rd"), "*counter_collection.csv"), os.path.join(out, f"{rnd}_pmc_fetch_size.csv"))
    shutil.copy(find(os.path.join(out, "kt"), "*kernel_trace.csv"), os.path.join(out, f"{rnd}_kernel_trace.csv"))
    write_b = wr_kib * 1024
    fetch_b = 2 * rd_kib * 1024
    alg = 4.5 * (L1 + 1) * (L2 + 1)
    j = {
        "round": rnd, "L1": L1, "L2": L2, "kernel": name, "avg_kernel_ns": avg_ns,
        "launches_traced": len(durs), "warmup_launches_skipped": min(warm, len(durs)),
        "steady_avg_kernel_ns": steady_ns, "steady_min_kernel_ns": min(steady), "steady_max_kernel_ns": max(steady),
        "alg_gbs_steady": 4.5 * (L1 + 1) * (L2 + 1) / steady_ns,
        "bench_line_under_profiler": None if bench_line is None else {
            "ms_per_step": bench_line.get("ms_per_step"),
            "kernel_ms": bench_line.get("roofline", {}).get("kernel_ms"),
            "frac": bench_line.get("roofline", {}).get("frac")},
        "write_bytes_per_launch": write_b, "fetch_bytes_per_launch": fetch_b,
        "hbm_bytes_per_launch": write_b + fetch_b,
        "alg_bytes_per_launch": alg, "traffic_over_alg": (write_b + fetch_b) / alg,
        "hbm_gbs_from_counters": (write_b + fetch_b) / avg_ns if avg_ns else None,
        "launches": {"WRITE_SIZE": nw, "FETCH_SIZE": nr},
        "correction": "WRITE_SIZE*1024 + 2*FETCH_SIZE*1024 (gfx950 FETCH_SIZE halves wide streams)",
        "sources": {"stats": f"profiles/{rnd}_kernel_stats.csv", "trace": f"profiles/{rnd}_kernel_trace.csv", "write": f"profiles/{rnd}_pmc_write_size.csv", "fetch": f"profiles/{rnd}_pmc_fetch_size.csv"},
    }
    with open(os.path.join(out, f"{rnd}_pmc_traffic.json"), "w") as f:
        json.dump(j, f, indent=1)
    print(json.dumps(j))


if __name__ == "__main__":
    main()
