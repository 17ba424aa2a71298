#!/usr/bin/env python3
"""Benchmark: GCUPS of the Needleman-Wunsch score-table fill on MI355X.

BASELINE.json metric: "GCUPS (cell updates/s) + achieved HBM GB/s, 100k x 100k
fill at 1/2/4/8 GPUs".  One *step* = one complete fill of the 100,000 x
100,000 table (configs[2]: random DNA, m=k=d=1) -- int32 scores plus packed
direction codes for all (L1+1)(L2+1) cells -- with the sequences already
resident in HBM.  value = L1*L2 / ms_per_step in GCUPS (whole job).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: one process per GPU.  Under torch.distributed.run (RANK/WORLD_SIZE
         set) this process is one rank; run plainly, it starts N rank
         processes itself (before touching any GPU) and exits with their
         status.  The table is split into row panels across the ranks
         (strong scaling of one table, bench_multi.py).

Extra JSON fields:
  roofline     -- the fill kernel's algorithmic bytes (4.5 B/cell: 4 B score
                  + 4 bits of direction code) / its average device time over
                  the timed steps (HIP events on the library's own stream),
                  vs 8 TB/s HBM3E; traffic = HBM bytes per launch from the
                  committed rocprofv3 PMC summary (profiles/*pmc*.json) of
                  this workload, with its source named.  Score-only fills
                  (--outputs '') are VALU-bound: int32 VALU lane-ops per cell
                  (from the generated block) x cells/s vs the int32 VALU peak.
  parity       -- the timed table vs the committed fixture for this workload
                  (tests/golden/): its corner, and the whole table -- every
                  score and direction code, hashed on the device after the
                  timed loop (column-chained FNV-1a-64).
  cpu_baseline -- the reference itself (oracle/_ref/ref_harness: its own
                  compute_table_scores, compiled from its sources) on this
                  host: serial and -p 16 on config C2 (10k x 10k), -p $(nproc)
                  on a smaller sample; fill phase alone and with the
                  reference's allocation + seeding; each leg's rate scaled to
                  100k x 100k (labelled extrapolated: the reference itself
                  would need 1.36 TB there); nproc and the CPU model recorded.
  c2           -- config C2 on the GPU (10k x 10k, same fill) next to it.
"""
import argparse
import glob
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "needleman-wunsch_amd"))

import nw_amd  # noqa: E402  (the library itself loads lazily, on first use)

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
# int32 VALU peak of the chip: 256 CUs x 4 SIMDs, each SIMD 32 lanes per clock
# (a wave64 VALU instruction issues over 2 cycles: MI355X_MICROARCH.md
# "Wave scheduling"), at 2.4 GHz.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# What the fill's own instruction mix can reach: its block is DPP, SDWA and
# three-operand VOP3 instructions, which a SIMD issues at one per ~4.1-4.4
# cycles whatever the wave count (tools/ubench_simd.hip,
# profiles/r01_ubench_simd.txt) -- 64 lanes / 4.1 clk.  A property of this
# code, reported beside the chip peak, not instead of it.
VALU_MIX_TOPS = 256 * 4 * (64 / 4.1) * 2.4e9 / 1e12
GOLDEN = os.path.join(ROOT, "tests", "golden")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--L1", type=int, default=100_000)
    ap.add_argument("--L2", type=int, default=100_000)
    ap.add_argument("--mkd", type=int, nargs=3, default=(1, 1, 1))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the 10k x 10k GPU line")
    ap.add_argument("--no-hash", action="store_true",
                    help="skip the whole-table hash of the timed table (A/B timing runs only)")
    ap.add_argument("--outputs", default="sd",
                    help="what the fill writes: s = scores, d = direction codes, t = stats "
                         "('' or 'none' = score-only); the metric's workload is 'sd'")
    ap.add_argument("--cpu-sample", type=int, default=10_000,
                    help="side of the square sample the CPU reference fills (config C2: 10k)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="-p threads of the reference's pthread leg (capped at nproc; 16 = one GPU's CPU share)")
    ap.add_argument("--transport", choices=("ipc", "rccl"), default="ipc",
                    help="N > 1: how a panel's bottom row reaches the next GPU (bench_multi.py)")
    ap.add_argument("--pg-backend", default="nccl",
                    help="N > 1: torch.distributed backend for barriers (gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--device", type=int, default=None,
                    help="N > 1: force every rank onto this device (rehearsal on one GPU)")
    a = ap.parse_args(argv)
    if a.outputs in ("none", "-"):
        a.outputs = ""
    return a


def mask_of(outputs):
    return ((nw_amd.NW_OUT_SCORES if "s" in outputs else 0) | (nw_amd.NW_OUT_DIRS if "d" in outputs else 0)
            | (nw_amd.NW_OUT_STATS if "t" in outputs else 0))


def workload_name(L1, L2, outputs, mkd):
    kind = ("full-table fill (scores+direction codes)" if outputs == "sd"
            else "score-only fill (last column)" if outputs == "" else f"fill writing '{outputs}'")
    return f"{L1}x{L2} {kind}, m,k,d={mkd[0]},{mkd[1]},{mkd[2]}"


def metric_name(L1, L2):
    return f"GCUPS (cell updates/s), {L1 // 1000}k x {L2 // 1000}k NW score-table fill"


# ---------------------------------------------------------------- fixtures
def fixture_for(L1, L2, mkd):
    """The committed fixture for this exact workload: (file, record) or None."""
    for name in ("big_colchain.json", "big_scoreonly.json"):
        try:
            with open(os.path.join(GOLDEN, name)) as f:
                recs = json.load(f)
        except OSError:
            continue
        for r in recs:
            if (r["L1"], r["L2"], r["m"], r["k"], r["d"]) == (L1, L2, *mkd):
                return name, r
    try:
        with open(os.path.join(GOLDEN, "ref_kats.json")) as f:
            for r in json.load(f):
                if r.get("kind") == "gen" and (r.get("L1"), r.get("L2")) == (L1, L2) and \
                        (r.get("m"), r.get("k"), r.get("d")) == tuple(mkd):
                    return "ref_kats.json", r
    except OSError:
        pass
    return None


def parity(L1, L2, mkd, stats):
    """Compare the timed table with the fixture: the corner, the stats when
    computed, and -- when the table was hashed (stats["hH2"] / ["hD2"], the
    column-chained FNV-1a-64 of every score and every direction code, computed
    on the device after the timed loop) -- the whole table."""
    fx = fixture_for(L1, L2, mkd)
    if fx is None:
        return {"fixture": None, "corner": stats.get("corner")}
    name, r = fx
    out = {"fixture": f"tests/golden/{name}", "corner": stats["corner"], "want_corner": r["corner"],
           "ok": stats["corner"] == r["corner"]}
    if stats.get("gav") is not None and "gav" in r:
        out["gav_ok"] = stats["gav"] == r["gav"]
        out["branch_count_ok"] = stats["bc"] == r.get("branch_count", r.get("bc"))
        out["ok"] = out["ok"] and out["gav_ok"] and out["branch_count_ok"]
    for key in ("hH2", "hD2"):
        if stats.get(key) is not None and key in r:
            out[key] = stats[key]
            out[key + "_ok"] = stats[key] == r[key]
            out["ok"] = out["ok"] and out[key + "_ok"]
    return out


# ---------------------------------------------------------------- roofline
def latest_traffic(L1, L2, outputs):
    """HBM bytes per fill launch from the newest committed rocprofv3 PMC summary of this workload."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(p) as f:
                j = json.load(f)
        except Exception:
            continue
        if j.get("L1") == L1 and j.get("L2") == L2 and j.get("outputs", "sd") == outputs \
                and "hbm_bytes_per_launch" in j:
            best = (os.path.relpath(p, ROOT), j)
    return best


def pair_valu_per_cell(P=True):
    """int32 VALU lane-ops per cell of the score-only pair block (generated by
    tools/gen_pair_asm.py, which stamps the count into nw_pair_chunk.inc)."""
    inc = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_pair_chunk.inc")
    try:
        with open(inc) as f:
            txt = f.read()
    except OSError:
        return None
    m = re.search(r"// VALU pair_chunk_asm<false, false, false, %s>: (\d+) per 8 columns x 128 rows"
                  % ("true" if P else "false"), txt)
    return int(m.group(1)) * 64 / (8 * 128) if m else None


def roofline(L1, L2, outputs, kern_ms):
    cells = L1 * L2
    bpc = (4.0 if "s" in outputs else 0.0) + (0.5 if "d" in outputs else 0.0)
    if bpc == 0.0:
        ops = pair_valu_per_cell()
        ach = cells / (kern_ms * 1e-3) * ops / 1e12 if ops else None
        return {"bound": "valu", "achieved": round(ach, 3) if ach else None, "peak": round(VALU_PEAK_TOPS, 2),
                "unit": "T int32 ops/s", "frac": round(ach / VALU_PEAK_TOPS, 4) if ach else None,
                "ops_per_cell": ops, "traffic": None, "kernel_ms": round(kern_ms, 4),
                "kernel_gcups": round(cells / (kern_ms * 1e-3) / 1e9, 2),
                "mix_ceiling": {"peak": round(VALU_MIX_TOPS, 2), "frac": round(ach / VALU_MIX_TOPS, 4) if ach else None,
                                "what": "issue rate of this block's DPP/SDWA/VOP3 mix (one instruction per "
                                        "~4.1 SIMD cycles, measured); not the chip's peak"},
                "note": "score-only: no table stream; peak = 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz"}
    alg = bpc * (L1 + 1) * (L2 + 1)
    ach = alg / (kern_ms * 1e-3) / 1e9
    tr = latest_traffic(L1, L2, outputs)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_cell": bpc,
            "traffic": tr[1]["hbm_bytes_per_launch"] if tr else None,
            "traffic_source": f"{tr[0]} ({tr[1].get('kernel', '?')[:60]})" if tr else None,
            "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg,
            "kernel_gcups": round(cells / (kern_ms * 1e-3) / 1e9, 2)}


# ---------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def run_ref(n, T, timeout=900):
    """One run of the compiled reference on an n x n sample with T threads:
    {"init_s": alloc + seeding, "fill_s": compute_table_scores, "corner": ...} or None."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    try:
        out = subprocess.run([harness, "gen", str(n), str(n), "1", "1", "1", str(T)], capture_output=True, text=True,
                             timeout=timeout, env=dict(os.environ, NW_REF_TIME_ONLY="1"))
    except subprocess.TimeoutExpired:
        return {"timeout_s": timeout}
    if out.returncode != 0:
        return None
    return json.loads(out.stdout)


def _leg(n, r, what):
    tot = r["init_s"] + r["fill_s"]
    return {"value": round(n * n / r["fill_s"] / 1e9, 5), "unit": "GCUPS",
            "value_with_alloc_seed": round(n * n / tot / 1e9, 5),
            "fill_s": round(r["fill_s"], 3), "alloc_seed_s": round(r["init_s"], 3),
            # The reference needs 136 B per cell: 1.36 TB at 100k x 100k, so it
            # cannot run there; its rate on the sample, scaled by the cell count.
            "extrapolated_100k_s": round(1e10 / (n * n) * tot, 1),
            "sample": f"{n}x{n} random DNA, m=k=d=1, {what}: alloc+seed {r['init_s']:.2f} s, "
                      f"fill {r['fill_s']:.2f} s; corner {r['corner']}"}


def cpu_baseline(n, threads, n_all=3000):
    """The reference's own fill on this host's cores, on bounded samples:
    serial and `-p threads` on an n x n table (config C2 when n = 10k), and
    `-p $(nproc)` -- what configs[1] names -- on an n_all x n_all table (every
    thread of that leg blocks on a per-cell condition variable,
    needleman-wunsch.c:444-475, so it is the slowest leg by far and gets the
    smallest sample).  `value` is the fill phase alone, like the GPU line;
    `value_with_alloc_seed` adds the reference's allocation and seeding, which
    under -p initialises a mutex and a condition variable per cell
    (computation.c:80-89)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    nproc = os.cpu_count() or 1
    if os.path.exists(harness):
        r = run_ref(n, 1)
        if r is not None and "fill_s" in r:
            res = _leg(n, r, "the reference's compute_table_scores (needleman-wunsch.c:583, serial, "
                             "-O3 -DNDEBUG), tables calloc'd cold as in the reference")
            res.update(cores=1, kind="reference", nproc=nproc, cpu_model=cpu_model())
            T = max(2, min(threads, nproc))
            rp = run_ref(n, T)
            if rp is not None and "fill_s" in rp:
                what = (f"-p {T} = -p $(nproc), configs[1]'s CPU leg" if T == nproc
                        else f"-p {T} (this GPU's CPU share of the host's {nproc})")
                res["pthread"] = dict(_leg(n, rp, what), threads=T)
            if nproc > T:
                ra = run_ref(n_all, nproc, timeout=150)
                if ra is not None and "fill_s" in ra:
                    res["pthread_nproc"] = dict(_leg(n_all, ra, f"-p {nproc} = -p $(nproc), configs[1]'s CPU leg, on "
                                                                f"a smaller sample to bound the run"), threads=nproc)
                elif ra is not None:
                    res["pthread_nproc"] = {"threads": nproc, "value": None,
                                            "sample": f"{n_all}x{n_all}, -p {nproc}: not finished in {ra['timeout_s']} s"}
            return res
    # Fallback: the clean-room restatement (same algorithm, dense layout).
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O  # checker/baseline only
    s1, s2 = O.gen_dna(1, n), O.gen_dna(2, n)
    t0 = time.perf_counter()
    O.fill(s1, s2, 1, 1, 1)
    dt = time.perf_counter() - t0
    return {"value": round(n * n / dt / 1e9, 5), "unit": "GCUPS", "cores": 1, "kind": "port", "nproc": nproc,
            "cpu_model": cpu_model(), "extrapolated_100k_s": round(1e10 / (n * n) * dt, 1),
            "sample": f"{n}x{n} random DNA, m=k=d=1: oracle/nw_oracle.c serial fill {dt:.2f} s"}


# ---------------------------------------------------------------- single GPU
def time_fills(L1, L2, mkd, outputs, steps, warmup, hash_table=True):
    m, k, d = mkd
    mask = mask_of(outputs)
    with nw_amd.Table(L1, L2, mask | nw_amd.NW_OUT_STATS) as t:
        t.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
        for _ in range(warmup):
            t.fill(m, k, d, mask)
        kern = []
        t0 = time.perf_counter()
        for _ in range(steps):
            t.fill(m, k, d, mask)        # synchronous: memsets + fill kernel
            kern.append(t.elapsed_ms()[0])
        dt = time.perf_counter() - t0
        st = t.stats()
        stats = {"corner": st.corner}
        if "t" in outputs:
            stats.update(gav=st.greatest_abs_interior, bc=st.branch_count)
        # Outside the timed region: the table the last timed step left in HBM,
        # hashed on the device (every score; every direction code when written).
        if "s" in outputs and hash_table:
            hH, hD = t.hash()
            stats["hH2"] = "%016x" % hH
            if "d" in outputs:
                stats["hD2"] = "%016x" % hD
        return dt, kern, t.waves, stats


def run_single(a):
    L1, L2 = a.L1, a.L2
    dt, kern, waves, stats = time_fills(L1, L2, a.mkd, a.outputs, a.steps, a.warmup, not a.no_hash)
    ms = dt / a.steps * 1e3
    kern_ms = sum(kern) / len(kern)
    out = {
        "metric": metric_name(L1, L2),
        "value": round(L1 * L2 / (ms * 1e-3) / 1e9, 2), "unit": "GCUPS", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int32", "data": "synthetic (splitmix64 DNA, seeds 1/2)",
        "config": {"workload": workload_name(L1, L2, a.outputs, a.mkd), "L1": L1, "L2": L2,
                   "parallelism": "single GPU", "waves_per_wg": waves, "corner": stats["corner"]},
        "roofline": roofline(L1, L2, a.outputs, kern_ms),
        "parity": parity(L1, L2, tuple(a.mkd), stats),
    }
    if not a.no_c2 and (L1, L2) != (10_000, 10_000):
        dt2, kern2, _, st2 = time_fills(10_000, 10_000, (1, 1, 1), "sd", 20, 5, not a.no_hash)
        ms2 = dt2 / 20 * 1e3
        out["c2"] = {"workload": workload_name(10_000, 10_000, "sd", (1, 1, 1)), "gcups": round(1e8 / (ms2 * 1e-3) / 1e9, 2),
                     "ms_per_step": round(ms2, 4), "kernel_ms": round(sum(kern2) / len(kern2), 4),
                     "parity": parity(10_000, 10_000, (1, 1, 1), st2)}
    out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(a.cpu_sample, a.cpu_threads)
    if out.get("c2") and out["cpu_baseline"] and a.cpu_sample == 10_000:
        cb = out["cpu_baseline"]
        out["c2"]["vs_cpu_serial"] = round(out["c2"]["gcups"] / cb["value"], 1)
        if "pthread" in cb:
            out["c2"]["vs_cpu_pthread"] = round(out["c2"]["gcups"] / cb["pthread"]["value"], 1)
    print(json.dumps(out), flush=True)


# ---------------------------------------------------------------- N > 1 launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a, argv):
    """Start one rank process per GPU (no GPU is touched here) and wait.

    The children are plain processes started with the env torch.distributed.run
    would give them; if one fails, the others are stopped rather than left
    waiting in a barrier."""
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a, argv))
    if a.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import bench_multi  # row-panel strong scaling (N > 1)
        return bench_multi.main(a)
    run_single(a)


if __name__ == "__main__":
    main()
