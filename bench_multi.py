"""bench.py --gpus N (N > 1): the 100k x 100k fill split into row panels.

Launched by the driver as
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
or started by a plain `python bench.py --gpus N` (bench.spawn_ranks), one
process per GPU (LOCAL_RANK = device).  Each rank fills its row panel
(include/nw_panel.h) of the SAME table; the panels hand their bottom row down
the chain as the fill runs.  `value` = L1*L2 / (max over ranks of the time of
one whole fill), i.e. strong scaling of one table.

Control traffic only (the boundary rows never touch it) goes through
torch.distributed: the RCCL rendezvous id or the hipIpc handles, the per-rank
stats records, the timing max.  The default process group is NCCL (RCCL); a
gloo side group carries the small Python objects.

Transports (--transport): "ipc" (default) -- the producer's kernel stores the
boundary row straight into the next GPU's buffer over xGMI; "rccl" -- a host
proxy forwards it in blocks with ncclSend/ncclRecv.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if os.path.join(ROOT, "needleman-wunsch_amd") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "needleman-wunsch_amd"))

import nw_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0
TRANSPORTS = {"ipc": nw_amd.NW_PANEL_IPC, "rccl": nw_amd.NW_PANEL_RCCL}


# ------------------------------------------------------------ control plane
# (host logic, covered by tests/test_panel_host.py on gloo)
def exchange_bytes(data: bytes, group=None) -> list[bytes]:
    """Every rank's `data`, in rank order."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, bytes(data), group=group)
    return out


def broadcast_bytes(data: bytes | None, group=None) -> bytes:
    import torch.distributed as dist
    box = [data]
    dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


def gather_records(rec, group=None) -> np.ndarray:
    """(world, NW_PANEL_REC) int64 records of all ranks."""
    rows = exchange_bytes(np.asarray(rec, dtype=np.int64).tobytes(), group)
    return np.stack([np.frombuffer(r, dtype=np.int64) for r in rows])


def max_over_ranks(x: float, group=None) -> float:
    return max(float(np.frombuffer(r, dtype=np.float64)[0])
               for r in exchange_bytes(np.float64(x).tobytes(), group))


def chain_hash_states(panel, L1: int, rank: int, world: int, group=None):
    """Whole-table parity across ranks: the per-column FNV states travel down
    the panel chain (rank r continues them over its own rows and hands them to
    rank r + 1; CPU tensors over gloo).  Every rank returns the folded
    (hH, hD) of the whole table."""
    import torch
    import torch.distributed as dist
    state = nw_amd.hash_states(L1)
    buf = torch.from_numpy(state.view(np.int64))
    if rank > 0:
        dist.recv(buf, src=rank - 1, group=group)
    panel.hash_columns(state)
    if rank + 1 < world:
        dist.send(buf, dst=rank + 1, group=group)
    out = [nw_amd.hash_fold(state) if rank == world - 1 else None]
    dist.broadcast_object_list(out, src=world - 1, group=group)
    return out[0]


def make_panel(transport: str, rank: int, world: int, device: int, L1: int, L2: int, mask: int, group=None):
    """Create + connect this rank's panel (collective)."""
    kind = TRANSPORTS[transport]
    rdv = None
    if kind == nw_amd.NW_PANEL_RCCL:
        rdv = broadcast_bytes(nw_amd.panel_get_id() if rank == 0 else None, group)
    p = nw_amd.Panel(kind, rank, world, L1, L2, mask, device=device, rdv_id=rdv)
    if kind == nw_amd.NW_PANEL_IPC:
        p.ipc_connect(b"".join(exchange_bytes(p.ipc_handle(), group)))
    return p


# ------------------------------------------------------------------- bench
def main(a) -> None:
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    transport = getattr(a, "transport", "ipc")
    pg_backend = getattr(a, "pg_backend", "nccl")
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    device = local if getattr(a, "device", None) is None else a.device
    torch.cuda.set_device(device)
    dist.init_process_group(backend=pg_backend, device_id=torch.device("cuda", device)
                            if pg_backend == "nccl" else None)
    ctl = dist.new_group(backend="gloo")
    m, k, d = a.mkd
    L1, L2 = a.L1, a.L2
    mask = ((nw_amd.NW_OUT_SCORES if "s" in a.outputs else 0) | (nw_amd.NW_OUT_DIRS if "d" in a.outputs else 0)
            | (nw_amd.NW_OUT_STATS if "t" in a.outputs else 0))
    p = make_panel(transport, rank, world, device, L1, L2, mask | nw_amd.NW_OUT_STATS, ctl)
    p.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
    row_base, rows = p.rows()

    for _ in range(a.warmup):
        p.fill(m, k, d, mask)
    kern = []
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        p.fill(m, k, d, mask)
        kern.append(p.elapsed_ms()[0])
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    ms = max_over_ranks(dt / a.steps * 1e3, ctl)
    recs = gather_records(p.record(), ctl)
    rc, st = nw_amd.panel_reduce(recs)
    kern_ms = float(np.mean(kern)) if kern else 0.0
    per_rank = exchange_bytes(json.dumps({"rank": rank, "rows": rows, "kernel_ms": kern_ms,
                                          "waves": p.table.waves}).encode(), ctl)
    # Outside the timed region: the table the last timed step left in the
    # ranks' HBM, hashed on the devices panel by panel (every score; every
    # direction code when written).
    hashes = None
    if "s" in a.outputs and rc == 0 and not getattr(a, "no_hash", False):
        hashes = chain_hash_states(p, L1, rank, world, ctl)
    p.close()
    if rank == 0:
        info = [json.loads(x) for x in per_rank]
        cells = L1 * L2
        value = cells / (ms * 1e-3) / 1e9
        bpc = (4.0 if "s" in a.outputs else 0.0) + (0.5 if "d" in a.outputs else 0.0)
        # dominant kernel: the slowest rank's panel fill
        slow = max(info, key=lambda r: r["kernel_ms"])
        alg = bpc * (L1 + 1) * (slow["rows"] + 1)
        achieved = alg / (slow["kernel_ms"] * 1e-3) / 1e9 if slow["kernel_ms"] > 0 else 0.0
        import bench
        stats = {"corner": st.corner}
        if "t" in a.outputs:
            stats.update(gav=st.greatest_abs_interior, bc=st.branch_count)
        if hashes is not None:
            stats["hH2"] = "%016x" % hashes[0]
            if "d" in a.outputs:
                stats["hD2"] = "%016x" % hashes[1]

        def rank_roofline(r):
            alg_r = bpc * (L1 + 1) * (r["rows"] + (1 if r["rank"] == 0 else 0))
            ach = alg_r / (r["kernel_ms"] * 1e-3) / 1e9 if r["kernel_ms"] > 0 else 0.0
            return {"rank": r["rank"], "rows": r["rows"], "kernel_ms": round(r["kernel_ms"], 4),
                    "waves_per_wg": r["waves"], "achieved_gbs": round(ach, 1),
                    "frac": round(ach / HBM_PEAK_GBS, 4)}
        out = {
            "metric": bench.metric_name(L1, L2),
            "value": round(value, 2), "unit": "GCUPS", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic (splitmix64 DNA, seeds 1/2)",
            "config": {"workload": bench.workload_name(L1, L2, a.outputs, (m, k, d)),
                       "L1": L1, "L2": L2, "parallelism": f"row panels x{world} ({transport})",
                       "corner": st.corner, "status": rc,
                       "panels": [rank_roofline(r) for r in info]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_cell": bpc, "traffic": None,
                         "kernel_ms": round(slow["kernel_ms"], 4), "alg_bytes_per_launch": alg,
                         "kernel_rank": slow["rank"]},
            "parity": dict(bench.parity(L1, L2, (m, k, d), stats), status=rc),
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    dist.barrier(group=ctl)
    dist.destroy_process_group()
