"""One rank of a multi-process panel fill (used by tests/test_gpu_panel.py).

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/panel_ipc_worker.py OUT.npz L1 L2 m k d transport device

Control over a gloo group (bench_multi.py's helpers); every rank runs its
panel on `device` (several ranks on one GPU rehearse the hipIpc path).  Rank
0 writes every rank's local scores/codes/last column + the reduced stats.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "needleman-wunsch_amd")]

import torch.distributed as dist  # noqa: E402

import bench_multi  # noqa: E402
import nw_amd  # noqa: E402


def main():
    out, L1, L2, m, k, d, transport, device = sys.argv[1], *map(int, sys.argv[2:7]), sys.argv[7], int(sys.argv[8])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = bench_multi.make_panel(transport, rank, world, device, L1, L2, nw_amd.NW_OUT_ALL)
    p.set_sequences(nw_amd.gen_dna(1, L1), nw_amd.gen_dna(2, L2))
    # NW_TEST_MKD_SEQ="m,k,d;m,k,d;..." runs those fills back to back (the
    # last one is checked); NW_TEST_DELAY="rank:seconds" makes that rank start
    # every fill late, so the panel above runs ahead and must wait for its
    # credit instead of overwriting a boundary row still being read.
    seq = [tuple(map(int, x.split(","))) for x in os.environ.get("NW_TEST_MKD_SEQ", "").split(";") if x]
    seq = seq or [(m, k, d)] * int(os.environ.get("NW_TEST_FILLS", "2"))
    delay_rank, delay_s = (os.environ.get("NW_TEST_DELAY", "-1:0").split(":") + ["0"])[:2]
    rcs = []
    for mkd in seq:
        if int(delay_rank) == rank:
            time.sleep(float(delay_s))
        rcs.append(p.fill_rc(*mkd, nw_amd.NW_OUT_ALL))
    base, rows = p.rows()
    t = p.table
    payload = {"rank": rank, "base": base, "rows": rows, "rcs": rcs}
    if rcs[-1] == 0 and rows > 0:
        payload["H"] = t.scores()
        payload["D"] = t.codes()
    recs = bench_multi.gather_records(p.record())
    allp = [None] * world
    dist.all_gather_object(allp, payload)
    if rank == 0:
        rc, st = nw_amd.panel_reduce(recs)
        np.savez(out, rc=rc, stats=np.array([st.corner, st.greatest_abs_interior, st.branch_count], dtype=np.int64),
                 **{f"H{r['rank']}": r["H"] for r in allp if "H" in r},
                 **{f"D{r['rank']}": r["D"] for r in allp if "D" in r},
                 meta=np.array([[r["rank"], r["base"], r["rows"], next((x for x in r["rcs"] if x), 0)]
                                   for r in allp], dtype=np.int64))
    dist.barrier()
    p.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
