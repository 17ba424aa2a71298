#!/usr/bin/env python3
"""How the 100k x 100k fill's kernel time varies between fills of one table
and between tables of one process (run via gpurun from the repo root):
    python3 tools/fill_variance.py [--tables 4] [--fills 8] [--L1 100000 --L2 100000]
Prints the kernel time of every fill.  tools/ab_run.py sees the same fill at
8.3 ms in one process and 9.0 ms in the next; this separates the table's
placement in HBM (new per table) from the process."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "needleman-wunsch_amd"))
import ctypes  # noqa: E402
import time  # noqa: E402

import nw_amd  # noqa: E402


def memset_ms(ptr, nbytes, reps=3):
    """Host-timed hipMemset of a device range (a plain streaming write of the same memory)."""
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    out = []
    for _ in range(reps):
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        rc = hip.hipMemset(ctypes.c_void_p(ptr), 0, nbytes)
        hip.hipDeviceSynchronize()
        out.append((time.perf_counter() - t0) * 1e3)
        assert rc == 0, rc
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=4)
    ap.add_argument("--fills", type=int, default=8)
    ap.add_argument("--L1", type=int, default=100000)
    ap.add_argument("--L2", type=int, default=100000)
    ap.add_argument("--memset", action="store_true", help="also time a hipMemset of the score tiles")
    ap.add_argument("--outputs", default="sd", help="what the fill writes: sd | s | d | none")
    a = ap.parse_args()
    s1, s2 = nw_amd.gen_dna(1, a.L1), nw_amd.gen_dna(2, a.L2)
    full = nw_amd.NW_OUT_SCORES | nw_amd.NW_OUT_DIRS
    mask = (nw_amd.NW_OUT_SCORES if "s" in a.outputs else 0) | (nw_amd.NW_OUT_DIRS if "d" in a.outputs else 0)
    for t_i in range(a.tables):
        with nw_amd.Table(a.L1, a.L2, full) as t:
            t.set_sequences(s1, s2)
            ms = []
            for _ in range(a.fills):
                t.fill(1, 1, 1, mask)
                ms.append(t.elapsed_ms()[0])
            tiles, words = t.device_buffers()
            nb = 4 * t.layout().score_pitch * ((a.L2 + 63) // 64)
            mm = memset_ms(tiles, nb) if a.memset else []
            print(f"table {t_i}: tiles 0x{tiles:x} words 0x{words:x}  kernel ms " + " ".join(f"{x:.3f}" for x in ms)
                  + ("  memset ms " + " ".join(f"{x:.3f}" for x in mm) if mm else ""), flush=True)


if __name__ == "__main__":
    main()
