#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (where /root/reference exists) after
`make -C oracle ref`:

    python tests/golden/make_golden.py            # KATs + CLI goldens (seconds)
    python tests/golden/make_golden.py --big      # + 100k x 100k colchain (minutes)

Sources:
  * ref_kats.json   -- oracle/_ref/ref_harness: the compiled reference's own
                       compute_table_scores() (needleman-wunsch.c:583-626) on
                       the listed inputs; stats + full-table FNV hashes, and the
                       full tables for tiny cases.
  * cli_cases.json  -- oracle/_ref/needleman-wunsch: stdout, stderr and exit
                       status of the reference CLI (needleman-wunsch.c:698-795)
                       run as `needleman-wunsch` (argv[0] matters: dbg.c:7-15).
  * walk_kats.json   -- oracle/_ref/needleman-wunsch: the optimal-alignment
                       count (`-q -s`, needleman-wunsch.c:250-255 via
                       print_summary, computation.c:271-281) and the first
                       alignment it prints (the first two stdout lines),
                       for the walk services (nw_table_count_alignments,
                       nw_table_first_path).
  * big_colchain.json -- 100k x 100k is beyond the reference (1.36 TB of
                       tables): produced by the clean-room restatement
                       oracle/libnworacle.so, which ref_kats.json pins against
                       the reference up to 10k x 10k (parity is transitive).
Only inputs and outputs are stored; no reference source travels.
"""
import argparse
import ctypes
import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
HARNESS = os.path.join(REF_DIR, "ref_harness")
REF_CLI = os.path.join(REF_DIR, "needleman-wunsch")

# (kind, A, B, m, k, d): kind "gen" -> splitmix64 DNA of lengths A, B
# (seeds 1, 2); kind "str" -> literal strings.
KATS = [
    ("str", "GCATGCU", "GATTACA", 1, 1, 1),
    ("str", "GAT", "GTA", 1, 1, 1),
    ("str", "GT", "GT", 1, 1, 1),
    ("str", "GT", "GA", 1, 1, 1),
    ("str", "AAAAAAAAAA", "A", 1, 1, 1),
    ("str", "A", "A", 2, 1, -1),
    ("str", "", "ACGT", 1, 1, 1),
    ("str", "ACGT", "", 1, 1, 1),
    ("str", "", "", 1, 1, 1),
    ("str", "hello,world!", "yellow~word?", 3, 2, 1),
    ("str", "AAAA", "AA", 1, 1, 1),
    ("gen", 1, 1, 1, 1, 1),
    ("gen", 1, 50, 1, 1, 1),
    ("gen", 50, 1, 1, 1, 1),
    ("gen", 63, 64, 1, 1, 1),
    ("gen", 64, 64, 1, 1, 1),
    ("gen", 65, 65, 1, 1, 1),
    ("gen", 100, 100, 1, 1, 1),
    ("gen", 127, 129, 0, 0, 0),
    ("gen", 300, 200, 2, 3, 5),
    ("gen", 200, 300, -1, -2, -3),
    ("gen", 1000, 777, 1, 1, 1),
    ("gen", 777, 1000, 1, 1, 1),
    ("gen", 1000, 1000, 1, 1, 1),
    ("gen", 1000, 1000, 2, 3, 5),
    ("gen", 1000, 1000, 5, -4, 2),
    ("gen", 1000, 1000, 1, 1, -1),
    ("gen", 4096, 4096, 1, 1, 1),
    ("gen", 3000, 5000, 4, 2, 3),
    ("gen", 10000, 10000, 1, 1, 1),
    ("gen", 10000, 7000, 2, 3, 5),
]
FULL_TABLE_MAX_CELLS = 400

CLI_CASES = [
    # name, args, stdin
    ("readme_table_q_s_t", ["-q", "-s", "-t", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("readme_q", ["-q", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("readme_s_t", ["-s", "-t", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("readme_l_s_t_u", ["-l", "-s", "-t", "-u", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("readme_all_color", ["-c", "-l", "-s", "-t", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("readme_color_u", ["-c", "-u", "-t", "-q", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("gt_gt", ["1", "1", "1"], "GT GT\n"),
    ("gt_ga", ["1", "1", "1"], "GT GA\n"),
    ("gat_gta", ["1", "1", "1"], "GAT GTA\n"),
    ("gat_gta_s", ["-s", "1", "1", "1"], "GAT GTA\n"),
    ("gat_gta_l", ["-l", "1", "1", "1"], "GAT GTA\n"),
    ("gat_gta_lq", ["-l", "-q", "1", "1", "1"], "GAT GTA\n"),
    ("gat_gta_t", ["-t", "1", "1", "1"], "GAT GTA\n"),
    ("gat_gta_c", ["-c", "1", "1", "1"], "GAT GTA\n"),
    ("width_quirk", ["-q", "-t", "1", "1", "1"], "AAAAAAAAAA A\n"),
    ("negative_operands", ["-s", "-t", "--", "2", "1", "-1"], "GATTA GCAT\n"),
    ("zero_operands", ["-s", "-l", "0", "0", "0"], "ACG TG\n"),
    ("many_alignments", ["-s", "-l", "1", "1", "1"], "AAAA AA\n"),
    ("empty_s1", ["-s", "-t", "1", "1", "1"], "   ACGT\n"),
    ("empty_s1_s2", ["-s", "-t", "1", "1", "1"], "\n\n  \n"),
    ("empty_s1_s2_q_s", ["-q", "-s", "1", "1", "1"], "\n\n  \n"),
    ("nul_token_q_s", ["-q", "-s", "1", "1", "1"], " \0"),
    ("empty_s1_q_s", ["-q", "-s", "1", "1", "1"], "   ACGT\n"),
    # many co-optimal alignments: the enumeration order (diag > left > up)
    ("many_alignments_924_l", ["-l", "-s", "1", "1", "1"], "AAAAAAAAAAAA AAAAAA\n"),
    ("many_alignments_252", ["1", "1", "1"], "AAAAAAAAAA AAAAA\n"),
    ("many_alignments_ql_t", ["-q", "-l", "-t", "1", "1", "1"], "ACACACACAC CACACA\n"),
    ("random_48_ql", ["-q", "-l", "-s", "--", "1", "1", "1"],
     "GGTCCTTGCTCGAACGTGCAGATACAGTTAGCCATTGACCGATTGCAA GGGTCCGGCGCCTATTCAGACGGAACCTGTTACCAGGATTACGCATT\n"),
    ("third_token_ignored", ["-s", "-l", "1", "1", "1"], "ACGT AGT CCCC\n"),
    ("multiline", ["-s", "1", "1", "1"], "ACGTTGCA\n\n\tAGTTCA"),
    ("threads_p2", ["-p", "2", "-s", "-t", "1", "1", "1"], "GCATGCU GATTACA\n"),
    ("random_20", ["-s", "-l", "-t", "-u", "1", "1", "1"], "GGTCCTTGCTCGAACGTGCA GGGTCCGGCGCCTATTCAGA\n"),
    ("random_quiet_summary", ["-q", "-s", "2", "3", "5"],
     "GGTCCTTGCTCGAACGTGCAGATACAGTTAGCCA GGGTCCGGCGCCTATTCAGACGGAACCTGTTA\n"),
    ("file_input", ["-s", "-f", "{FILE}", "1", "1", "1"], "GATTACA GCATGCU\n"),
    # error paths (all exit 1)
    ("err_no_operands", [], "A B\n"),
    ("err_two_operands", ["1", "1"], "A B\n"),
    ("err_four_operands", ["1", "1", "1", "1"], "A B\n"),
    ("err_p1", ["-p", "1", "1", "1", "1"], "A B\n"),
    ("err_help", ["-h"], ""),
    ("err_bad_option", ["-x", "1", "1", "1"], "A B\n"),
    ("err_missing_p_arg", ["-p"], ""),
    ("err_eof_one_token", ["1", "1", "1"], "ACGT"),
    ("err_eof_empty", ["1", "1", "1"], ""),
    ("err_no_file", ["-f", "/nonexistent/nw_input.txt", "1", "1", "1"], ""),
]


def run_harness(kind, a, b, m, k, d, dump=None):
    args = [HARNESS, kind, str(a), str(b), str(m), str(k), str(d), "1"]
    if dump:
        args.append(dump)
    return json.loads(subprocess.check_output(args))


def make_kats():
    out = []
    for kind, a, b, m, k, d in KATS:
        with tempfile.NamedTemporaryFile(suffix=".bin") as tf:
            r = run_harness(kind, a, b, m, k, d, tf.name)
            case = {"kind": kind, "m": m, "k": k, "d": d, "L1": r["L1"], "L2": r["L2"],
                    "corner": r["corner"], "gav": r["gav"], "branch_count": r["branch_count"],
                    "hH": r["hH"], "hD": r["hD"]}
            if kind == "str":
                case["s1"], case["s2"] = a, b
            ncell = (r["L1"] + 1) * (r["L2"] + 1)
            if ncell <= FULL_TABLE_MAX_CELLS:
                raw = open(tf.name, "rb").read()
                case["H"] = list(struct.unpack("<%di" % ncell, raw[:4 * ncell]))
                case["codes"] = list(raw[4 * ncell:5 * ncell])
        out.append(case)
        print("kat", kind, case["L1"], case["L2"], m, k, d, case["corner"], case["hH"], file=sys.stderr)
    return out


def run_cli(binary, args, stdin, file_content=None):
    tmp = None
    if any("{FILE}" in a for a in args):
        tmp = tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False)
        tmp.write(file_content if file_content is not None else stdin)
        tmp.close()
        args = [tmp.name if a == "{FILE}" else a for a in args]
        stdin = ""
    try:
        p = subprocess.run(["needleman-wunsch"] + args, executable=binary, input=stdin.encode(),
                           capture_output=True, timeout=120)
    finally:
        if tmp:
            os.unlink(tmp.name)
    return p.returncode, p.stdout, p.stderr


def make_cli():
    out = []
    for name, args, stdin in CLI_CASES:
        rc, so, se = run_cli(REF_CLI, args, stdin)
        out.append({"name": name, "args": args, "stdin": stdin, "rc": rc,
                    "stdout": so.decode("utf-8"), "stderr": se.decode("utf-8")})
        print("cli", name, rc, len(so), len(se), file=sys.stderr)
    return out


def make_big():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "libnworacle.so"))

    class St(ctypes.Structure):
        _fields_ = [("corner", ctypes.c_int32), ("gav", ctypes.c_int32), ("bc", ctypes.c_uint32)]

    out = []
    # 100k x 100k (configs[2]) first: the tests index it as record 0; then
    # configs[1] in the same column-chained form, for bench.py's C2 line.
    for L1, L2, m, k, d in [(100000, 100000, 1, 1, 1), (10000, 10000, 1, 1, 1)]:
        b1, b2 = ctypes.create_string_buffer(L1), ctypes.create_string_buffer(L2)
        lib.nwo_gen_dna(ctypes.c_uint64(1), ctypes.c_int64(L1), b1)
        lib.nwo_gen_dna(ctypes.c_uint64(2), ctypes.c_int64(L2), b2)
        st, h1, h2 = St(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.nwo_fill_colchain(b1, ctypes.c_int64(L1), b2, ctypes.c_int64(L2), m, k, d,
                              ctypes.byref(h1), ctypes.byref(h2), ctypes.byref(st))
        out.append({"L1": L1, "L2": L2, "m": m, "k": k, "d": d, "corner": st.corner, "gav": st.gav,
                    "branch_count": st.bc, "hH2": "%016x" % h1.value, "hD2": "%016x" % h2.value,
                    "source": "oracle/libnworacle.so nwo_fill_colchain (restatement; transitive parity)"})
        print("big", out[-1], file=sys.stderr)
    return out


# Walk services (alignment count, first printed alignment): (kind, A, B, m, k, d).
# Kept only when the reference's exhaustive walk finishes within WALK_TIMEOUT.
WALK_CASES = [
    ("str", "GCATGCU", "GATTACA", 1, 1, 1),
    ("str", "GAT", "GTA", 1, 1, 1),
    ("str", "GATTA", "GCAT", 2, 1, -1),
    ("str", "ACG", "TG", 0, 0, 0),
    ("str", "AAAA", "AA", 1, 1, 1),
    ("str", "AAAAAAAAAA", "A", 1, 1, 1),
    ("str", "hello,world!", "yellow~word?", 3, 2, 1),
    ("str", "A", "ACGTACGT", 1, 1, 1),
    ("gen", 1, 1, 1, 1, 1),
    ("gen", 1, 50, 1, 1, 1),
    ("gen", 50, 1, 1, 1, 1),
    ("gen", 40, 40, 1, 1, 1),
    ("gen", 60, 50, 1, 1, 1),
    ("gen", 63, 65, 2, 3, 5),
    ("gen", 64, 64, 1, 1, 1),
    ("gen", 100, 100, 1, 1, 1),
    ("gen", 129, 70, 2, 3, 5),
    ("gen", 200, 200, 3, 5, 7),
    ("gen", 150, 300, 3, 5, 7),
    ("gen", 300, 150, 5, -4, 2),
    ("gen", 400, 300, 5, -4, 2),
    ("gen", 200, 200, 1, 1, -1),
    ("gen", 250, 250, 0, 0, 0),
]
WALK_TIMEOUT = 20


def make_walk():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    out = []
    for kind, a, b, m, k, d in WALK_CASES:
        s1, s2 = (a.encode(), b.encode()) if kind == "str" else (O.gen_dna(1, a), O.gen_dna(2, b))
        ops = [str(m), str(k), str(d)]
        try:
            p = subprocess.run(["needleman-wunsch", "-q", "-s", "--"] + ops, executable=REF_CLI,
                               input=s1 + b" " + s2 + b"\n", capture_output=True, timeout=WALK_TIMEOUT)
        except subprocess.TimeoutExpired:
            print("walk", kind, len(s1), len(s2), m, k, d, "reference walk too long, skipped", file=sys.stderr)
            continue
        err = p.stderr.decode().split("\n")
        count = int(err[0].split()[0]) & 0xFFFFFFFF      # printed with %d from an unsigned
        score = int(err[1].split()[-1])
        # first printed alignment: the first two stdout lines; stop the walk there
        q = subprocess.Popen(["needleman-wunsch", "--"] + ops, executable=REF_CLI, stdin=subprocess.PIPE,
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
        q.stdin.write(s1 + b" " + s2 + b"\n")
        q.stdin.close()
        top = q.stdout.readline().rstrip(b"\n")
        side = q.stdout.readline().rstrip(b"\n")
        q.kill()
        q.wait()
        case = {"kind": kind, "m": m, "k": k, "d": d, "L1": len(s1), "L2": len(s2), "count": count,
                "score": score, "first_top": top.decode(), "first_side": side.decode()}
        if kind == "str":
            case["s1"], case["s2"] = a, b
        out.append(case)
        print("walk", kind, len(s1), len(s2), m, k, d, count, score, file=sys.stderr)
    return out


def make_big_walk():
    """100k x 100k walk services: count and first path from the restatement
    (10 GB code table in host RAM; the oracle's walk is pinned to the reference
    by walk_kats.json)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    out = []
    for L1, L2, m, k, d in [(100000, 100000, 1, 1, 1)]:
        s1, s2 = O.gen_dna(1, L1), O.gen_dna(2, L2)
        D = np.empty((L1 + 1, L2 + 1), dtype=np.uint8)
        st = O.Stats()
        O.lib().nwo_fill(s1, L1, s2, L2, m, k, d, None, D.ctypes.data, ctypes.byref(st))
        count = O.count_paths(D)
        mv = O.first_path(D)
        del D
        out.append({"L1": L1, "L2": L2, "m": m, "k": k, "d": d, "corner": st.corner, "count": count,
                    "path_len": int(len(mv)), "path_fnv": "%016x" % O.fnv(mv),
                    "path_head": "".join("DUL"[[1, 2, 4].index(x)] for x in mv[:64].tolist()),
                    "path_tail": "".join("DUL"[[1, 2, 4].index(x)] for x in mv[-64:].tolist()),
                    "source": "oracle/libnworacle.so nwo_fill + nwo_count_paths + nwo_first_path "
                              "(restatement; transitive parity via walk_kats.json)"})
        print("big_walk", out[-1], file=sys.stderr)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--big-walk", action="store_true", help="only the 100k walk fixture (+ the fast ones)")
    ap.add_argument("--only-big", action="store_true", help="rewrite big_colchain.json alone")
    a = ap.parse_args()
    if a.only_big:
        with open(os.path.join(HERE, "big_colchain.json"), "w") as f:
            json.dump(make_big(), f, indent=1)
        return
    if not os.path.exists(HARNESS):
        sys.exit("build the reference first: make -C oracle ref")
    with open(os.path.join(HERE, "ref_kats.json"), "w") as f:
        json.dump(make_kats(), f, indent=0)
    with open(os.path.join(HERE, "cli_cases.json"), "w") as f:
        json.dump(make_cli(), f, indent=1, ensure_ascii=False)
    with open(os.path.join(HERE, "walk_kats.json"), "w") as f:
        json.dump(make_walk(), f, indent=0)
    if a.big:
        with open(os.path.join(HERE, "big_colchain.json"), "w") as f:
            json.dump(make_big(), f, indent=1)
    if a.big or a.big_walk:
        with open(os.path.join(HERE, "big_walk.json"), "w") as f:
            json.dump(make_big_walk(), f, indent=1)


if __name__ == "__main__":
    main()
