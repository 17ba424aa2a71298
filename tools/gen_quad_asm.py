#!/usr/bin/env python3
"""Generate needleman-wunsch_amd/csrc/nw_quad_chunk.inc: the hand-scheduled
8-step block of the one-row scan kernel with skewed 16-lane row groups
(nw_quad.hip).

    python tools/gen_quad_asm.py [--out PATH]

Lane l holds row l of a 64-row stripe; its DPP row q = l / 16 runs q columns
behind row 0.  Step s of a block (G' domain of nw_quad.hip; T_s = the row
above the stripe at row 0's column, from the ring):

    C   T_s   = v_mov_b32_dpp G_{s-1} row_bcast:15 row_mask:0xe    rows 1..3: the last lane of the
                                                                   row above (its column, one step ago)
    D   sh_s  = v_mov_b32_dpp G_{s-1} row_shr:1 INTO T_{s-1}       first lane of each row keeps T_{s-1},
                                                                   the same neighbour two steps ago
    A1  dg_s  = sh_s + sub'(s)                                     SDWA sext byte of the profile lookup
    A2  X_s   = max3(G_{s-1}, dg_s, T_s)
    S1..S4  G_s = prefix max of X_s inside the DPP row             4 x v_max_i32_dpp in place

Step 0 takes sh_0 and G_{-1} from the previous block (its tail runs D for
step 7).  Every DPP needs two instructions after the VALU that wrote its
source; those gaps take the previous step's work: its code (candidate - G' is
0 exactly for the candidates that attain the max, so the sign bit of one
v_sub is the inverted flag, shifted in with v_alignbit_b32), the ring write of
lane 63's G (the row above of the wave below, which is three columns behind
row 0: steps 0..2 finish the previous chunk's slot, whose progress counter is
published after step 2; steps 3..7 start this chunk's), and the chunk's LDS
traffic (cons, the next slot's {prog, cons}, 8 T and the chunk's symbols, the
symbols down the ring).  The block ends with lgkmcnt(K), K = the LDS ops
issued after its last read.

The symbols differ per row group: v_perm_b32 with a per-lane selector takes
this row group's window out of {this chunk's words, the previous chunk's}.

Template quad_chunk_asm<HH, FF, P>: HH = scores (the block's own G registers
are the outputs: the tiles hold G'), FF = direction codes, P = profile lookups
(symbols coded 0..7) instead of byte compares.
"""
import argparse
import os
import re

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_quad_chunk.inc")
READ_AT = 6            # step whose gaps issue the next slot's progress and data reads


def G(s):
    return "gc" if s in (-1, 7) else f"g{s}"


def T(s):
    return f"ta{s}" if s < 4 else f"tb{s - 4}"


def SH(s):
    """sh_s: step 0 takes the carried register, steps 1..7 shift into T_{s-1}; the tail into shc."""
    return "shc" if s in (0, 8) else T(s - 1)


def DG(s):
    return f"dg{s % 2}"


class It:
    def __init__(self, name, text, deps=(), lds=False):
        self.name, self.text, self.deps, self.lds = name, text, list(deps), lds


def sub_items(s, P):
    """dg_s = sh_s + sub'(s)."""
    if P:
        prof = "sub0" if s < 4 else "sub1"
        return [f"v_add_u32_sdwa %[{DG(s)}], %[{SH(s)}], sext(%[{prof}]) dst_sel:DWORD dst_unused:UNUSED_PAD "
                f"src0_sel:DWORD src1_sel:BYTE_{s % 4}"]
    w = "tq0" if s < 4 else "tq1"
    return [f"v_cmp_eq_u32_sdwa vcc, %[{w}], %[c2] src0_sel:BYTE_{s % 4} src1_sel:DWORD",
            "v_cndmask_b32_e64 %[sub], %[vck], %[vcm], vcc",
            f"v_add_u32_e32 %[{DG(s)}], %[{SH(s)}], %[sub]"]


def ring_item(c):
    """Lane 63's G of step c: column position c - 3 of this chunk's slot, or c + 5 of the previous one's."""
    if c >= 3:
        return It(f"R{c}", f"ds_write_b32 %[ra], %[{G(c)}] offset:{4 * (c - 3)}", lds=True)
    return It(f"R{c}", f"ds_write_b32 %[rap], %[{G(c)}] offset:{4 * (c + 5)}", lds=True)


def column_items(c, FF):
    """Code (FF) and ring write of step c (the up flag needs sh_{c+1}: dep 'D')."""
    its = [ring_item(c)]
    if c == 2:      # the previous chunk's slot is complete: the wave below may take it
        its.append(It("PV", "v_add_u32_e32 %[cvp], -1, %[cv]"))             # prog[w+1] = c: chunk c - 1 complete
        its.append(It("PW", "ds_write_b32 %[cb], %[cvp] offset:16", ["R2", "PV"], lds=True))
        its.append(It("CV", "v_add_u32_e32 %[cv], 1, %[cv]", ["PV", "CW"]))    # the next block's chunk
    if not FF:
        return its
    its.append(It(f"L{c}", f"v_sub_u32_e32 %[dL], %[{G(c - 1)}], %[{G(c)}]"))
    its.append(It(f"Dg{c}", f"v_sub_u32_e32 %[dD], %[{DG(c)}], %[{G(c)}]"))
    its.append(It(f"U{c}", f"v_sub_u32_e32 %[dU], %[{SH(c + 1)}], %[{G(c)}]", ["D"]))
    hi = "0" if c == 0 else "%[acc]"
    its.append(It(f"b1{c}", f"v_alignbit_b32 %[acc], {hi}, %[dL], 31", [f"L{c}"]))
    its.append(It(f"b2{c}", "v_alignbit_b32 %[acc], %[acc], %[dU], 31", [f"U{c}", f"b1{c}"]))
    its.append(It(f"b3{c}", "v_alignbit_b32 %[acc], %[acc], %[dD], 31", [f"Dg{c}", f"b2{c}"]))
    return its


def block(P, FF):
    out = []
    done = set()

    def emit(it):
        out.append(it)
        done.add(it.name)

    def take(pool, k):
        got = []
        for it in list(pool):
            if len(got) == k:
                break
            if all(d_ in done or d_ in [g.name for g in got] for d_ in it.deps):
                got.append(it)
                pool.remove(it)
        return got

    def gap(pool):
        got = take(pool, 2)
        for g in got:
            emit(g)
        if len(got) == 1:
            out.append(It("", "s_nop 0"))
        elif not got:
            out.append(It("", "s_nop 1"))

    mem = {0: [It("CW", "ds_write_b32 %[cb], %[cv] offset:4", lds=True),             # cons[w] = c + 1
               It("W8", "ds_write2_b32 %[ra], %[tc0], %[tc1] offset0:8 offset1:9", lds=True)],   # symbols down the ring
           READ_AT: [It("PQ", "ds_read_b64 %[pq], %[cb] offset:8", lds=True),        # {prog[w], cons[w+1]}
                     It("TA", "ds_read_b128 %[nA], %[rd]", lds=True)],
           READ_AT + 1: [It("TB", "ds_read_b128 %[nB], %[rd] offset:16", lds=True),
                         It("TC", "ds_read_b64 %[nC], %[rd] offset:32", lds=True)]}
    # head: this row group's symbol window, then the profile lookups
    out += [It("", "v_perm_b32 %[tq0], %[tc0], %[ptc1], %[selq]"),
            It("", "v_perm_b32 %[tq1], %[tc1], %[tc0], %[selq]")]
    if P:
        out += [It("", "v_perm_b32 %[sub0], %[ph], %[pl], %[tq0]"),
                It("", "v_perm_b32 %[sub1], %[ph], %[pl], %[tq1]")]
    for s in range(8):
        done.discard("D")
        pool = []
        if s > 0:
            pool += column_items(s - 1, FF)
        pool += mem.get(s, [])
        if s == 1:
            # the next block's window starts in this chunk's symbols 4..7: carried in
            # place (a copy between the blocks costs an instruction and a branch there)
            pool.append(It("PT", "v_mov_b32_e32 %[ptc1], %[tc1]"))
        if s > 0:
            gap(pool)                                                              # C, D read G_{s-1}
        emit(It("C", f"v_mov_b32_dpp %[{T(s)}], %[{G(s - 1)}] row_bcast:15 row_mask:0xe bank_mask:0xf"))
        if s > 0:
            emit(It("D", f"v_mov_b32_dpp %[{SH(s)}], %[{G(s - 1)}] row_shr:1 row_mask:0xf bank_mask:0xf"))
        else:
            done.add("D")
        for t in sub_items(s, P):
            emit(It("A1", t))
        emit(It("A2", f"v_max3_i32 %[{G(s)}], %[{G(s - 1)}], %[{DG(s)}], %[{T(s)}]"))
        g = G(s)
        for dp in ("row_shr:1", "row_shr:2", "row_shr:4", "row_shr:8"):
            gap(pool)
            emit(It("", f"v_max_i32_dpp %[{g}], %[{g}], %[{g}] {dp} row_mask:0xf bank_mask:0xf"))
        while pool:
            got = take(pool, 1)
            assert got, [p.name for p in pool]
            emit(got[0])
    # tail: sh_8 into the carried register (its first lanes keep T_7), then step 7's code and ring write
    done.discard("D")
    pool = [It("P", f"v_mov_b32_e32 %[shc], %[{T(7)}]")] + column_items(7, FF)
    pool = [p for p in pool if "D" not in p.deps] + [p for p in pool if "D" in p.deps]
    gap(pool)
    assert "P" in done
    emit(It("D", f"v_mov_b32_dpp %[shc], %[{G(7)}] row_shr:1 row_mask:0xf bank_mask:0xf"))
    while pool:
        got = take(pool, 1)
        assert got, [p.name for p in pool]
        emit(got[0])
    if FF:
        emit(It("", "v_xor_b32_e32 %[acc], 0xffffff, %[acc]"))              # flags were collected inverted
    lines = [it.text for it in out]
    last = max(i for i, x in enumerate(lines) if x.startswith("ds_read"))
    k = sum(1 for x in lines[last + 1:] if x.startswith("ds_"))
    lines.append(f"s_waitcnt lgkmcnt({min(k, 15)})")
    check(lines)
    return lines


def check(lines):
    """DPP sources: two wait states (instructions, or s_nop N = N + 1) after the
    VALU that wrote them."""
    def dst(x):
        if x.startswith(("ds_", "s_")):
            return None
        return x.split()[1].rstrip(",")

    def states(x):
        return int(x.split()[1]) + 1 if x.startswith("s_nop") else 1
    for i, x in enumerate(lines):
        if "_dpp" in x:
            src = x.split()[2].rstrip(",")
            ws = 0
            for j in range(i - 1, -1, -1):
                if dst(lines[j]) == src:
                    assert ws >= 2, (i, x, lines[j])
                    break
                ws += states(lines[j])
                if ws >= 2:
                    break


OPERANDS = r'''
    : [g0] "=&v"(r.h[0]), [g1] "=&v"(r.h[1]), [g2] "=&v"(r.h[2]), [g3] "=&v"(r.h[3]),
      [g4] "=&v"(r.h[4]), [g5] "=&v"(r.h[5]), [g6] "=&v"(r.h[6]), [gc] "+v"(r.g), [shc] "+v"(r.sh),
      [dg0] "=&v"(dg_[0]), [dg1] "=&v"(dg_[1]), [dL] "=&v"(t_[0]), [dU] "=&v"(t_[1]), [dD] "=&v"(t_[2]),
      [sub] "=&v"(t_[3]), [tq0] "=&v"(tq_[0]), [tq1] "=&v"(tq_[1]), [sub0] "=&v"(sp_[0]), [sub1] "=&v"(sp_[1]),
      [acc] "=&v"(r.acc), [ptc1] "+v"(r.ptc1), [cv] "+v"(r.cv), [cvp] "=&v"(t_[4]), [pq] "=&v"(r.pq), [nA] "=&v"(ns.a), [nB] "=&v"(ns.b), [nC] "=&v"(ns.c),
      [ta0] "+v"(ts.a[0]), [ta1] "+v"(ts.a[1]), [ta2] "+v"(ts.a[2]), [ta3] "+v"(ts.a[3]),
      [tb0] "+v"(ts.b[0]), [tb1] "+v"(ts.b[1]), [tb2] "+v"(ts.b[2]), [tb3] "+v"(ts.b[3])
    : [tc0] "v"(ts.c[0]), [tc1] "v"(ts.c[1]), [selq] "v"(k.selq),
      [c2] "v"(k.c2), [vcm] "v"(k.vcm), [vck] "v"(k.vck), [pl] "v"(k.pl), [ph] "v"(k.ph),
      [cb] "v"(k.cb), [ra] "v"(ra), [rap] "v"(rap), [rd] "v"(rd)
'''


def operands(text):
    """Only the operands the block names (an unbound early-clobber output would still take a VGPR)."""
    outs_txt, ins_txt = OPERANDS.split("    : [tc0]")
    ins_txt = "[tc0]" + ins_txt
    pat = re.compile(r'\[(\w+)\] "([^"]*)"\(([^()]*)\)')
    used = set(re.findall(r"%\[(\w+)\]", text))
    fmt = lambda lst: ", ".join(f'[{n}] "{c}"({e})' for n, c, e in lst if n in used)
    return f"        : {fmt(pat.findall(outs_txt))}\n        : {fmt(pat.findall(ins_txt))}\n"


def cstr(lines):
    return "\n".join(f'        "{ln}\\n\\t"' for ln in lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--read-at", type=int, default=READ_AT)
    args = ap.parse_args()
    globals()["READ_AT"] = args.read_at
    parts = ["// GENERATED by tools/gen_quad_asm.py -- do not edit; see the generator for the schedule.\n",
             "// r.cv: the block's chunk + 1 (counted on in the block); ra / rap: ring slot addresses of\n"
             "// that chunk and the one before; rd: the next slot.\n"
             "template <bool HH, bool FF, bool P>\n"
             "__device__ __forceinline__ void quad_chunk_asm(QuadRegs& r, const QuadConst& k, QuadSlot& ts,\n"
             "                                               QuadSlot& ns, int ra, int rap, int rd);\n"]
    decl = "    [[maybe_unused]] int dg_[2], t_[5];\n    [[maybe_unused]] uint32_t tq_[2], sp_[2];\n"
    tf = lambda b: "true" if b else "false"
    for HH in (1, 0):
        for FF in (1, 0):
            for P in (0, 1):
                lines = block(P, bool(FF))
                nvalu = sum(1 for x in lines if x.startswith("v_"))
                parts.append(f"// VALU quad_chunk_asm<{tf(HH)}, {tf(FF)}, {tf(P)}>: {nvalu} per 8 steps x 64 rows\n")
                parts.append(
                    f"template <> __device__ __forceinline__ void quad_chunk_asm<{tf(HH)}, {tf(FF)}, {tf(P)}>"
                    f"(QuadRegs& r, const QuadConst& k, QuadSlot& ts, QuadSlot& ns, int ra, int rap, int rd) {{\n"
                    f"{decl}    asm volatile(\n{cstr(lines)}\n{operands(chr(10).join(lines))}"
                    f"        : \"vcc\", \"memory\");\n}}\n")
    with open(args.out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
