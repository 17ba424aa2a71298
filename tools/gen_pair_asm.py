#!/usr/bin/env python3
"""Generate needleman-wunsch_amd/csrc/nw_pair_chunk.inc: the hand-scheduled
8-column block of the two-rows-per-lane scan kernel (nw_pair.hip).

    python tools/gen_pair_asm.py [--out PATH]

Lane l holds rows a = 2l and b = 2l + 1 of a 128-row stripe.  Column step s
(G' domain of nw_pair.hip; sh_s = wave_shr1(Gb_{s-1}) with lane 0 = T_{s-1}):

    D   sh_s  = v_mov_b32_dpp Gb_{s-1} wave_shr:1   (lane 0 pre-filled with T_{s-1})
    F   Ga_{s-1} = max(Xa_{s-1}, sh_s)              (row a of the previous column is final)
    A1  dga_s = sh_s + sub'_a(s)                    (SDWA sext byte of the row-a profile)
    A3  dgb_s = Ga_{s-1} + sub'_b(s)
    A2  Xa_s  = max3(Ga_{s-1}, dga_s, T_s)
    A4  Xb_s  = max3(Gb_{s-1}, dgb_s, Xa_s)
    S1..S6  Gb_s = prefix max of Xb_s           (6 x v_max_i32_dpp in place)

Step 0 takes sh_0, Ga_{-1}, Gb_{-1} from the previous block (its tail runs D
and F for column 7).  Every DPP needs two instructions after the VALU that
wrote its source; those gaps take the previous column's work: its two code
words (a flag is v_cmp_eq_u32_e32 candidate, G' into VCC and
v_addc_co_u32_e32 acc = 2 acc + VCC -- two 4-byte encodings: a lone wave's
time follows the bytes of code it fetches, and a subtract plus v_alignbit_b32
is 12), its scores H = G' + nlo + kd, the ring write of lane 63's
Gb (the row above of the wave below), the lane-0 pre-fill of the next shift
and the chunk's LDS traffic (cons, the next slot's {prog, cons}, 8 T and the
chunk's symbols, the symbols down the ring, prog after the last ring write).
The block ends with lgkmcnt(K), K = the LDS ops issued after its last read.

pair_chunk_pipe<P> (raw scores + codes, the 100k x 100k fill) is software
pipelined across blocks: column 7's twelve flag instructions, the code words'
final xor and every table store would otherwise run after the block, outside
any DPP gap, while step 0's gaps (no previous column in this block) sit
empty.  So a block leaves column 7's candidates in carried registers and the
NEXT block finishes the previous block's code words in its step-0..3 gaps and
stores them together with the previous block's scores of columns 4..7; its
own scores of columns 0..3 go out in the gaps of steps 4..7.  The G'
registers of a row are fixed VGPRs (v80..v87 row a, v88..v95 row b) so that
four columns are one global_store_dwordx4 from inside the block; addresses
are an SGPR base plus a per-lane VGPR offset.  The caller flushes the last
block's pending half (nw_pair.hip).

Template pair_chunk_asm<HH, FF, ST, P>: HH = scores, FF = direction codes
(score-only fills skip both), ST = |H| max for the stats (rows a, b apart;
needs HH and FF), P = profile lookups (symbols coded 0..7) instead of byte
compares.
"""
import argparse
import os
import re

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_pair_chunk.inc")
READ_AT = 3            # step whose gaps issue the next slot's progress and data reads
ALIGN = None           # None, or the byte phase (0 / 4) mod 8 at which every block starts
# The DPP shift of column s writes into the register of T_{s-1} (the row
# above at column s-1, not needed after column s-1's max3): lanes >= 1 take
# the shifted Gb, lane 0 keeps T_{s-1} -- the value the shift must give it --
# so no per-column v_mov pre-fill of lane 0 (only the block's last, into the
# carried shc).  The T operands become read-write.
SHIFT_INTO_T = True
# Ring writes of lane 63's Gb in pairs of columns (ds_write2_b32 after the odd
# column) and the two symbol words in one ds_write2_b32: 11 LDS ops a block
# instead of 16.
RING2 = True
# Timing-only experiments (wrong results; never the product): drop the two
# cross-row prefix levels (row_bcast:15/31) and/or the score adds, to price
# the chain against the issue count on the GPU (GEN=... PAIR_ONLY=1 tools/ab_build.sh).
EXP_NO_BCAST = False
EXP_NO_SCORES = False
STORE_POLICY = "nt"    # cache policy of the pipelined block's table stores
EXP_FLAGS9 = False     # 9 flag instructions per column instead of 12 (drops row b's three shift-ins)
# pair_chunk_pipe: the fixed VGPRs of G' (row a columns 0..7, row b columns 0..7)
PIPE_REGS = {**{f"ga{s}": f"v{80 + s}" for s in range(7)}, "gac": "v87",
             **{f"gb{s}": f"v{88 + s}" for s in range(7)}, "gbc": "v95"}
PIPE_DEADLINE = 3      # step by whose end the previous block's deferred work is out


def GA(s):
    return "gac" if s in (-1, 7) else f"ga{s}"


def GB(s):
    return "gbc" if s in (-1, 7) else f"gb{s}"


def SH(s):
    if SHIFT_INTO_T and 1 <= s <= 7:
        return T(s - 1)      # the shift overwrites T_{s-1}, whose lane 0 it keeps
    return "shc" if s in (0, 8) else f"sh{s}"


def XA(s):
    return f"xa{s % 2}"


def DGA(s):
    return f"dga{s % 2}"


def DGB(s):
    return f"dgb{s % 2}"


def T(s):
    return f"ta{s}" if s < 4 else f"tb{s - 4}"


class It:
    """One schedulable item: one instruction, or two that must stay together
    (a compare into VCC and the add-with-carry that consumes it)."""
    def __init__(self, name, text, deps=(), lds=False, carry=False):
        self.name, self.text, self.deps, self.lds, self.carry = name, text, list(deps), lds, carry
        self.n = text.count("\n") + 1


def flag(name, acc, cand, g, deps=(), src=None, **kw):
    """acc = 2 * src + (cand == g): one direction flag shifted into a code word."""
    src = src or acc
    return It(name, f"v_cmp_eq_u32_e32 vcc, %[{cand}], %[{g}]\n"
                    f"v_addc_co_u32_e32 %[{acc}], vcc, %[{src}], %[{src}], vcc", deps, **kw)


def deferred_items():
    """pair_chunk_pipe, step 0: the previous block's column-7 flags (its G' of
    columns 6, 7 are still in the fixed registers, its dg and shift in carried
    operands), code words and stores of columns 4..7."""
    C = dict(carry=True)
    return [flag("qB1", "tB", "gb6", "gbc", src="pB", **C),
            flag("qA1", "tA", "ga6", "gac", src="pA", **C),
            It("sQb1", "global_store_dwordx4 %[vob], v[92:95], %[hbp] offset:1024 nt", **C),
            It("sQa1", "global_store_dwordx4 %[voa], v[84:87], %[hbp] offset:1024 nt", **C),
            flag("qB2", "tB", "gac", "gbc", ["qB1"], **C),
            flag("qA2", "tA", "shc", "gac", ["qA1"], **C),
            flag("qB3", "tB", "pdgb", "gbc", ["qB2"], **C),
            flag("qA3", "tA", "pdga", "gac", ["qA2"], **C),
            It("stA", "global_store_dword %[vda], %[tA], %[dbp] nt", ["qA3"], **C),
            It("stB", "global_store_dword %[vdb], %[tB], %[dbp] nt", ["qB3"], **C)]


def sub_items(s, P, row):
    """dg of row a (from sh_s) or b (from Ga_{s-1}) at step s."""
    if row == "a":
        dst, src, prof = DGA(s), SH(s), ("subA0" if s < 4 else "subA1")
    else:
        dst, src, prof = DGB(s), GA(s - 1), ("subB0" if s < 4 else "subB1")
    if P:
        return [f"v_add_u32_sdwa %[{dst}], %[{src}], sext(%[{prof}]) dst_sel:DWORD dst_unused:UNUSED_PAD "
                f"src0_sel:DWORD src1_sel:BYTE_{s % 4}"]
    w = "tc0" if s < 4 else "tc1"
    c2 = "c2a" if row == "a" else "c2b"
    return [f"v_cmp_eq_u32_sdwa vcc, %[{w}], %[{c2}] src0_sel:BYTE_{s % 4} src1_sel:DWORD",
            "v_cndmask_b32_e64 %[sub], %[vck], %[vcm], vcc",
            f"v_add_u32_e32 %[{dst}], %[{src}], %[sub]"]


def ring_items(c):
    """Ring write of lane 63's Gb at column c (the row above of the wave below)."""
    if not RING2:
        return [It("R", f"ds_write_b32 %[ra], %[{GB(c)}] offset:{4 * c}", lds=True)]
    if c % 2 == 0:
        return []
    return [It("R", f"ds_write2_b32 %[ra], %[{GB(c - 1)}], %[{GB(c)}] offset0:{c - 1} offset1:{c}", lds=True)]


def column_items(c, ST, HH=True, FF=True):
    """Codes (FF), scores (HH), ring write of column c (needs Ga_c final: dep 'F')."""
    its = ring_items(c)
    if not HH and not FF:
        return its
    if EXP_NO_SCORES:
        HH, ST = False, False
    if not FF:
        return its + [It("Hb", f"v_add3_u32 %[hb{c}], %[{GB(c)}], %[nlob], %[kd{c}]"),
                      It("Ha", f"v_add3_u32 %[ha{c}], %[{GA(c)}], %[nloa], %[kd{c}]", ["F"])]
    its = []
    n = lambda x: f"{x}{c}"      # (a dependency must not be met by an earlier column's item)
    # row b's left flag needs no F (row a's final max); the code of a column
    # is left, up, diag from the top: shifted in in that order
    its.append(flag(n("Lb"), "accB", GB(c - 1), GB(c)))
    if HH:
        its.append(It("Hb", f"v_add3_u32 %[hb{c}], %[{GB(c)}], %[nlob], %[kd{c}]"))
    its += ring_items(c)
    its.append(flag(n("La"), "accA", GA(c - 1), GA(c), ["F"]))
    its.append(flag(n("Ub"), "accB", GA(c), GB(c), ["F", n("Lb")]))
    its.append(flag(n("Ua"), "accA", SH(c + 1), GA(c), ["F", n("La")]))
    its.append(flag(n("Db"), "accB", DGB(c), GB(c), [n("Ub")]))
    its.append(flag(n("Da"), "accA", DGA(c), GA(c), ["F", n("Ua")]))
    if HH:
        its.append(It("Ha", f"v_add3_u32 %[ha{c}], %[{GA(c)}], %[nloa], %[kd{c}]", ["F"]))
    if EXP_FLAGS9:
        its = [it for it in its if it.name not in (n("Lb"), n("Ub"), n("Db"))]
    if ST:
        its.append(It("Za", f"v_sub_u32_e32 %[tmp], 0, %[ha{c}]", ["Ha"]))
        its.append(It("Ma", f"v_max3_i32 %[gavA], %[gavA], %[ha{c}], %[tmp]", ["Za"]))
        its.append(It("Zb", f"v_sub_u32_e32 %[tmp], 0, %[hb{c}]", ["Hb", "Ma"]))
        its.append(It("Mb", f"v_max3_i32 %[gavB], %[gavB], %[hb{c}], %[tmp]", ["Zb"]))
    return its


def block(ST, P, HH=True, FF=True, pipe=False):
    out = []          # list of It
    done = set()
    carried = []      # pipe: items that may move on into the next step's gaps

    def emit(it):
        out.append(it)
        done.add(it.name)

    def take(pool, k, ready, slots=99):
        """Up to k ready items of the pool, in its order, of at most `slots`
        instructions together."""
        got = []
        for it in list(pool):
            if len(got) == k or slots == 0:
                break
            if it.n <= slots and all(d_ in done or d_ in ready or d_ in [g.name for g in got] for d_ in it.deps):
                got.append(it)
                slots -= it.n
                pool.remove(it)
        return got

    def gap(pool, ready=()):
        """The two wait states before a DPP instruction."""
        got = take(pool, 2, ready, slots=2)
        for g in got:
            emit(g)
        n = sum(g.n for g in got)
        if n == 1:
            out.append(It("", "s_nop 0"))
        elif n == 0:
            out.append(It("", "s_nop 1"))

    sym = ([It("W8", "ds_write2_b32 %[ra], %[tc0], %[tc1] offset0:8 offset1:9", lds=True)] if RING2 else
           [It("W8", "ds_write_b32 %[ra], %[tc0] offset:32", lds=True),             # symbols down the ring
            It("W9", "ds_write_b32 %[ra], %[tc1] offset:36", lds=True)])
    mem = {0: [It("CW", "ds_write_b32 %[cb], %[cv] offset:4", lds=True)] + sym,      # cons[w] = c+1
           # (READ_AT: how late in the block the next slot is read; the
           # producer runs one chunk ahead, so an early read usually misses it
           # and the caller takes the slow re-read)
           }
    reads = [It("PQ", "ds_read_b64 %[pq], %[cb] offset:8", lds=True),       # {prog[w], cons[w+1]}
             It("TA", "ds_read_b128 %[nA], %[rd]", lds=True),
             It("TB", "ds_read_b128 %[nB], %[rd] offset:16", lds=True),
             It("TC", "ds_read_b64 %[nC], %[rd] offset:32", lds=True)]
    # READ_AT <= 6: two reads in that step's gaps, two in the next step's;
    # 7: all four in step 7's; 8: all four in the tail (after column 7's shift)
    if READ_AT <= 6:
        mem.setdefault(READ_AT, []).extend(reads[:2])
        mem.setdefault(READ_AT + 1, []).extend(reads[2:])
    elif READ_AT == 7:
        mem.setdefault(7, []).extend(reads)
    # head: profile lookups of the chunk, pre-fill of sh_1
    if P:
        out += [It("", "v_perm_b32 %[subA0], %[pha], %[pla], %[tc0]"),
                It("", "v_perm_b32 %[subA1], %[pha], %[pla], %[tc1]"),
                It("", "v_perm_b32 %[subB0], %[phb], %[plb], %[tc0]"),
                It("", "v_perm_b32 %[subB1], %[phb], %[plb], %[tc1]")]
    if FF:
        out += [It("", "v_mov_b32_e32 %[accA], 0"), It("", "v_mov_b32_e32 %[accB], 0")]
    for s in range(8):
        done.discard("F")
        pool = []
        if s > 0:
            pool += column_items(s - 1, ST, HH, FF)
        if not SHIFT_INTO_T or s == 7:
            pool.append(It("P", f"v_mov_b32_e32 %[{SH(s + 1)}], %[{T(s)}]"))        # lane 0's next shift
        pool += mem.get(s, [])
        if pipe:
            if s == 0:
                carried = deferred_items()
            if s == 4:
                # this block's scores of columns 0..3: row b is final after step
                # 3's scan, row a after step 4's F
                carried += [It("sQb0", "global_store_dwordx4 %[vob], v[88:91], %[hbs] nt", carry=True),
                            It("sQa0", "global_store_dwordx4 %[voa], v[80:83], %[hbs] nt", ["F"], carry=True)]
            pool += carried
        chain = []
        if s > 0:
            gap(pool)                                                              # D reads Gb_{s-1}
            emit(It("D", f"v_mov_b32_dpp %[{SH(s)}], %[{GB(s - 1)}] wave_shr:1 row_mask:0xf bank_mask:0xf"))
        for t in sub_items(s, P, "a"):
            emit(It("A1", t))
        if s > 0:
            emit(It("F", f"v_max_i32_e32 %[{GA(s - 1)}], %[{XA(s - 1)}], %[{SH(s)}]"))
        else:
            done.add("F")
        for t in sub_items(s, P, "b"):
            emit(It("A3", t))
        emit(It("A2", f"v_max3_i32 %[{XA(s)}], %[{GA(s - 1)}], %[{DGA(s)}], %[{T(s)}]"))
        emit(It("A4", f"v_max3_i32 %[{GB(s)}], %[{GB(s - 1)}], %[{DGB(s)}], %[{XA(s)}]"))
        dpps = ["row_shr:1 row_mask:0xf", "row_shr:2 row_mask:0xf", "row_shr:4 row_mask:0xf",
                "row_shr:8 row_mask:0xf", "row_bcast:15 row_mask:0xa", "row_bcast:31 row_mask:0xc"]
        if EXP_NO_BCAST:
            dpps = dpps[:4]
        g = GB(s)
        for dp in dpps:
            gap(pool)
            emit(It("", f"v_max_i32_dpp %[{g}], %[{g}], %[{g}] {dp} bank_mask:0xf"))
        carried = [it for it in pool if it.carry and not (pipe and s == PIPE_DEADLINE)]
        pool = [it for it in pool if it not in carried]
        while pool:
            got = take(pool, 1, ())
            assert got, [p.name for p in pool]
            emit(got[0])
    # tail: D and F of column 7, its codes / scores / ring write, then prog
    done.discard("F")
    pool = (ring_items(7) + carried) if pipe else column_items(7, ST, HH, FF)
    if READ_AT >= 8:
        pool = reads + pool
    gap(pool)
    emit(It("D", f"v_mov_b32_dpp %[{SH(8)}], %[{GB(7)}] wave_shr:1 row_mask:0xf bank_mask:0xf"))
    emit(It("F", f"v_max_i32_e32 %[{GA(7)}], %[{XA(7)}], %[{SH(8)}]"))
    while pool:
        got = take(pool, 1, ())
        assert got, [p.name for p in pool]
        emit(got[0])
    emit(It("PW", "ds_write_b32 %[cb], %[cv] offset:16", lds=True))         # prog[w+1] = c+1
    lines = [ln for it in out for ln in it.text.split("\n")]
    if pipe and STORE_POLICY != "nt":
        lines = [re.sub(r" nt$", (" " + STORE_POLICY).rstrip(), ln) if ln.startswith("global_store") else ln
                 for ln in lines]
    if pipe:
        lines = [re.sub(r"%\[(\w+)\]", lambda m: PIPE_REGS.get(m.group(1), m.group(0)), ln) for ln in lines]
    if ALIGN is not None:
        # start the block at a fixed place in a 64-byte line (MI355X_MICROARCH.md,
        # "Code-placement sensitivity"), jumping over the padding: the block's
        # own layout no longer depends on the compiler's code around it
        lines = ["s_branch 1f", ".p2align 6", "1:"] + (["s_nop 0"] if ALIGN == 4 else []) + lines
    last = max(i for i, x in enumerate(lines) if x.startswith("ds_read"))
    k = sum(1 for x in lines[last + 1:] if x.startswith("ds_"))
    lines.append(f"s_waitcnt lgkmcnt({min(k, 15)})")
    check(lines)
    return lines


def check(lines):
    """DPP sources: two wait states (instructions, or s_nop N = N + 1) after the
    VALU that wrote them."""
    def dst(x):
        if x.startswith(("ds_", "s_", "global_")):
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
#define NW_PAIR_OPERANDS                                                                                   \
    : [ga0] "=&v"(ga_[0]), [ga1] "=&v"(ga_[1]), [ga2] "=&v"(ga_[2]), [ga3] "=&v"(ga_[3]),                  \
      [ga4] "=&v"(ga_[4]), [ga5] "=&v"(ga_[5]), [ga6] "=&v"(ga_[6]), [gac] "+v"(r.ga),                     \
      [gb0] "=&v"(gb_[0]), [gb1] "=&v"(gb_[1]), [gb2] "=&v"(gb_[2]), [gb3] "=&v"(gb_[3]),                  \
      [gb4] "=&v"(gb_[4]), [gb5] "=&v"(gb_[5]), [gb6] "=&v"(gb_[6]), [gbc] "+v"(r.gb),                     \
      [sh1] "=&v"(sh_[1]), [sh2] "=&v"(sh_[2]), [sh3] "=&v"(sh_[3]), [sh4] "=&v"(sh_[4]),                  \
      [sh5] "=&v"(sh_[5]), [sh6] "=&v"(sh_[6]), [sh7] "=&v"(sh_[7]), [shc] "+v"(r.sh),                     \
      [xa0] "=&v"(xa_[0]), [xa1] "=&v"(xa_[1]), [dga0] "=&v"(dga_[0]), [dga1] "=&v"(dga_[1]),              \
      [dgb0] "=&v"(dgb_[0]), [dgb1] "=&v"(dgb_[1]),                                                        \
      [dLa] "=&v"(t_[0]), [dUa] "=&v"(t_[1]), [dDa] "=&v"(t_[2]), [dLb] "=&v"(t_[3]), [dUb] "=&v"(t_[4]),   \
      [dDb] "=&v"(t_[5]), [tmp] "=&v"(t_[6]), [sub] "=&v"(t_[7]),                                          \
      [subA0] "=&v"(sp_[0]), [subA1] "=&v"(sp_[1]), [subB0] "=&v"(sp_[2]), [subB1] "=&v"(sp_[3]),          \
      [ha0] "=&v"(r.ha[0]), [ha1] "=&v"(r.ha[1]), [ha2] "=&v"(r.ha[2]), [ha3] "=&v"(r.ha[3]),              \
      [ha4] "=&v"(r.ha[4]), [ha5] "=&v"(r.ha[5]), [ha6] "=&v"(r.ha[6]), [ha7] "=&v"(r.ha[7]),              \
      [hb0] "=&v"(r.hb[0]), [hb1] "=&v"(r.hb[1]), [hb2] "=&v"(r.hb[2]), [hb3] "=&v"(r.hb[3]),              \
      [hb4] "=&v"(r.hb[4]), [hb5] "=&v"(r.hb[5]), [hb6] "=&v"(r.hb[6]), [hb7] "=&v"(r.hb[7]),              \
      [accA] "=&v"(r.accA), [accB] "=&v"(r.accB), [gavA] "+v"(r.gavA), [gavB] "+v"(r.gavB),                 \
      [pq] "=&v"(r.pq), [nA] "=&v"(ns.a), [nB] "=&v"(ns.b), [nC] "=&v"(ns.c),                              \
      [ta0] "+v"(ts.a[0]), [ta1] "+v"(ts.a[1]), [ta2] "+v"(ts.a[2]), [ta3] "+v"(ts.a[3]),                  \
      [tb0] "+v"(ts.b[0]), [tb1] "+v"(ts.b[1]), [tb2] "+v"(ts.b[2]), [tb3] "+v"(ts.b[3])                   \
    : [tc0] "v"(ts.c[0]), [tc1] "v"(ts.c[1]),                                                              \
      [kd0] "v"(k.kd[0]), [kd1] "v"(k.kd[1]), [kd2] "v"(k.kd[2]), [kd3] "v"(k.kd[3]),                      \
      [kd4] "v"(k.kd[4]), [kd5] "v"(k.kd[5]), [kd6] "v"(k.kd[6]), [kd7] "v"(k.kd[7]),                      \
      [nloa] "v"(r.nloa), [nlob] "v"(r.nlob), [c2a] "v"(k.c2a), [c2b] "v"(k.c2b), [vcm] "v"(k.vcm),         \
      [vck] "v"(k.vck), [pla] "v"(k.pla), [pha] "v"(k.pha), [plb] "v"(k.plb), [phb] "v"(k.phb),             \
      [cb] "v"(k.cb), [cv] "v"(cv), [ra] "v"(ra), [rd] "v"(rd)
'''


def operands(text):
    """The operand lists of one block: only the NW_PAIR_OPERANDS entries its
    text names (an unbound early-clobber output would still take a VGPR --
    about 30 in the score-only block)."""
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
    ap.add_argument("--align", type=int, choices=(0, 4), default=ALIGN)
    ap.add_argument("--exp-no-bcast", action="store_true")
    ap.add_argument("--exp-no-scores", action="store_true")
    ap.add_argument("--exp-flags9", action="store_true")
    ap.add_argument("--store-policy", default="nt", help="cache policy suffix of the pipelined block's table stores "
                    "(nt | sc1 | sc0+sc1 | none); anything but nt is a timing experiment")
    args = ap.parse_args()
    globals()["EXP_NO_BCAST"] = args.exp_no_bcast
    globals()["EXP_NO_SCORES"] = args.exp_no_scores
    globals()["EXP_FLAGS9"] = args.exp_flags9
    globals()["STORE_POLICY"] = "" if args.store_policy == "none" else args.store_policy.replace("+", " ")
    globals()["READ_AT"] = args.read_at
    globals()["ALIGN"] = args.align
    parts = ["// GENERATED by tools/gen_pair_asm.py -- do not edit; see the generator for the schedule.\n",
             "template <bool HH, bool FF, bool ST, bool P>\n"
             "__device__ __forceinline__ void pair_chunk_asm(PairRegs& r, const PairConst& k, PairSlot& ts,\n"
             "                                               PairSlot& ns, int cv, int ra, int rd);\n"]
    decl = "    [[maybe_unused]] int ga_[7], gb_[7], sh_[8], xa_[2], dga_[2], dgb_[2], t_[8], sp_[4];\n"
    tf = lambda b: "true" if b else "false"
    for HH, FF, ST in ((1, 1, 1), (1, 1, 0), (1, 0, 0), (0, 1, 0), (0, 0, 0)):
        for P in (0, 1):
            lines = block(ST, P, HH, FF)
            nvalu = sum(1 for x in lines if x.startswith("v_"))
            parts.append(f"// VALU pair_chunk_asm<{tf(HH)}, {tf(FF)}, {tf(ST)}, {tf(P)}>: {nvalu} per 8 columns x 128 rows\n")
            parts.append(
                f"template <> __device__ __forceinline__ void pair_chunk_asm<{tf(HH)}, {tf(FF)}, {tf(ST)}, {tf(P)}>"
                f"(PairRegs& r, const PairConst& k, PairSlot& ts, PairSlot& ns, int cv, int ra, int rd) {{\n"
                f"{decl}    asm volatile(\n{cstr(lines)}\n{operands(chr(10).join(lines))}"
                f"        : \"vcc\", \"memory\");\n}}\n")
    # Raw-score blocks (nw_pair.hip, fills with scores and without stats): no
    # H = G' + nlo + kd adds; the block's own G' registers of columns 0..6 are
    # the score outputs (r.ha / r.hb; column 7 is r.ga / r.gb), and the
    # readers add the affine offset back (nwk::raw_offset).
    parts.append("template <bool FF, bool P>\n"
                 "__device__ __forceinline__ void pair_chunk_raw(PairRegs& r, const PairConst& k, PairSlot& ts,\n"
                 "                                               PairSlot& ns, int cv, int ra, int rd);\n")
    for FF in (1, 0):
        for P in (0, 1):
            lines = block(0, P, False, bool(FF))
            nvalu = sum(1 for x in lines if x.startswith("v_"))
            ops = operands(chr(10).join(lines))
            for q in range(7):
                ops = ops.replace(f"(ga_[{q}])", f"(r.ha[{q}])").replace(f"(gb_[{q}])", f"(r.hb[{q}])")
            parts.append(f"// VALU pair_chunk_raw<{tf(FF)}, {tf(P)}>: {nvalu} per 8 columns x 128 rows\n")
            parts.append(
                f"template <> __device__ __forceinline__ void pair_chunk_raw<{tf(FF)}, {tf(P)}>"
                f"(PairRegs& r, const PairConst& k, PairSlot& ts, PairSlot& ns, int cv, int ra, int rd) {{\n"
                f"{decl}    asm volatile(\n{cstr(lines)}\n{ops}"
                f"        : \"vcc\", \"memory\");\n}}\n")
    # The pipelined raw block (scores + codes): see the module docstring.
    parts.append("template <bool P>\n"
                 "__device__ __forceinline__ void pair_chunk_pipe(PairRegs& r, const PairConst& k, PairSlot& ts,\n"
                 "                                                PairSlot& ns, int cv, int ra, int rd, int voa, int vob,\n"
                 "                                                int vda, int vdb, const int32_t* hbs, const int32_t* hbp,\n"
                 "                                                const uint32_t* dbp);\n")
    for P in (0, 1):
        lines = block(0, P, False, True, pipe=True)
        nvalu = sum(1 for x in lines if x.startswith("v_"))
        ops = operands(chr(10).join(lines))
        ops = ops.replace("(dga_[1])", "(r.dga1)").replace("(dgb_[1])", "(r.dgb1)")
        outs, ins = ops.rstrip("\n").split("\n")
        outs += (', [pLa] "=&v"(p_[0]), [pUa] "=&v"(p_[1]), [pDa] "=&v"(p_[2]), [pLb] "=&v"(p_[3]), '
                 '[pUb] "=&v"(p_[4]), [pDb] "=&v"(p_[5]), [tA] "=&v"(p_[6]), [tB] "=&v"(p_[7]), '
                 '[qa1] "+{v[84:87]}"(r.qa1), [qb1] "+{v[92:95]}"(r.qb1)')
        ins += (', [pdga] "v"(r.dga1), [pdgb] "v"(r.dgb1), [pA] "v"(r.accA), [pB] "v"(r.accB), [voa] "v"(voa), '
                '[vob] "v"(vob), [vda] "v"(vda), [vdb] "v"(vdb), [hbs] "s"(hbs), [hbp] "s"(hbp), [dbp] "s"(dbp)')
        clob = ", ".join(f'"v{n}"' for n in list(range(80, 84)) + list(range(88, 92)))
        parts.append(f"// VALU pair_chunk_pipe<{tf(P)}>: {nvalu} per 8 columns x 128 rows\n")
        parts.append(
            f"template <> __device__ __forceinline__ void pair_chunk_pipe<{tf(P)}>"
            f"(PairRegs& r, const PairConst& k, PairSlot& ts, PairSlot& ns, int cv, int ra, int rd, int voa, int vob,\n"
            f"        int vda, int vdb, const int32_t* hbs, const int32_t* hbp, const uint32_t* dbp) {{\n"
            f"{decl}    [[maybe_unused]] int p_[8];\n    asm volatile(\n{cstr(lines)}\n{outs}\n{ins}\n"
            f"        : \"vcc\", \"memory\", {clob});\n}}\n")
    with open(args.out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
