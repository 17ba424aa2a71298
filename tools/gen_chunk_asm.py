#!/usr/bin/env python3
"""Generate needleman-wunsch_amd/csrc/nw_chunk.inc: the hand-scheduled
column steps of the fill kernel, one inline-asm block per 8-column chunk.

    python tools/gen_chunk_asm.py [--out PATH] [--read-step S]

Per column step s (G' = H + r*d + (i - base)*d, r = row in the workgroup,
i = column; see nw_fill.hip) the loop-carried chain is

    sh_s = wave_shr1(G'_{s-1}, lane 0 <- T'_{s-1})         v_mov_b32_dpp
    dg_s = sh_s + sub_s                                      v_add_u32
    X_s  = max3(G'_{s-1}, dg_s, T'_s)                        v_max3_i32
    G'_s = prefix max of X_s over the 64 lanes               6 x v_max_i32_dpp

Every DPP that reads a VGPR the previous VALU wrote needs two wait states
(7 gaps per step).  The gaps hold everything else the chunk does:
  * the direction code, score and |H| of column s-1 (the up flag needs sh_s,
    so that work trails by one step).  A code bit is the sign of
    (G' - 1) - candidate (every candidate is <= G'), shifted into the word by
    v_alignbit_b32 -- no compares, no SGPR masks;
  * sub' of column s+1 (of column 0 in the first gap): one SDWA byte compare
    of the chunk's top-string bytes against this lane's side-string byte and
    a v_cndmask;
  * all of the chunk's memory traffic.  G'_s of every lane goes to the LDS
    ring (only lane 63's address is the real slot; the other lanes write a
    dummy), H_s to the score tile (one coalesced 256-byte global_store_dword
    per column), the previous chunk's code word to the code tile; the ring
    counters (cons = this chunk taken, at the start; prog = the wave below
    may take it, after the last ring write) and the chunk's top-string bytes
    (which travel down the ring with T').  A chunk followed by another one
    also reads the next ring slot (producer progress first, then 8 T' and the
    2 words of top-string bytes) and the consumer's progress.
Memory items "float": they fill whatever gap slots the arithmetic leaves,
within a window of steps.  No scalar memory op is issued in the chunk loop, so
lgkmcnt is exact: the block's single wait is lgkmcnt(K) with K = the LDS ops
issued after its last read (the ledger in resolve_waits), never a wait for
the writes behind them.

Register roles are fixed so that nothing is copied between chunks: G'_6 and
G'_7 are written into the carried operands gp6 / gin, the code word of the
chunk grows in accp (the previous chunk's word is finished at step 0 and
copied to acc), tm takes T'_7 for the next chunk.  The caller alternates the
t / n (this / next ring slot) arrays.

One block = N steps (1..8).  NEXT: a chunk followed by another one (N = 8):
it reads the next slot, computes H of its own last column and advances the
carried offsets.  Otherwise the flush block finishes the last column's code
and score (the stripe's last column has no next step) and publishes it.

Templates: chunk_asm<SH, SD, ST, N, NEXT> / flush_asm<SH, SD, ST, N> with
SH = store scores, SD = direction codes, ST = stats (codes + |H| max).
"""
import argparse
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_chunk.inc")
READ_STEP = 2          # first step whose gaps may issue the next slot's reads
STORE = "normal"       # score stores: normal | fixed (diagnostic: one address)
STORE_HINT = "nt"      # cache-policy bits of the score stores (e.g. "nt", "sc1")
SCORE_X4 = True        # scores leave as 2 x global_store_dwordx4 per chunk from C++ (quad tiles)
CODE_HINT = "nt"       # cache-policy bits of the code-word stores
EXP_NO_BCAST = False   # timing-only experiment (wrong results): drop the two cross-row prefix levels


def gname(s):
    """Register of G'_s (s = -1, -2: the previous chunk's last two columns)."""
    return {-2: "gp6", -1: "gin", 6: "gp6", 7: "gin"}.get(s, f"g{s}")


SHIFT_INTO_T = True    # the DPP of step s writes into T'_{s-1}'s register (see shreg)


def shreg(s):
    """Register of sh_s = wave_shr1(G'_{s-1}) with T'_{s-1} in lane 0: the DPP
    leaves lane 0 (no source lane) at the register's old value.  Steps 1..7
    shift into T'_{s-1}'s own register (read for the last time by X_{s-1}'s
    max3), so lane 0 already holds T'_{s-1} and no pre-fill is needed (the T'
    operands are read-write); step 0 uses tm (the previous chunk's T'_7), and
    the flush of a full chunk's last column a rotating sh register with a
    pre-fill."""
    if s == 0:
        return "tm"
    if SHIFT_INTO_T and s <= 7:
        return f"t{s - 1}"
    return f"sh{s % 3}"


def dg_reg(s):
    return "dgA" if s % 2 == 0 else "dgB"


def sub_reg(s):
    return "subA" if s % 2 == 0 else "subB"


class Item:
    """One filler instruction: name, text, dependencies, needs sh_s, LDS op, step window."""

    def __init__(self, name, text, deps=(), needs_sh=False, lds=False, lo=0, hi=99):
        self.name, self.text, self.deps, self.needs_sh = name, text, list(deps), needs_sh
        self.lds, self.lo, self.hi = lds, lo, hi


def code_items(s, sh, SD):
    """Flags of column s-1 (sh = register holding wave_shr1 of G'_{s-1}) into its word.

    Every candidate X is <= G'_{s-1} (G' is their max), so X - G' is 0 for a
    candidate that attains the max and negative otherwise: the sign bit of one
    cheap v_sub is the INVERTED flag, shifted into the word by v_alignbit_b32
    (acc << 1 | d >> 31).  The word is inverted back once per chunk (MV).
    Neighbouring scores differ by a few |m|+|k|+|d|, so the subtraction cannot
    wrap.
    """
    Gp, Gpp, DGp = gname(s - 1), gname(s - 2), dg_reg(s - 1)
    hi = "0" if s == 1 else "%[accp]"      # first code of this chunk's word starts from 0
    items = [Item("L", f"v_sub_u32_e32 %[dL], %[{Gpp}], %[{Gp}]"),
             Item("D", f"v_sub_u32_e32 %[dD], %[{DGp}], %[{Gp}]"),
             Item("U", f"v_sub_u32_e32 %[dU], %[{sh}], %[{Gp}]", [], True),
             Item("b1", f"v_alignbit_b32 %[accp], {hi}, %[dL], 31", ["L"]),
             Item("b2", "v_alignbit_b32 %[accp], %[accp], %[dU], 31", ["U", "b1"], True),
             Item("b3", "v_alignbit_b32 %[accp], %[accp], %[dD], 31", ["D", "b2"], True)]
    if s == 0:                # the previous chunk's word is complete: hand it out (and store it)
        items.append(Item("MV", "v_xor_b32_e32 %[acc], 0xffffff, %[accp]", ["b3"], True))
        if SD:                # (chunk 0 stores its garbage word into the stripe's pad row)
            hint = f" {CODE_HINT}" if CODE_HINT else ""
            items.append(Item("CS", f"global_store_dword %[dv], %[acc], %[db]{hint}", ["MV"], True))
            items.append(Item("CV", "v_add_u32_e32 %[dv], 0x100, %[dv]", ["CS"], True))
    return items


def score_items(s, A, S):
    """H (and its store, and |H| max) of column s-1.  With SCORE_X4 the caller
    computes and stores H (16 bytes per lane per 4 columns); the block only
    needs H for the stats."""
    if SCORE_X4:
        S = False
        if not A:
            return []
    h = f"h{s - 1}"
    items = [Item("H", f"v_add3_u32 %[{h}], %[{gname(s - 1)}], %[nlo], %[k{s - 1}]")]
    if S:
        off = 0 if STORE == "fixed" else 256 * (s - 1)
        hint = (" " + STORE_HINT) if STORE_HINT else ""
        items.append(Item("ST", f"global_store_dword %[hv], %[{h}], %[hb] offset:{off}{hint}", ["H"]))
    if A:
        items.append(Item("A1", f"v_sub_u32_e32 %[tmp], 0, %[{h}]", ["H"]))
        items.append(Item("A2", f"v_max3_i32 %[gav], %[gav], %[{h}], %[tmp]", ["A1"]))
    return items


def ring_item(s):
    """G'_{s-1} of every lane to the ring (lane 63: the slot)."""
    return Item("R", f"ds_write_b32 %[ra], %[{gname(s - 1)}] offset:{4 * (s - 1)}", lds=True)


def sub_items(b):
    """sub' of column b of this chunk: byte compare of top-string byte b + select."""
    src, sel = ("t8", b) if b < 4 else ("t9", b - 4)
    return [Item("M", f"v_cmp_eq_u32_sdwa vcc, %[{src}], %[c2] src0_sel:BYTE_{sel} src1_sel:DWORD"),
            Item("X", f"v_cndmask_b32_e64 %[{sub_reg(b)}], %[vck], %[vcm], vcc", ["M"])]


def floating_items(N, nxt, P=False):
    """Memory items with a window of steps [lo, hi]; issued in list order.

    Ring counters: cb = &ctr[2w], ctr[2v+2] = prog[v] (chunks in wave v's ring),
    ctr[2v+3] = cons[v+1] (chunks wave v+1 took), so this wave's producer
    progress and consumer progress are one 8-byte pair at cb+8, its own cons at
    cb+4 and the prog of the wave below at cb+16.
    """
    last = N - 1
    its = [Item(f"SH{s}", f"v_mov_b32_e32 %[{shreg(s)}], %[t{s - 1}]", lo=max(s - 2, 0), hi=s - 1)
           for s in range(1, N) if shreg(s) != f"t{s - 1}"]
    if P and N > 4:                  # profile lookup of steps 4..7, before step 4
        its.append(Item("PB", "v_perm_b32 %[subB], %[ph], %[pl], %[t9]", hi=3))
    its += [Item("CW", "ds_write_b32 %[cb], %[cv] offset:4", lds=True, hi=last),  # ring slot taken
           Item("W8", "ds_write_b32 %[ra], %[t8] offset:32", lds=True, hi=last),  # top-string bytes
           Item("W9", "ds_write_b32 %[ra], %[t9] offset:36", lds=True, hi=last)]  # go down the ring
    if nxt:
        # the next chunk's slot: progress first (slot data read after a
        # progress value that covers it is valid), then T' and the bytes
        # (deadline step 5: the block's final wait finds them done)
        lo, hi = READ_STEP, min(READ_STEP + 3, last)
        its.append(Item("PQ", "ds_read_b64 %[pq], %[cb] offset:8", lds=True, lo=lo, hi=hi))
        its.append(Item("TA", "ds_read_b128 %[nA], %[rd]", lds=True, lo=lo, hi=hi))
        its.append(Item("TB", "ds_read_b128 %[nB], %[rd] offset:16", lds=True, lo=lo, hi=hi))
        its.append(Item("CC", "ds_read_b64 %[nC], %[rd] offset:32", lds=True, lo=lo, hi=hi))
        # tm (sh_0's register) is free after step 0: T'_7 for the next chunk
        its.append(Item("TM", "v_mov_b32_e32 %[tm], %[t7]", lo=1, hi=last))
    return its


def step(s, N, F, H, A, S, SD, nxt, floating, P=False):
    Gp = gname(s - 1)
    Tm = shreg(s)
    fill = []
    if s == 0:
        if P:                           # first gap: sub' bytes of steps 0..3 (profile lookup)
            fill.append(Item("PA", "v_perm_b32 %[subA], %[ph], %[pl], %[t8]"))
        else:
            fill += sub_items(0)        # first gap: sub' of this step itself
    if F:
        fill += code_items(s, Tm, SD)
    if s > 0:
        fill.append(ring_item(s))
    if H and s > 0:
        fill += score_items(s, A, S)
    if s + 1 < N and not P:
        fill += sub_items(s + 1)
    if P:                               # diagonal: sign-extended sub' byte of this step
        add = (f"v_add_u32_sdwa %[{dg_reg(s)}], %[{Tm}], sext(%[{'subA' if s < 4 else 'subB'}]) "
               f"dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_{s % 4}")
    else:
        add = f"v_add_u32_e32 %[{dg_reg(s)}], %[{Tm}], %[{sub_reg(s)}]"
    chain_head = [
        f"v_mov_b32_dpp %[{Tm}], %[{Gp}] wave_shr:1 row_mask:0xf bank_mask:0xf",
        add,
        f"v_max3_i32 %[{gname(s)}], %[{Gp}], %[{dg_reg(s)}], %[t{s}]",
    ]
    dpps = ["row_shr:1 row_mask:0xf", "row_shr:2 row_mask:0xf", "row_shr:4 row_mask:0xf",
            "row_shr:8 row_mask:0xf", "row_bcast:15 row_mask:0xa", "row_bcast:31 row_mask:0xc"]
    if EXP_NO_BCAST:
        dpps = dpps[:4]
    out = []
    done = set()
    pending = list(fill)

    def take(allow_sh, k=2):
        got = []
        names = lambda: [g.name for g in got]
        for it in list(pending):
            if len(got) == k:
                break
            if it.needs_sh and not allow_sh:
                continue
            if all(dd in done or dd in names() for dd in it.deps):
                got.append(it)
                pending.remove(it)
        while len(got) < k:               # earliest deadline first; reads keep their order
            ok = [f for f in floating if f.lo <= s]
            if not ok:
                break
            f = min(ok, key=lambda f: f.hi)
            floating.remove(f)
            got.append(f)
        for g in got:
            done.add(g.name)
        return got

    def gap(allow_sh):
        got = take(allow_sh)
        out.extend(got)
        if len(got) == 1:
            out.append(Item("", "s_nop 0"))
        elif not got:
            out.append(Item("", "s_nop 1"))

    gap(False)                     # before the DPP shift of G'_{s-1}
    out.extend(Item("", t) for t in chain_head)
    g = gname(s)
    for dp in dpps:
        gap(True)                  # before each DPP max reading the previous VALU result
        out.append(Item("", f"v_max_i32_dpp %[{g}], %[{g}], %[{g}] {dp} bank_mask:0xf"))
    while pending:                 # anything left runs after the scan
        got = take(True, 1)
        assert got, [p.name for p in pending]
        out.extend(got)
    for f in [f for f in floating if f.hi <= s]:
        floating.remove(f)
        out.append(f)
    return out


def resolve_waits(items):
    """Turn s_waitcnt lgkmcnt(@X) into the count of LDS ops issued after the LDS op X."""
    text = []
    for i, it in enumerate(items):
        t = it.text
        if "@" in t:
            tag = t[t.index("@") + 1:t.index(")")]
            pos = [j for j, x in enumerate(items[:i]) if x.name == tag and x.lds]
            assert pos, tag
            after = sum(1 for x in items[pos[-1] + 1:i] if x.lds)
            t = t.replace("@" + tag, str(min(after, 15)))
        text.append(t)
    return text


def block(N, F, H, A, S, SD, nxt, P=False):
    items = []
    if STORE == "fixed" and S and not SCORE_X4:     # diagnostic: every store to this lane's first word (hv = lane*4)
        items.append(Item("HF", "v_and_b32_e32 %[hv], 0xff, %[hv]"))
    floating = floating_items(N, nxt, P)
    for s in range(N):
        items += step(s, N, F, H, A, S, SD, nxt, floating, P)
    assert not floating, [f.name for f in floating]
    if nxt:                        # the chunk's last column (G'_7 is final now)
        items.append(ring_item(8))
        if H:
            items += score_items(8, A, S)
        items.append(Item("PW", "ds_write_b32 %[cb], %[cv] offset:16", lds=True))   # wave below may go
        items.append(Item("CA", "v_add_u32_e32 %[cv], 1, %[cv]"))
        if STORE != "fixed" and S and not SCORE_X4:
            items.append(Item("HA", "v_add_u32_e32 %[hv], 0x800, %[hv]"))
        items.append(Item("NA", "v_subrev_u32_e32 %[nlo], %[d8], %[nlo]"))
        last_read = [it.name for it in items if it.lds and it.text.startswith("ds_read")][-1]
        items.append(Item("WE", f"s_waitcnt lgkmcnt(@{last_read})"))   # progress and the next slot are in
    return resolve_waits(items)


def flush(N, F, H, A, S):
    """Code, ring entry and score of the block's last column s = N-1; then the wave below may go."""
    s = N
    out = [ring_item(s).text]
    if F:
        sh = shreg(s)
        items = {it.name: it.text for it in code_items(s, sh, False)}
        out += ([] if sh == f"t{s - 1}" else [f"v_mov_b32_e32 %[{sh}], %[t{s - 1}]"]) + [items["L"], items["D"],
                f"v_mov_b32_dpp %[{sh}], %[{gname(s - 1)}] wave_shr:1 row_mask:0xf bank_mask:0xf",
                items["U"], items["b1"], items["b2"], items["b3"],
                f"v_xor_b32_e32 %[accp], {hex((1 << 3 * N) - 1)}, %[accp]"]     # (flags were collected inverted)
    if H:
        out += [it.text for it in score_items(s, A, S)]
    out.append("ds_write_b32 %[cb], %[cv] offset:16")
    return out


OPERANDS = r'''
#define NW_CHUNK_OPERANDS                                                                                  \
    : [g0] "=&v"(r.g[0]), [g1] "=&v"(r.g[1]), [g2] "=&v"(r.g[2]), [g3] "=&v"(r.g[3]),                      \
      [g4] "=&v"(r.g[4]), [g5] "=&v"(r.g[5]), [gp6] "+v"(r.gp6), [gin] "+v"(r.gin),                       \
      [sh0] "=&v"(sh0_), [sh1] "=&v"(sh1_), [sh2] "=&v"(sh2_),                                             \
      [nA] "=&v"(ns.a), [nB] "=&v"(ns.b), [nC] "=&v"(ns.c), [pq] "=&v"(r.pq),                              \
      [tm] "+v"(r.tm), [dgA] "+v"(r.dgA), [dgB] "+v"(r.dgB), [subA] "+v"(r.subA), [subB] "+v"(r.subB),     \
      [h0] "=&v"(r.h[0]), [h1] "=&v"(r.h[1]), [h2] "=&v"(r.h[2]), [h3] "=&v"(r.h[3]),                      \
      [h4] "=&v"(r.h[4]), [h5] "=&v"(r.h[5]), [h6] "=&v"(r.h[6]), [h7] "=&v"(r.h[7]),                      \
      [accp] "+v"(r.accp), [acc] "=&v"(r.acc), [gav] "+v"(r.gav), [tmp] "=&v"(tmp_),                      \
      [dL] "=&v"(dL_), [dU] "=&v"(dU_), [dD] "=&v"(dD_),                                \
      [cv] "+v"(r.cv), [hv] "+v"(r.hv), [dv] "+v"(r.dv),         \
      [nlo] "+v"(r.nlo),                                                                                   \
      [t0] "+v"(ts.a[0]), [t1] "+v"(ts.a[1]), [t2] "+v"(ts.a[2]), [t3] "+v"(ts.a[3]),                      \
      [t4] "+v"(ts.b[0]), [t5] "+v"(ts.b[1]), [t6] "+v"(ts.b[2]), [t7] "+v"(ts.b[3])                       \
    : [t8] "v"(ts.c[0]),                                                                                   \
      [t9] "v"(ts.c[1]), [c2] "v"(k.c2), [vcm] "v"(k.vcm), [vck] "v"(k.vck), [d8] "s"(k.d8),                                \
      [k0] "v"(k.kd[0]), [k1] "v"(k.kd[1]), [k2] "v"(k.kd[2]), [k3] "v"(k.kd[3]),                          \
      [k4] "v"(k.kd[4]), [k5] "v"(k.kd[5]), [k6] "v"(k.kd[6]), [k7] "v"(k.kd[7]),                          \
      [ra] "v"(ra), [rd] "v"(rd), [cb] "v"(k.cb), [hb] "s"(k.hb), [db] "s"(k.db), [pl] "v"(k.pl),         \
      [ph] "v"(k.ph)
'''
# The flush reads values the chunk block produced: every value operand is read-write.
FLUSH_OPERANDS = (OPERANDS.replace("NW_CHUNK_OPERANDS", "NW_FLUSH_OPERANDS")
                  .replace('"=&v"(r.g', '"+v"(r.g').replace('"=&v"(r.h', '"+v"(r.h')
                  .replace('[acc] "=&v"', '[acc] "+v"'))


def cstr(lines):
    return "\n".join(f'        "{ln}\\n\\t"' for ln in lines)


def tf(b):
    return "true" if b else "false"


def main():
    global OUT, READ_STEP, STORE, STORE_HINT, SCORE_X4, CODE_HINT, EXP_NO_BCAST
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--read-step", type=int, default=READ_STEP)
    ap.add_argument("--store", choices=("normal", "fixed"), default=STORE)
    ap.add_argument("--store-hint", default=STORE_HINT)
    ap.add_argument("--x4", type=int, default=int(SCORE_X4))
    ap.add_argument("--code-hint", default=CODE_HINT)
    ap.add_argument("--exp-no-bcast", action="store_true")
    args = ap.parse_args()
    EXP_NO_BCAST = args.exp_no_bcast
    OUT, READ_STEP, STORE, STORE_HINT = args.out, args.read_step, args.store, args.store_hint
    SCORE_X4 = bool(args.x4)
    CODE_HINT = args.code_hint
    parts = ["// GENERATED by tools/gen_chunk_asm.py -- do not edit; see the generator for the schedule.\n",
             f"#define NW_SCORE_X4 {int(SCORE_X4)}\n#define NW_SCORE_HINT \"{(' ' + STORE_HINT) if STORE_HINT else ''}\"\n",
             OPERANDS, FLUSH_OPERANDS,
             "template <bool SH, bool SD, bool ST, bool P, int N, bool NEXT>\n"
             "__device__ __forceinline__ void chunk_asm(ChunkRegs& r, const ChunkConst& k, RingSlot& ts,\n"
             "                                          RingSlot& ns, int ra, int rd);\n"
             "template <bool SH, bool SD, bool ST, int N>\n"
             "__device__ __forceinline__ void flush_asm(ChunkRegs& r, const ChunkConst& k, RingSlot& ts, int ra);\n"]
    decl = "    int tmp_, dL_, dU_, dD_, sh0_, sh1_, sh2_;\n"
    unpack = ""
    for SH in (0, 1):
        for SD in (0, 1):
            for ST in (0, 1):
                F, H, A, S = SD or ST, SH or ST, ST, SH
                head = f"{tf(SH)}, {tf(SD)}, {tf(ST)}"
                for N in range(1, 9):
                    for nxt in ((0, 1) if N == 8 else (0,)):
                        for P in (0, 1):
                            parts.append(
                                f"template <> __device__ __forceinline__ void chunk_asm<{head}, {tf(P)}, {N}, {tf(nxt)}>"
                                f"(ChunkRegs& r, const ChunkConst& k, RingSlot& ts, RingSlot& ns, int ra, int rd) {{\n"
                                f"{decl}{unpack}    asm volatile(\n{cstr(block(N, F, H, A, S, SD, nxt, P))}\n"
                                f"        NW_CHUNK_OPERANDS : \"vcc\", \"scc\", \"memory\");\n}}\n")
                    parts.append(
                        f"template <> __device__ __forceinline__ void flush_asm<{head}, {N}>"
                        f"(ChunkRegs& r, const ChunkConst& k, RingSlot& ts, int ra) {{\n{decl}"
                        f"    RingSlot ns;\n    const int rd = 0;\n"
                        f"    asm volatile(\n{cstr(flush(N, F, H, A, S))}\n"
                        f"        NW_FLUSH_OPERANDS : \"vcc\", \"scc\", \"memory\");\n}}\n")
    parts.append("#undef NW_CHUNK_OPERANDS\n#undef NW_FLUSH_OPERANDS\n")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
