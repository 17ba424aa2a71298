#!/usr/bin/env python3
"""Generate needleman-wunsch_amd/csrc/nw_chunk.inc: the hand-scheduled
column steps of the fill kernel, one inline-asm block per chunk.

    python tools/gen_chunk_asm.py            (rewrites the .inc)

Per column step s (G' = H + r*d + (i - base)*d, r = row in the workgroup,
i = column; see nw_fill.hip) the loop-carried chain is

    sh_s = wave_shr1(G'_{s-1}, lane 0 <- T'_{s-1})         v_mov_b32_dpp
    dg_s = sh_s + sub_s                                      v_add_u32
    X_s  = max3(G'_{s-1}, dg_s, T'_s)                        v_max3_i32
    G'_s = prefix max of X_s over the 64 lanes               6 x v_max_i32_dpp

Every DPP that reads a VGPR the previous VALU wrote needs two wait states
(7 gaps per step).  The gaps hold the step's other work instead of s_nop:
the direction code, score and |H| of step s-1 (the up flag needs sh_s, so
that work trails by one step) and the substitution score of step s+1.  The
3-bit code of a cell is shifted into a per-lane word with v_addc
(acc = 2*acc + flag: left, up, diag; see code_items), so 8 codes fill
bits 0..23.

Register roles are fixed so that nothing is copied between chunks: G'_6 and
G'_7 are written into the carried operands gp6 / gin, the code word of the
chunk grows in accp (the previous chunk's word is finished at step 0 and
copied to acc), tm takes T'_7 for the next chunk.

One block = N steps (1..8).  NEXT: a chunk followed by another one (N = 8):
it also prepares sub for the next chunk's step 0 and computes H of its own
last column.  Otherwise the flush block finishes the last column's code and
score (the stripe's last column has no next step).

The block also does the chunk's memory traffic in the gaps: G'_s of every
lane goes to the LDS ring (only lane 63's address is the real slot; the
others write a dummy) and H_s to the score tile, one coalesced 256-byte
global_store_dword per column (column-major stripe tiles).  Nothing waits
on these inside the block; the caller's lgkmcnt/vmcnt waits cover them.

Templates: chunk_asm<SH, SD, ST, N, NEXT> / flush_asm<SH, SD, ST, N> with
SH = store scores, SD = direction codes, ST = stats (codes + |H| max).
"""
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_chunk.inc")


def gname(s):
    """Register of G'_s (s = -1, -2: the previous chunk's last two columns)."""
    return {-2: "gp6", -1: "gin", 6: "gp6", 7: "gin"}.get(s, f"g{s}")


def dg_reg(s):
    return "dgA" if s % 2 == 0 else "dgB"


def sub_reg(s):
    return "subA" if s % 2 == 0 else "subB"


def byte_src(s):
    """(sgpr operand, bfe offset) of the character of step s (s == 8: next chunk's byte 0)."""
    if s == 8:
        return "chn", 0
    return ("chlo", 8 * s) if s < 4 else ("chhi", 8 * (s - 4))


CODES = "align"    # or "cmp" (v_cmp + v_addc, the previous scheme; A/B runs)


def code_items_cmp(s, sh):
    """Flags of column s-1 via v_cmp -> SGPR mask -> v_addc shift-in (A/B reference)."""
    Gp, Gpp, DGp = gname(s - 1), gname(s - 2), dg_reg(s - 1)
    fresh = "0, 0" if s == 1 else "%[accp], %[accp]"
    items = [("L", f"v_cmp_eq_i32_e64 %[sL], %[{Gp}], %[{Gpp}]", [], False),
             ("D", f"v_cmp_eq_i32_e64 %[sD], %[{Gp}], %[{DGp}]", [], False),
             ("U", f"v_cmp_eq_i32_e64 %[sU], %[{Gp}], %[{sh}]", [], True),
             ("b1", f"v_addc_co_u32_e64 %[accp], vcc, {fresh}, %[sL]", ["L"], False),
             ("b2", "v_addc_co_u32_e64 %[accp], vcc, %[accp], %[accp], %[sU]", ["U", "b1"], True),
             ("b3", "v_addc_co_u32_e64 %[accp], vcc, %[accp], %[accp], %[sD]", ["D", "b2"], True),
             ("G1", "s_nop 0", [], False)]
    if s == 0:
        items.append(("MV", "v_mov_b32_e32 %[acc], %[accp]", ["b3"], True))
    return items


def code_items(s, sh):
    """Flags of column s-1 (sh = register holding wave_shr1 of G'_{s-1}) into its word.

    Every candidate X is <= G'_{s-1} (it is a max over them), so X == G' exactly
    when (G' - 1) - X < 0: the flag is the sign bit of one cheap VOP2
    subtraction, shifted into the word by v_alignbit_b32 (acc << 1 | d >> 31).
    Neighbouring scores differ by a few |m|+|k|+|d|, so the subtraction cannot
    wrap.  No compares, no SGPR masks.
    """
    if CODES == "cmp":
        return code_items_cmp(s, sh)
    Gp, Gpp, DGp = gname(s - 1), gname(s - 2), dg_reg(s - 1)
    hi = "0" if s == 1 else "%[accp]"      # first code of this chunk's word starts from 0
    items = [("G1", f"v_add_u32_e32 %[gm1], -1, %[{Gp}]", [], False),
             ("L", f"v_sub_u32_e32 %[dL], %[gm1], %[{Gpp}]", ["G1"], False),
             ("D", f"v_sub_u32_e32 %[dD], %[gm1], %[{DGp}]", ["G1"], False),
             ("U", f"v_sub_u32_e32 %[dU], %[gm1], %[{sh}]", ["G1"], True),
             ("b1", f"v_alignbit_b32 %[accp], {hi}, %[dL], 31", ["L"], False),
             ("b2", "v_alignbit_b32 %[accp], %[accp], %[dU], 31", ["U", "b1"], True),
             ("b3", "v_alignbit_b32 %[accp], %[accp], %[dD], 31", ["D", "b2"], True)]
    if s == 0:                # the previous chunk's word is complete: hand it out
        items.append(("MV", "v_mov_b32_e32 %[acc], %[accp]", ["b3"], True))
    return items


def score_items(s, A, S=False):
    """H (and |H| max, and its store) of column s-1."""
    h = f"h{s - 1}"
    items = [("H", f"v_add3_u32 %[{h}], %[{gname(s - 1)}], %[nlo], %[k{s - 1}]", [], False)]
    if S:
        items.append(("ST", f"global_store_dword %[hv], %[{h}], %[hb] offset:{256 * (s - 1)}", ["H"], False))
    if A:
        items.append(("A1", f"v_sub_u32_e32 %[tmp], 0, %[{h}]", ["H"], False))
        items.append(("A2", f"v_max3_i32 %[gav], %[gav], %[{h}], %[tmp]", ["A1"], False))
    return items


def ring_item(s):
    """G'_{s-1} of every lane to the ring (lane 63: the slot)."""
    return ("R", f"ds_write_b32 %[ra], %[{gname(s - 1)}] offset:{4 * (s - 1)}", [], False)


def step(s, N, F, H, A, nxt, S=False):
    Gp = gname(s - 1)
    Tm = "tm" if s == 0 else f"t{s - 1}"
    fill = []
    if F:
        fill += code_items(s, Tm)
    if s > 0:
        fill.append(ring_item(s))
    if H and s > 0:
        fill += score_items(s, A, S)
    if s + 1 < N or nxt:
        src, off = byte_src(s + 1)
        bfe = f"s_bfe_u32 %[sC], %[{src}], {hex(off | (8 << 16))}" if off else f"s_and_b32 %[sC], %[{src}], 0xff"
        fill.append(("S", bfe, [], False))
        fill.append(("M", "v_cmp_eq_u32_e64 %[sM], %[sC], %[c2]", ["S"], False))
        fill.append(("X", f"v_cndmask_b32_e64 %[{sub_reg(s + 1)}], %[vck], %[vcm], %[sM]", ["M"], False))
    if s == 7 and nxt:
        fill.append(("TM", "v_mov_b32_e32 %[tm], %[t7]", [], False))
    chain_head = [
        f"v_mov_b32_dpp %[{Tm}], %[{Gp}] wave_shr:1 row_mask:0xf bank_mask:0xf",
        f"v_add_u32_e32 %[{dg_reg(s)}], %[{Tm}], %[{sub_reg(s)}]",
        f"v_max3_i32 %[{gname(s)}], %[{Gp}], %[{dg_reg(s)}], %[t{s}]",
    ]
    dpps = ["row_shr:1 row_mask:0xf", "row_shr:2 row_mask:0xf", "row_shr:4 row_mask:0xf",
            "row_shr:8 row_mask:0xf", "row_bcast:15 row_mask:0xa", "row_bcast:31 row_mask:0xc"]
    out = []
    done = set()
    pending = list(fill)

    def take(allow_sh, k=2):
        got = []
        for it in list(pending):
            if len(got) == k:
                break
            name, text, deps, needs_sh = it
            if needs_sh and not allow_sh:
                continue
            if all(dd in done or dd in [g[0] for g in got] for dd in deps):
                got.append(it)
                pending.remove(it)
        for g in got:
            done.add(g[0])
        return [g[1] for g in got]

    def gap(allow_sh):
        got = take(allow_sh)
        if len(got) == 2:
            out.extend(got)
        elif len(got) == 1:
            out.extend(got + ["s_nop 0"])
        else:
            out.append("s_nop 1")

    gap(False)                     # before the DPP shift of G'_{s-1}
    out.extend(chain_head)
    g = gname(s)
    for dp in dpps:
        gap(True)                  # before each DPP max reading the previous VALU result
        out.append(f"v_max_i32_dpp %[{g}], %[{g}], %[{g}] {dp} bank_mask:0xf")
    while pending:                 # anything left runs after the scan
        got = take(True, 1)
        assert got, pending
        out.extend(got)
    return out


def block(N, F, H, A, nxt, S):
    lines = []
    for s in range(N):
        lines += step(s, N, F, H, A, nxt, S)
    if nxt:                        # the chunk's last column (G'_7 is final now)
        lines.append(ring_item(8)[1])
        if H:
            lines += [t for _, t, _, _ in score_items(8, A, S)]
    return lines


def flush(N, F, H, A, S):
    """Code, ring entry and score of the block's last column s = N-1 (no next step)."""
    s = N
    out = [ring_item(s)[1]]
    if F:
        items = {n: t for n, t, _, _ in code_items(s, f"t{s - 1}")}
        out += [items["G1"], items["L"], items["D"],
                f"v_mov_b32_dpp %[t{s - 1}], %[{gname(s - 1)}] wave_shr:1 row_mask:0xf bank_mask:0xf",
                items["U"], items["b1"], items["b2"], items["b3"]]
    if H:
        out += [t for _, t, _, _ in score_items(s, A, S)]
    return out


OPERANDS = r'''
#define NW_CHUNK_OPERANDS                                                                                  \
    : [g0] "=&v"(r.g[0]), [g1] "=&v"(r.g[1]), [g2] "=&v"(r.g[2]), [g3] "=&v"(r.g[3]),                      \
      [g4] "=&v"(r.g[4]), [g5] "=&v"(r.g[5]), [gp6] "+v"(r.gp6), [gin] "+v"(r.gin),                       \
      [t0] "+v"(r.t[0]), [t1] "+v"(r.t[1]), [t2] "+v"(r.t[2]), [t3] "+v"(r.t[3]),                          \
      [t4] "+v"(r.t[4]), [t5] "+v"(r.t[5]), [t6] "+v"(r.t[6]), [t7] "+v"(r.t[7]),                          \
      [tm] "+v"(r.tm), [dgA] "+v"(r.dgA), [dgB] "+v"(r.dgB), [subA] "+v"(r.subA), [subB] "+v"(r.subB),     \
      [h0] "=&v"(r.h[0]), [h1] "=&v"(r.h[1]), [h2] "=&v"(r.h[2]), [h3] "=&v"(r.h[3]),                      \
      [h4] "=&v"(r.h[4]), [h5] "=&v"(r.h[5]), [h6] "=&v"(r.h[6]), [h7] "=&v"(r.h[7]),                      \
      [accp] "+v"(r.accp), [acc] "=&v"(r.acc), [gav] "+v"(r.gav), [tmp] "=&v"(tmp_),                      \
      [gm1] "=&v"(gm1_), [dL] "=&v"(dL_), [dU] "=&v"(dU_), [dD] "=&v"(dD_), [sM] "=&s"(sM_), [sC] "=&s"(sC_), \
      [sL] "=&s"(sL_), [sU] "=&s"(sU_), [sD] "=&s"(sD_)                                                  \
    : [c2] "v"(k.c2), [vcm] "v"(k.vcm), [vck] "v"(k.vck), [nlo] "v"(k.nlo),                               \
      [chlo] "s"(ch.lo), [chhi] "s"(ch.hi), [chn] "s"(ch.nlo),                                            \
      [k0] "v"(k.kd[0]), [k1] "v"(k.kd[1]), [k2] "v"(k.kd[2]), [k3] "v"(k.kd[3]),                          \
      [k4] "v"(k.kd[4]), [k5] "v"(k.kd[5]), [k6] "v"(k.kd[6]), [k7] "v"(k.kd[7]),                          \
      [ra] "v"(ra), [hv] "v"(k.hv), [hb] "s"(hb)
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
    global OUT, CODES
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--codes", choices=("align", "cmp"), default="align")
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    OUT, CODES = args.out, args.codes
    parts = ["// GENERATED by tools/gen_chunk_asm.py -- do not edit; see the generator for the schedule.\n",
             OPERANDS, FLUSH_OPERANDS,
             "template <bool SH, bool SD, bool ST, int N, bool NEXT>\n"
             "__device__ __forceinline__ void chunk_asm(ChunkRegs& r, const ChunkConst& k, const ChunkChars& ch,\n"
             "                                          int ra, const int32_t* hb);\n"
             "template <bool SH, bool SD, bool ST, int N>\n"
             "__device__ __forceinline__ void flush_asm(ChunkRegs& r, const ChunkConst& k, int ra, const int32_t* hb);\n"]
    decl = "    int tmp_, gm1_, dL_, dU_, dD_; uint64_t sM_, sL_, sU_, sD_; uint32_t sC_;\n"
    for SH in (0, 1):
        for SD in (0, 1):
            for ST in (0, 1):
                F, H, A, S = SD or ST, SH or ST, ST, SH
                head = f"{tf(SH)}, {tf(SD)}, {tf(ST)}"
                for N in range(1, 9):
                    for nxt in ((0, 1) if N == 8 else (0,)):
                        parts.append(
                            f"template <> __device__ __forceinline__ void chunk_asm<{head}, {N}, {tf(nxt)}>"
                            f"(ChunkRegs& r, const ChunkConst& k, const ChunkChars& ch, int ra, const int32_t* hb) {{\n"
                            f"{decl}    asm volatile(\n{cstr(block(N, F, H, A, nxt, S))}\n"
                            f"        NW_CHUNK_OPERANDS : \"vcc\", \"scc\", \"memory\");\n}}\n")
                    parts.append(
                        f"template <> __device__ __forceinline__ void flush_asm<{head}, {N}>"
                        f"(ChunkRegs& r, const ChunkConst& k, int ra, const int32_t* hb) {{\n{decl}"
                        f"    const ChunkChars ch{{0u, 0u, 0u}};\n"
                        f"    asm volatile(\n{cstr(flush(N, F, H, A, S))}\n"
                        f"        NW_FLUSH_OPERANDS : \"vcc\", \"scc\", \"memory\");\n}}\n")
    parts.append("#undef NW_CHUNK_OPERANDS\n#undef NW_FLUSH_OPERANDS\n")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
