#!/usr/bin/env python3
"""Generate needleman-wunsch_amd/csrc/nw_skew_chunk.inc: the hand-scheduled
8-step chunk block of the skewed-stripe fill kernel (nw_skew.hip).

    python tools/gen_skew_asm.py [--out PATH]

At step s of a chunk (t = 8c + s) lane l computes cell (i = t - l + 1, j0 + l)
in the domain E = H + (t + 1 - base)*d (see nw_skew.hip):

    u_s  = wave_shr1(E_{s-1}), lane 0 <- T_s + P + s*d      v_mov_b32_dpp (lane 0 pre-filled)
    dg_s = u_{s-1} + sub'_s                                    v_add_u32 (SDWA sext byte of the profile)
    E_s  = max3(E_{s-1}, u_s, dg_s)                            v_max3_i32

so the loop-carried chain is DPP -> max3 -> DPP: two instructions and the two
wait states a DPP needs after the VALU that wrote its source.  Everything else
of the step fills those gaps and follows:
  * the direction code of the SAME step (all three candidates are at hand):
    candidate - E_s is 0 exactly for the candidates that attain the max and
    negative otherwise, so the sign bit of one v_sub is the inverted flag,
    shifted into the word with v_alignbit_b32 (word inverted once per chunk);
  * H_s = E_s + M + kd_s (plain score: tile store, ring, stats);
  * the ring write of H_s (lane 63 into the slot of the wave below, the other
    lanes into a per-lane dummy), the pre-fill of u_{s+2} for lane 0 and the
    diagonal candidate of step s+1;
  * the chunk's LDS traffic: cons (slot taken), the next {prog, cons} pair, the
    next slot's 8 T and the next chunk's 8 window symbols, prog (after the last
    ring write).  The block ends with lgkmcnt(K), K = the LDS ops issued after
    its last read, so the caller finds the reads done.

Lane 63 computes column 8c + s - 62 at step s: positions 1..7 of ring slot
c - 8 (= the chunk's own slot modulo R = 4) in steps 0..6, position 0 of slot
c - 7 in step 7.

Template: skew_chunk_asm<ST, P>: ST = |H| max for the stats, P = profile
lookups (symbols coded 0..7, sub' as int8) instead of byte compares.
Scores/codes are stored by the caller from h[0..7] / acc.
"""
import argparse
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "needleman-wunsch_amd", "csrc", "nw_skew_chunk.inc")


def E(s):
    """Register of E_s (s = -1: the carried value of the previous chunk)."""
    return "ein" if s in (-1, 7) else f"e{s}"


def U(s):
    """Register of u_s (s = -1 / 7: the carried up value)."""
    return "upc" if s in (-1, 7) else f"u{s}"


def dg(s):
    """dg_s: three rotate (dg_{s+1} is written while dg_{s-1} is still read)."""
    return f"dg{s % 3}"


def sub_src(s, P):
    """Diagonal candidate dg_s = u_{s-1} + sub'_s."""
    if P:
        reg = "subA" if s < 4 else "subB"
        return [f"v_add_u32_sdwa %[{dg(s)}], %[{U(s - 1)}], sext(%[{reg}]) dst_sel:DWORD "
                f"dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_{s % 4}"]
    w = "wx" if s < 4 else "wy"
    return [f"v_cmp_eq_u32_sdwa vcc, %[{w}], %[c2] src0_sel:BYTE_{s % 4} src1_sel:DWORD",
            f"v_cndmask_b32_e64 %[sub], %[vck], %[vcm], vcc",
            f"v_add_u32_e32 %[{dg(s)}], %[{U(s - 1)}], %[sub]"]


def prefill(s):
    """Lane 0's u_s before the DPP: T_s + P + s*d (the other lanes are overwritten)."""
    t = f"ta{s}" if s < 4 else f"tb{s - 4}"
    return f"v_add3_u32 %[{U(s)}], %[{t}], %[P], %[sd{s}]"


def code_items(s):
    """Inverted flags of step s into the word: L, U, D subs and three v_alignbit."""
    hi = "0" if s == 0 else "%[acc]"
    return {"L": f"v_sub_u32_e32 %[dL], %[{E(s - 1)}], %[{E(s)}]",
            "U": f"v_sub_u32_e32 %[dU], %[{U(s)}], %[{E(s)}]",
            "D": f"v_sub_u32_e32 %[dD], %[{dg(s)}], %[{E(s)}]",
            "B1": f"v_alignbit_b32 %[acc], {hi}, %[dL], 31",
            "B2": "v_alignbit_b32 %[acc], %[acc], %[dU], 31",
            "B3": "v_alignbit_b32 %[acc], %[acc], %[dD], 31"}


def block(ST, P):
    """Software-pipelined: the code of step s is computed during step s + 1, so
    no instruction directly follows the one it depends on (a dependent VALU
    right behind its producer stalls a lone wave)."""
    out = []
    out.append(prefill(0))
    out.append(prefill(1))
    if P:
        out.append("v_perm_b32 %[subA], %[ph], %[pl], %[wx]")
        out.append("v_perm_b32 %[subB], %[ph], %[pl], %[wy]")
    out.append("ds_write_b32 %[cb], %[cv] offset:4")          # cons[w] = c+1: slot c taken
    out += sub_src(0, P)
    mem = {2: ["ds_read_b64 %[pq], %[cb] offset:8"],          # {prog[w], cons[w+1]}
           3: ["ds_read_b128 %[nA], %[rd]"],                  # next slot: T_0..3
           4: ["ds_read_b128 %[nB], %[rd] offset:16"],        # T_4..7
           5: ["ds_read_b64 %[nw], %[wa]"]}                   # next chunk's 8 symbols
    for s in range(8):
        cp = code_items(s - 1) if s > 0 else {}
        out.append(f"v_mov_b32_dpp %[{U(s)}], %[{E(s - 1)}] wave_shr:1 row_mask:0xf bank_mask:0xf")
        if cp:
            out.append(cp["L"])
        out.append(f"v_max3_i32 %[{E(s)}], %[{E(s - 1)}], %[{U(s)}], %[{dg(s)}]")
        if cp:
            out += [cp["U"], cp["D"]]
        out.append(f"v_add3_u32 %[h{s}], %[{E(s)}], %[M], %[kd{s}]")
        if s + 1 < 8:
            out += sub_src(s + 1, P)
        if cp:
            out.append(cp["B1"])
        if s + 2 < 8:
            out.append(prefill(s + 2))
        if cp:
            out.append(cp["B2"])
        if s < 7:
            out.append(f"ds_write_b32 %[ra], %[h{s}] offset:{4 * (s + 1)}")
        else:
            out.append("ds_write_b32 %[ra1], %[h7]")
        if cp:
            out.append(cp["B3"])
        if ST:
            out.append(f"v_sub_u32_e32 %[tmp], 0, %[h{s}]")
            out.append(f"v_max3_i32 %[gav], %[gav], %[h{s}], %[tmp]")
        out += mem.get(s, [])
    # tail: the code of step 7 (E_7 = ein, u_7 = upc)
    cp = code_items(7)
    out += [cp["L"], cp["U"], cp["D"], "ds_write_b32 %[cb], %[cv] offset:16",   # prog[w+1] = c+1
            cp["B1"], cp["B2"], cp["B3"],
            "v_xor_b32_e32 %[acc], 0xffffff, %[acc]"]                            # flags were inverted
    # lgkmcnt: LDS ops after the last read (the window read)
    last = max(i for i, x in enumerate(out) if x.startswith("ds_read"))
    k = sum(1 for x in out[last + 1:] if x.startswith("ds_"))
    out.append(f"s_waitcnt lgkmcnt({k})")
    check_dpp(out)
    return out


def check_dpp(lines):
    """A DPP reading a VGPR needs two instructions after the VALU that wrote it."""
    def dst(x):
        if x.startswith(("ds_", "s_")):
            return None
        return x.split()[1].rstrip(",")
    for i, x in enumerate(lines):
        if "_dpp" in x:
            src = x.split()[2].rstrip(",")
            for j in (i - 1, i - 2):
                assert dst(lines[j]) != src, (i, x, lines[j])


OPERANDS = r'''
#define NW_SKEW_OPERANDS                                                                                   \
    : [e0] "=&v"(r.e[0]), [e1] "=&v"(r.e[1]), [e2] "=&v"(r.e[2]), [e3] "=&v"(r.e[3]),                      \
      [e4] "=&v"(r.e[4]), [e5] "=&v"(r.e[5]), [e6] "=&v"(r.e[6]), [ein] "+v"(r.ein),                       \
      [u0] "=&v"(u_[0]), [u1] "=&v"(u_[1]), [u2] "=&v"(u_[2]), [u3] "=&v"(u_[3]),                          \
      [u4] "=&v"(u_[4]), [u5] "=&v"(u_[5]), [u6] "=&v"(u_[6]), [upc] "+v"(r.upc),                          \
      [dg0] "=&v"(dg_[0]), [dg1] "=&v"(dg_[1]), [dg2] "=&v"(dg_[2]), [dL] "=&v"(dL_), [dU] "=&v"(dU_), [dD] "=&v"(dD_),              \
      [subA] "=&v"(subA_), [subB] "=&v"(subB_), [sub] "=&v"(sub_), [tmp] "=&v"(tmp_),                      \
      [h0] "=&v"(r.h[0]), [h1] "=&v"(r.h[1]), [h2] "=&v"(r.h[2]), [h3] "=&v"(r.h[3]),                      \
      [h4] "=&v"(r.h[4]), [h5] "=&v"(r.h[5]), [h6] "=&v"(r.h[6]), [h7] "=&v"(r.h[7]),                      \
      [acc] "=&v"(r.acc), [gav] "+v"(r.gav), [pq] "=&v"(r.pq),                                             \
      [nA] "=&v"(ns.a), [nB] "=&v"(ns.b), [nw] "=&v"(ns.w)                                            \
    : [ta0] "v"(ts.a[0]), [ta1] "v"(ts.a[1]), [ta2] "v"(ts.a[2]), [ta3] "v"(ts.a[3]),                      \
      [tb0] "v"(ts.b[0]), [tb1] "v"(ts.b[1]), [tb2] "v"(ts.b[2]), [tb3] "v"(ts.b[3]),                      \
      [wx] "v"(ts.w[0]), [wy] "v"(ts.w[1]),                                                                \
      [sd0] "v"(k.sd[0]), [sd1] "v"(k.sd[1]), [sd2] "v"(k.sd[2]), [sd3] "v"(k.sd[3]),                      \
      [sd4] "v"(k.sd[4]), [sd5] "v"(k.sd[5]), [sd6] "v"(k.sd[6]), [sd7] "v"(k.sd[7]),                      \
      [kd0] "v"(k.kd[0]), [kd1] "v"(k.kd[1]), [kd2] "v"(k.kd[2]), [kd3] "v"(k.kd[3]),                      \
      [kd4] "v"(k.kd[4]), [kd5] "v"(k.kd[5]), [kd6] "v"(k.kd[6]), [kd7] "v"(k.kd[7]),                      \
      [P] "s"(Pc), [M] "s"(Mc), [c2] "v"(k.c2), [vcm] "v"(k.vcm), [vck] "v"(k.vck),                        \
      [pl] "v"(k.pl), [ph] "v"(k.ph), [cb] "v"(k.cb), [cv] "v"(cv), [ra] "v"(ra), [ra1] "v"(ra1),          \
      [rd] "v"(rd), [wa] "v"(wa)
'''


def cstr(lines):
    return "\n".join(f'        "{ln}\\n\\t"' for ln in lines)


def main():
    global OUT
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    parts = ["// GENERATED by tools/gen_skew_asm.py -- do not edit; see the generator for the schedule.\n",
             OPERANDS,
             "template <bool ST, bool P>\n"
             "__device__ __forceinline__ void skew_chunk_asm(SkewRegs& r, const SkewConst& k, const SkewSlot& ts,\n"
             "                                               SkewSlot& ns, int Pc, int Mc, int cv, int ra, int ra1,\n"
             "                                               int rd, int wa);\n"]
    decl = "    int u_[7], dg_[3], dL_, dU_, dD_, subA_, subB_, sub_, tmp_;\n"
    for ST in (0, 1):
        for P in (0, 1):
            lines = block(ST, P)
            tf = lambda b: "true" if b else "false"
            parts.append(
                f"template <> __device__ __forceinline__ void skew_chunk_asm<{tf(ST)}, {tf(P)}>"
                f"(SkewRegs& r, const SkewConst& k, const SkewSlot& ts, SkewSlot& ns, int Pc, int Mc, int cv,\n"
                f"    int ra, int ra1, int rd, int wa) {{\n{decl}"
                f"    asm volatile(\n{cstr(lines)}\n"
                f"        NW_SKEW_OPERANDS : \"vcc\", \"memory\");\n}}\n")
    parts.append("#undef NW_SKEW_OPERANDS\n")
    with open(args.out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
