// nw_quad.hip -- the one-row column-scan fill kernel with skewed 16-lane row
// groups (the "quad" kernel; launched by nwi::fill_launch in nw_fill.hip;
// shared definitions in nw_kern.h).
//
// Same hot path -- compute_table_scores() (needleman-wunsch.c:583-626 ->
// score_cell :418-510) -- and the same stripe pipeline as nw_fill_kernel (a
// wave owns 64 rows, lane l = row j0 + l; waves of a workgroup chained through
// an LDS ring, workgroups through tagged granules, a loader and a publisher
// wave per workgroup).  What differs is the prefix max that resolves the
// vertical dependency.  nw_fill_kernel scans all 64 lanes per column: six DPP
// levels, each behind two wait states, the longest part of a column step.
// Here the wave's four 16-lane DPP rows ("row groups" q = lane / 16) run one
// column apart: at step t row group q computes column i = t - q + 1, so
//
//   * the scan stays inside a DPP row: four levels (row_shr 1 / 2 / 4 / 8);
//   * the cell above a row group's first lane -- the last lane of the row
//     group above, same column -- was computed one step earlier and arrives
//     with one row_bcast:15, off the critical path (for row group 0 it is the
//     row above the stripe, T, from the ring as before);
//   * the diagonal of that first lane is the same neighbour two steps
//     earlier, which is what the row_shr:1 shift leaves in place there (the
//     shift writes into the register that held the previous step's
//     row-above value).
//
// One step, in the domain G' = H + r*d + i*d (r = row offset inside the
// workgroup, i = column; left and up cost nothing, diag = G'(i-1, r-1) + sub',
// sub' = m + 2d | 2d - k, needleman-wunsch.c:429-465; no moving column base,
// the launcher checks the range):
//
//   Tp  = row_bcast15(G) into rows 1..3, row 0 keeps T_t      the row above, column i
//   dg  = sh + sub'                                            sh = row_shr1 of the previous G
//   X   = max3(G, dg, Tp)                                      left, diag, row above
//   G   = prefix max of X inside the DPP row                   4 levels
//   sh  = row_shr1(G), first lane of each row keeps Tp
//
// Direction flags: needleman-wunsch.c:485-503.  The wave below takes lane 63's
// row, which trails row group 0 by three columns: ring writes of a chunk
// straddle two 8-step blocks and a stripe runs ceil((L1 + 3) / 8) blocks.
//
// Layout (nw_table.skew = 2): the column layout stored by step, step t of row r
// = column (i - 1) + ((r & 63) >> 4); score tiles hold G' (raw = 2).  No stats
// variant: fills that ask for stats run nw_fill_kernel.

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "nw_kern.h"

#ifndef NW_QUAD_ASM
#define NW_QUAD_ASM 1     // 0: every block through the C++ path (a reference for the generated block)
#endif

namespace nwk {
namespace {

// row_bcast:15 into rows 1..3 (row 0 keeps old).
__device__ __forceinline__ int bcast15(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, 0x142, 0xe, 0xf, false); }
// row_shr:1, first lane of each row keeps old.
__device__ __forceinline__ int rshr1(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xf, 0xf, false); }

// Inclusive prefix max inside each 16-lane DPP row.
__device__ __forceinline__ int rowmax(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xf, 0xf, false));
    return x;
}

__device__ __forceinline__ void quad_store_scores(const int* h, int32_t* p) {
    __builtin_nontemporal_store(v4i{h[0], h[1], h[2], h[3]}, reinterpret_cast<v4i*>(p));
    __builtin_nontemporal_store(v4i{h[4], h[5], h[6], h[7]}, reinterpret_cast<v4i*>(p + 256));
}

// Operands of the generated block (nw_quad_chunk.inc).
struct QuadSlot {
    v4i a, b;           // T (row above, G') of columns 0..3, 4..7 of the chunk
    v2i c;              // the chunk's 8 top-string symbols
};
struct QuadRegs {
    int g;              // in/out: G' at the previous / this block's last step
    int sh;             // in/out: row_shr1(g), first lanes = the row above at that step
    int h[8];           // out: G' of the block's 8 steps (raw scores)
    uint32_t acc;       // out: the block's code word
    uint64_t pq;        // out: {prog[w], cons[w+1]} read mid-block
    uint32_t ptc1;      // in/out: symbols 4..7 of the previous / this chunk
    int cv;             // in/out: the block's chunk + 1 (cons[w] when its slot is taken; prog[w+1] = cv - 1)
};
struct QuadConst {
    uint32_t c2;        // side symbol of this lane's row
    int vcm, vck;       // sub' for match / mismatch
    uint32_t pl, ph;    // profile: byte q = sub' of symbol q (int8)
    uint32_t selq;      // v_perm selector of this row group's symbol window
    int cb;             // LDS address of ctr[2w]
};

#include "nw_quad_chunk.inc"

// Slow path: {prog[w], cons[w+1]}, then the slot.  Waited for.
__device__ __forceinline__ uint64_t quad_read_slot(int cb, int rd, QuadSlot& s) {
    uint64_t pq;
    asm volatile(
        "ds_read_b64 %[pq], %[cb] offset:8\n\t"
        "ds_read_b128 %[a], %[rd]\n\t"
        "ds_read_b128 %[b], %[rd] offset:16\n\t"
        "ds_read_b64 %[c], %[rd] offset:32\n\t"
        "s_waitcnt lgkmcnt(0)"
        : [pq] "=&v"(pq), [a] "=&v"(s.a), [b] "=&v"(s.b), [c] "=&v"(s.c)
        : [cb] "v"(cb), [rd] "v"(rd)
        : "memory");
    return pq;
}

// Workgroup = W compute waves + the loader + the publisher (<= 16 waves).
template <int W, bool SH, bool SD, bool PROF>
__global__ __launch_bounds__(64 * (W + 2)) void nw_quad_kernel(FillArgs a) {
    constexpr int R = 4;
    constexpr int NOCONS = 1 << 30;
    __shared__ __attribute__((aligned(16))) int tring[(W + 1) * R * SLOT];
    __shared__ __attribute__((aligned(8))) int ctr[2 * W + 4];
    __shared__ int scratch[64 + 2 * R * SLOT];   // dummy target of the block's ring writes (lanes 0..62)
    __shared__ int sh_sidx;
    __shared__ int sh_abort;

    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6);
    const bool loader = (w == W);          // feeds ring 0
    const bool pubw = (w == W + 1);        // drains the last compute wave's ring into granules
    const int d = a.d;
    const int vcm = a.m + 2 * a.d;
    const int vck = 2 * a.d - a.k;
    const int NC = a.NC;                      // chunks of real columns (granules, publisher)
    const int NCH = a.NCH;                    // 8-step blocks of a stripe = ceil((L1 + 3) / 8)
    const int nlast = a.L1 - CH * (NC - 1);   // columns in the last chunk (1..8)

    for (;;) {
        if (threadIdx.x == 0) {
            const int sidx = (int)atomicAdd(&a.ctl[CTL_NEXT], 1u);
            sh_sidx = sidx;
            sh_abort = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - (sidx * a.SQ + min(sidx, a.SR)));
            const bool drain = sidx + 1 < a.NSW || (a.xout && sidx * a.SQ + min(sidx, a.SR) + nw - 1 == a.NG - 1);
            for (int v = 0; v <= W; ++v) {
                ctr[2 * v + 2] = 0;
                ctr[2 * v + 1] = v < nw || (v == nw && drain) ? 0 : NOCONS;   // the publisher drains ring nw
            }
        }
        __syncthreads();
        const int sidx = uni(sh_sidx);
        if (sidx >= a.NSW || sh_abort) break;
        if (a.trace && threadIdx.x == 0) {
            a.trace[8 * (int64_t)sidx + 0] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 3] = (uint64_t)blockIdx.x | ((uint64_t)__smid() << 32);
        }
        const int g0 = sidx * a.SQ + min(sidx, a.SR);                 // first stripe of the WG-stripe
        const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - g0);
        const int g = g0 + w;
        const bool real = w < nw;
        const int j0 = 1 + 64 * g;                 // first row of the stripe
        const int jrow = j0 + lane;

        if (pubw) {
            // ---------------- publisher wave (as nw_fill_kernel's) ----------------
            const bool publish = sidx + 1 < a.NSW;
            const bool xpublish = a.xout && g0 + nw - 1 == a.NG - 1;
            uint64_t* gout = a.gran + (int64_t)((sidx + 1) % a.nslot) * a.gpitch;
            const int* bot = &tring[nw * R * SLOT];
            int cd = 0;
            if (xpublish && !xcredit_wait(a, &sh_abort)) {
                if (lane == 0) __hip_atomic_store(&sh_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                cd = NC;
            }
            cd = uni(cd);
            const uint32_t tag = publish ? a.gtag | (uint32_t)(sidx + 1) : a.epoch;
            gu64* const gdst = (gu64*)(publish ? gout : a.xout);
            // (plain domain: H - d = G' - 64*nw*d - i*d, i = CH*cd + lane + 1)
            int nklane = -(64 * nw * d + (lane + 1) * d);
            asm volatile("" : "+v"(nklane));
            const int* const botl = bot + lane;
            while ((publish || xpublish) && cd < NC) {
                const int p = uni(lds_ld(&ctr[2 * nw + 2]));          // prog of the last wave's ring
                if (p <= cd) {
                    if (uni(lds_ld(&sh_abort))) break;
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                lds_order();
                for (; cd < min(p, NC); ++cd) {
                    const int n = (cd == NC - 1) ? nlast : CH;
                    const int nsv = -(CH * cd) * d;
                    gu64* const gp = gdst + CH * (int64_t)cd;
                    if (lane < n) {
                        const int v = botl[(cd % R) * SLOT] + nklane + nsv;
                        const uint64_t gr = ((uint64_t)tag << 32) | (uint32_t)v;
                        if (publish)
                            __hip_atomic_store(gp + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        else
                            __hip_atomic_store(gp + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    if (xpublish && a.xflag && ((cd + 1) % a.xblk == 0 || cd == NC - 1)) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the block is out before its flag
                        if (lane == 0)
                            __hip_atomic_store(&a.xflag[cd / a.xblk], a.epoch, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                lds_order();
                if (lane == 0) lds_publish(&ctr[2 * nw + 1], cd);        // those ring slots are free again
            }
            // (a stripe's blocks past the last real chunk only write a slot that nobody waits for)
            if (lane == 0) lds_publish(&ctr[2 * nw + 1], NOCONS);
        } else if (loader) {
            // ---------------- loader wave: ring 0 (as nw_fill_kernel's) ----------------
            // It feeds NCH chunks: the chunks past the last real column carry
            // nothing (row group 3 still finishes its last columns there).
            const bool seeded = sidx == 0 && !a.xin;
            const bool xsrc = sidx == 0 && a.xin;
            const uint64_t* gin = xsrc ? a.xin : a.gran + (int64_t)(sidx % a.nslot) * a.gpitch;
            const uint32_t want = xsrc ? a.epoch : a.gtag | (uint32_t)sidx;
            const uint32_t* s1w = reinterpret_cast<const uint32_t*>(a.s1);
            const int wk = lane >> 3, wb = lane & 7;
            const int64_t ngr = (int64_t)CH * NC;
            auto gload = [&](int cf) -> uint64_t {
                const int64_t x = (int64_t)CH * cf + lane;
                return x < ngr ? ld_gran(gin + x, xsrc) : 0ull;
            };
            const int64_t nsw = 2 * (int64_t)NC + 16;
            auto sload = [&](int cf) -> uint32_t {
                const int64_t x = 2 * (int64_t)cf + 2 * wk + (wb & 1);
                return x < nsw ? s1w[x] : 0u;
            };
            // (H - d of the row above -> G' of row -1: + i*d, i = CH*c + wb + 1)
            int kwb = (wb + 1) * d;
            asm volatile("" : "+v"(kwb));
            const int dst0 = lds_addr(tring) + 4 * wb;
            auto window = [&](int cw, uint64_t& cur, uint64_t& nxt, uint32_t& scur, uint32_t& snxt) -> bool {
                asm volatile("" ::"v"(cur), "v"(scur));
                if (!seeded) nxt = gload(cw + CH);
                snxt = sload(cw + CH);
                const int ce = min(cw + CH, NCH);
                for (int c = cw; c < ce; ++c) {
                    const int n = c < NC - 1 ? CH : c == NC - 1 ? nlast : 0;
                    if (uni(lds_ld(&ctr[1])) < c - R + 1) {                      // ring slot not free yet
                        while (uni(lds_ld(&ctr[1])) < c - R + 1) {
                            if (uni(lds_ld(&sh_abort))) break;
                            __builtin_amdgcn_s_sleep(1);
                        }
                        if (uni(lds_ld(&sh_abort))) return false;
                    }
                    const int k = c - cw;
                    const bool mine = wk == k;                                  // lanes 8k .. 8k+7
                    const int nbase = (CH * c) * d;
                    int v;
                    if (seeded) {
                        // row 0: H[i][0] - d = -(i+1)*d (computation.c:102-110) -> G' = -d
                        v = -d;
                    } else {
                        const uint64_t need = (n == CH ? 0xffull : (1ull << n) - 1) << (8 * k);
                        if ((__ballot((uint32_t)(cur >> 32) == want) & need) != need) {
                            const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
                            bool stop = false;
                            for (;;) {
                                __builtin_amdgcn_s_sleep(1);
                                if (wk >= k && (uint32_t)(cur >> 32) != want) cur = gload(cw);
                                if ((__ballot((uint32_t)(cur >> 32) == want) & need) == need) break;
                                const int64_t now = (int64_t)__builtin_amdgcn_s_memrealtime();
                                const uint32_t ab = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT);
                                const bool peer = xsrc && __any(mine && wb < n && (uint32_t)(cur >> 32) == (want | POISON_BIT));
                                if (ab || peer || now - t0 > a.spin_ticks) {
                                    if (lane == 0) {
                                        __hip_atomic_store(&a.ctl[CTL_ABORT], 1u, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                                        if (!ab)
                                            atomicCAS(&a.ctl[CTL_ERR], 0u,
                                                      (uint32_t)(peer ? NW_ERR_PEER : NW_ERR_TIMEOUT));
                                        __hip_atomic_store(&sh_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    }
                                    stop = true;
                                    break;
                                }
                            }
                            if (stop) return false;
                        }
                        v = (int)(uint32_t)cur + kwb + nbase;
                        if (xsrc && mine && wb < n) a.row0[CH * c + wb] = (int)(uint32_t)cur;
                    }
                    if (mine) {
                        const int ad = dst0 + (c % R) * SLOT * 4;
                        asm volatile("ds_write2_b32 %0, %1, %2 offset1:8" :: "v"(ad), "v"(v), "v"(scur) : "memory");
                    }
                    lds_order();
                    if (lane == 0) lds_publish(&ctr[2], c + 1);
                }
                return true;
            };
            uint64_t gA = seeded ? 0ull : gload(0), gB = 0;
            uint32_t sA = sload(0), sB = 0;
            for (int cw = 0; cw < NCH; cw += 2 * CH) {
                if (!window(cw, gA, gB, sA, sB)) break;
                if (cw + CH < NCH && !window(cw + CH, gB, gA, sB, sA)) break;
            }
            if (xsrc) xcredit_post(a);
        } else if (real) {
            // ---------------- compute wave: its 64-row stripe, block by block ----
            const int q = lane >> 4;                   // row group: q columns behind row group 0
            int32_t* tile = a.H + (int64_t)g * a.spitch;
            uint32_t* dtile = a.D + (int64_t)g * (NCH + 1) * 64;
            const int* tin = &tring[w * R * SLOT];
            int* tout = &tring[(w + 1) * R * SLOT];
            const int* cin = &ctr[2 * w + 1];          // {cons[w], prog[w], cons[w+1]}
            QuadConst kc;
            kc.c2 = a.s2[jrow - 1];
            kc.vcm = vcm;
            kc.vck = vck;
            asm volatile("" : "+v"(kc.c2), "+v"(kc.vcm), "+v"(kc.vck));
            kc.pl = kc.ph = 0;
            if (PROF) {
#pragma unroll
                for (int x = 0; x < 8; ++x) {
                    const uint32_t b = (uint32_t)((uint32_t)x == kc.c2 ? vcm : vck) & 0xffu;
                    if (x < 4) kc.pl |= b << (8 * x);
                    else kc.ph |= b << (8 * (x - 4));
                }
            }
            // symbols of steps s - q, s = 0..3: bytes 4 - q .. 7 - q of {this word, the word before}
            kc.selq = 0x07060504u - 0x01010101u * (uint32_t)q;
            kc.cb = lds_addr(&ctr[2 * w]);
            asm volatile("" : "+v"(kc.cb), "+v"(kc.selq));
            // Ring writes: lane 63 into the slot, the other lanes into a per-lane dummy.
            const int ring0 = lane == 63 ? lds_addr(tout) : lds_addr(&scratch[lane]);
            int ra[R], rd[R];
#pragma unroll
            for (int x = 0; x < R; ++x) {
                ra[x] = ring0 + x * SLOT * 4;
                rd[x] = lds_addr(tin) + x * SLOT * 4;
                asm volatile("" : "+v"(ra[x]), "+v"(rd[x]));
            }
            // column 0 (and every column before it): G' = -(row_base + 64*g0 + 1)*d
            const int C0 = -(1 + a.row_base + 64 * g0) * d;
            // H = G' - (64*w + lane)*d - i*d
            const int nlo = -(64 * w + lane) * d;
            QuadRegs r;
            r.g = r.sh = C0;
            r.pq = 0;
            r.ptc1 = 0;
            r.cv = 0;
            bool aborted = false;
            if (a.trace && lane == 0 && w == 0) {
                a.trace[8 * (int64_t)sidx + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * (int64_t)sidx + 4] = __builtin_amdgcn_s_memtime();
            }
            if (a.trace && lane == 0 && w == nw - 1) a.trace[8 * (int64_t)sidx + 6] = __builtin_amdgcn_s_memrealtime();

            // ---- generic block (C++): the first block, where row groups 1..3
            // are still before column 1, and the last two, which hold every
            // row group's column L1 ----
            auto generic_block = [&](int c) -> bool {
                for (;;) {
                    const int pin = uni(lds_ld(&cin[1]));
                    const int pout = uni(lds_ld(&cin[2]));
                    if (pin > c && pout >= c - R + 1) break;
                    if (uni(lds_ld(&sh_abort))) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
                lds_order();
                const int* slot = &tin[(c % R) * SLOT];
                int T[CH];
#pragma unroll
                for (int s = 0; s < CH; ++s) T[s] = slot[s];
                const uint32_t sy0 = (uint32_t)slot[8], sy1 = (uint32_t)slot[9];
                lds_order();
                if (lane == 0) lds_publish(&ctr[2 * w + 1], c + 1);
                if (lane == 63) {                      // the chunk's symbols go down the ring
                    int* so = &tout[(c % R) * SLOT];
                    so[8] = (int)sy0;
                    so[9] = (int)sy1;
                }
                // this row group's symbol window: bytes 4 - q .. of {sy0, ptc1}, {sy1, sy0}
                const uint64_t win = ((uint64_t)sy0 << 32) | r.ptc1;
                const uint64_t win2 = ((uint64_t)sy1 << 32) | sy0;
                const uint32_t tq0 = (uint32_t)(win >> (8 * (4 - q))), tq1 = (uint32_t)(win2 >> (8 * (4 - q)));
                int h[CH];
                uint32_t acc = 0;
#pragma unroll
                for (int s = 0; s < CH; ++s) {
                    const int t = CH * c + s;
                    const int i = t - q + 1;               // this lane's column at this step
                    const uint32_t sym = ((s < 4 ? tq0 >> (8 * s) : tq1 >> (8 * (s - 4)))) & 0xffu;
                    const int Tp = bcast15(T[s], r.g);
                    const int dg = r.sh + (sym == kc.c2 ? vcm : vck);
                    const int X = max(max(r.g, dg), Tp);
                    int Gn = rowmax(X);
                    if (i < 1) Gn = C0;
                    const int shn = rshr1(Tp, Gn);
                    const uint32_t code = (dg == Gn ? 1u : 0u) | (shn == Gn ? 2u : 0u) | (r.g == Gn ? 4u : 0u);
                    acc = (acc << 3) | code;
                    h[s] = Gn;
                    if (!SH && i == a.L1) a.lastcol[jrow] = Gn + nlo - i * d;   // score-only: H[L1][*]
                    // lane 63's value is the row above of the wave below, 3 columns back
                    const int ci = t - 3;
                    if (lane == 63 && ci >= 0) tout[((ci >> 3) % R) * SLOT + (ci & 7)] = Gn;
                    if ((ci & 7) == 7 && ci >= 0) {
                        lds_order();
                        if (lane == 0) lds_publish(&ctr[2 * w + 4], (ci >> 3) + 1);
                    }
                    r.g = Gn;
                    r.sh = shn;
                }
                r.ptc1 = sy1;
                if (SH) quad_store_scores(h, tile + (int64_t)c * 512 + lane * 4);
                if (SD) __builtin_nontemporal_store(acc, dtile + (int64_t)(c + 1) * 64 + lane);
                return true;
            };
            // ---- full blocks: the generated block (nw_quad_chunk.inc) ----
            QuadSlot tA, tB;
            auto wait_slot = [&](int c, QuadSlot& tt) -> bool {
                for (;;) {
                    const uint64_t pq = quad_read_slot(kc.cb, rd[c % R], tt);
                    const int pin = uni((int)(uint32_t)pq), pout = uni((int)(pq >> 32));
                    if (pin > c && pout >= c - R + 1) return true;
                    if (uni(lds_ld(&sh_abort))) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            auto full_block = [&](int c, auto slotc, QuadSlot& cur, QuadSlot& nxt, bool more) -> bool {
                constexpr int Q = decltype(slotc)::value;
                quad_chunk_asm<SH, SD, PROF>(r, kc, cur, nxt, ra[Q], ra[(Q + R - 1) % R], rd[(Q + 1) % R]);
                r.h[7] = r.g;
                if (SH) quad_store_scores(r.h, tile + (int64_t)c * 512 + lane * 4);
                if (SD) __builtin_nontemporal_store(r.acc, dtile + (int64_t)(c + 1) * 64 + lane);
                if (!more) return true;                // the next block is a generic one
                // (prog[w] > c + 1 and cons[w+1] >= c + 2 - R, as one sign test: the common case falls through)
                if (__builtin_expect(((uni((int)(uint32_t)r.pq) - (c + 2)) | (uni((int)(r.pq >> 32)) - (c + 2 - R))) >= 0, 1))
                    return true;
                return wait_slot(c + 1, nxt);
            };
            using S0 = std::integral_constant<int, 0>;
            using S1 = std::integral_constant<int, 1>;
            using S2 = std::integral_constant<int, 2>;
            using S3 = std::integral_constant<int, 3>;
            const int cend = NCH - 2;                  // generic blocks: 0 and cend .. NCH-1
            int c = 0;
            aborted = !generic_block(0);
            c = 1;
#if NW_QUAD_ASM
            if (!aborted && c < cend) {
                aborted = !wait_slot(c, tB);           // block 1 sits in ring slot 1
                r.cv = c + 1;
                // blocks are unrolled by ring slot: c % 4 = 1, 2, 3, 0
                // (one loop with an end check per block: the same blocks in groups
                // of four without end checks ran 1.6% slower -- code placement,
                // profiles/r04n_ab_interblock.txt)
                while (!aborted && c < cend) {
                    const bool m1 = c + 1 < cend, m2 = c + 2 < cend, m3 = c + 3 < cend, m4 = c + 4 < cend;
                    aborted = !full_block(c, S1{}, tB, tA, m1);
                    if (!aborted && m1) aborted = !full_block(c + 1, S2{}, tA, tB, m2);
                    if (!aborted && m2) aborted = !full_block(c + 2, S3{}, tB, tA, m3);
                    if (!aborted && m3) aborted = !full_block(c + 3, S0{}, tA, tB, m4);
                    c += 4;
                }
                c = cend;
            }
#endif
            for (c = max(c < cend ? c : cend, 1); c < NCH && !aborted; ++c) aborted = !generic_block(c);
            // the last chunk's slot is only part written: the wave below may take it
            if (!aborted) {
                lds_order();
                if (lane == 0) lds_publish(&ctr[2 * w + 4], NCH);
            }
        }
        if (a.trace && real && w == nw - 1 && lane == 0) {
            a.trace[8 * (int64_t)sidx + 2] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 5] = __builtin_amdgcn_s_memtime();
        }
        __syncthreads();
        if (sh_abort) break;
    }
}

template <int W, bool P>
KernelFn pick_flags(bool sh, bool sd) {
    if (sh && sd) return nw_quad_kernel<W, true, true, P>;
    if (sh) return nw_quad_kernel<W, true, false, P>;
    if (sd) return nw_quad_kernel<W, false, true, P>;
    return nw_quad_kernel<W, false, false, P>;
}

}  // namespace

KernelFn pick_quad(int W, bool prof, bool sh, bool sd) {
    switch (W) {
        case 1: return prof ? pick_flags<1, true>(sh, sd) : pick_flags<1, false>(sh, sd);
        case 2: return prof ? pick_flags<2, true>(sh, sd) : pick_flags<2, false>(sh, sd);
        case 3: return prof ? pick_flags<3, true>(sh, sd) : pick_flags<3, false>(sh, sd);
        case 4: return prof ? pick_flags<4, true>(sh, sd) : pick_flags<4, false>(sh, sd);
        case 8: return prof ? pick_flags<8, true>(sh, sd) : pick_flags<8, false>(sh, sd);
        default: return nullptr;
    }
}

}  // namespace nwk
