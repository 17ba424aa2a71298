// nw_pair.hip -- the two-rows-per-lane column-scan fill kernel (the "pair"
// kernel; launched by nwi::fill_launch in nw_fill.hip, which also holds the
// one-row scan kernel; shared definitions in nw_kern.h).
//
// Same hot path -- compute_table_scores() (needleman-wunsch.c:583-626 ->
// score_cell :418-510) -- and the same stripe scan as nw_fill_kernel, but a
// wave owns a 128-row stripe: lane l holds rows a = j0 + 2l and b = a + 1.
// At 100k rows that is 782 waves instead of 1563, so every SIMD runs at most
// one compute wave (the one-row kernel doubles up on half of them and the
// whole stripe chain moves at the two-wave rate).  One column step:
//
//   Xa  = max3(Ga, sh + sub'_a, T)          left, diag (lane l-1's row b), row above
//   Xb  = max3(Gb, Ga + sub'_b, Xa)          left, diag (own row a), up (own row a)
//   Gb' = prefix max of Xb over the lanes    the 6-level DPP scan of the one-row kernel
//   sh' = wave_shr1(Gb'), lane 0 <- T        row b of lane l-1 = the cell above row a
//   Ga' = max(Xa, sh')
//
// in the one-row kernel's domain G' = H + r*d + (i - base)*d (r = row offset
// inside the workgroup, i = column), where left and up cost nothing and
// diag = G'(i-1, r-1) + sub', sub' = m + 2d | 2d - k (needleman-wunsch.c:
// 429-465).  Including the row above T in every lane's Xa is harmless: G' is
// non-decreasing down a column.  Direction flags: needleman-wunsch.c:485-503.
//
// Layout (nw_table.pair = 1): the one-row kernel's layout with rows
// permuted -- row r of the table is row rperm(r) = 64*(2*(r/128) + r%2) +
// (r%128)/2 of a 64-row layout ("virtual stripes" 2g and 2g+1 hold the a and
// b rows of pair stripe g), so every reader only maps the row.

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "nw_kern.h"

#ifndef NW_PAIR_PIPE
#define NW_PAIR_PIPE 1     // 0: the raw scores + codes fill runs the unpipelined block (pair_chunk_raw)
#endif

namespace nwk {
namespace {

// Count 3-bit codes of a word (8 per word, bits 0..23) with >= 2 directions.
__device__ __forceinline__ uint32_t branch_codes(uint32_t x) {
    const uint32_t y = (x & (x >> 1)) | (x & (x >> 2)) | ((x >> 1) & (x >> 2));
    return __builtin_popcount(y & 0x249249u);
}

// wave_shr:1, lane 0 <- old.
__device__ __forceinline__ int shr1(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false); }

// Inclusive prefix max over the 64 lanes (row_shr 1/2/4/8, row_bcast 15/31).
__device__ __forceinline__ int prefmax(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x143, 0xc, 0xf, false));
    return x;
}

__device__ __forceinline__ void pair_store_scores(const int* h, int32_t* p) {
    __builtin_nontemporal_store(v4i{h[0], h[1], h[2], h[3]}, reinterpret_cast<v4i*>(p));
    __builtin_nontemporal_store(v4i{h[4], h[5], h[6], h[7]}, reinterpret_cast<v4i*>(p + 256));
}

// Operands of the generated chunk block (nw_pair_chunk.inc).
struct PairSlot {
    v4i a, b;           // T (row above, G') of columns 0..3, 4..7 of the chunk
    v2i c;              // the chunk's 8 top-string symbols
};
struct PairRegs {
    int ga, gb;         // in/out: final G' of rows a, b at the previous / this chunk's last column
    int sh;             // in/out: wave_shr1(gb), lane 0 = the row above at that column
    int ha[8], hb[8];   // out: H of rows a, b
    uint32_t accA, accB;// out: the chunk's code words of rows a, b
    int gavA, gavB;     // in/out: running max |H| (stats)
    uint64_t pq;        // out: {prog[w], cons[w+1]} read mid-chunk
    int nloa, nlob;     // H = G' + nlo - (s+1)d (moved by -8d per chunk by the caller)
    // pair_chunk_pipe (raw scores + codes, pipelined across blocks): G' of
    // columns 4..7 of rows a / b in fixed registers (.w = the carried ga / gb),
    // column 7's diagonal candidates, and accA / accB = the block's code words
    // still without column 7; the next block -- or flush_pending -- finishes
    // and stores them.
    v4i qa1, qb1;
    int dga1, dgb1;
};
struct PairConst {
    int kd[8];          // -(s+1)*d
    uint32_t c2a, c2b;  // side symbols of rows a, b (byte compares)
    int vcm, vck;       // sub' for match / mismatch
    uint32_t pla, pha, plb, phb;   // profiles of rows a, b: byte q = sub' of symbol q (int8)
    int cb;             // LDS address of ctr[2w]
};

#include "nw_pair_chunk.inc"

// Slow path: {prog[w], cons[w+1]}, then the slot (in order per wave: slot
// data read after a progress value that covers it is valid).  Waited for.
__device__ __forceinline__ uint64_t pair_read_slot(int cb, int rd, PairSlot& s) {
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
template <int W, bool SH, bool SD, bool ST, bool PROF>
__global__ __launch_bounds__(64 * (W + 2)) void nw_pair_kernel(FillArgs a) {
    constexpr int R = 4;
    // Raw scores (fills with scores and without stats): the tiles hold G'
    // itself, the readers add the affine offset back (nwk::raw_offset; the
    // table's raw flag).  Two v_add3 fewer per column: 100k^2 9.21 -> 8.89 ms.
    constexpr bool RAW = SH && !ST;
    // (raw scores + codes: the block pipelined across chunks, pair_chunk_pipe)
    constexpr bool PIPE = RAW && SD && NW_PAIR_PIPE;
    constexpr int NOCONS = 1 << 30;
    __shared__ __attribute__((aligned(16))) int tring[(W + 1) * R * SLOT];
    __shared__ __attribute__((aligned(8))) int ctr[2 * W + 4];
    __shared__ int scratch[64 + R * SLOT];     // dummy target of the block's ring writes (lanes 0..62)
    __shared__ int sh_sidx;
    __shared__ int sh_abort;

    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6);
    const bool loader = (w == W);          // feeds ring 0
    const bool pubw = (w == W + 1);        // drains the last compute wave's ring into granules
    const int d = a.d;
    const int vcm = a.m + 2 * a.d;
    const int vck = 2 * a.d - a.k;
    const int NC = a.NC;
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
                ctr[2 * v + 1] = v < nw || (v == nw && drain) ? 0 : NOCONS;   // the loader drains ring nw
            }
        }
        __syncthreads();
        const int sidx = uni(sh_sidx);
        if (sidx >= a.NSW || sh_abort) break;
        if (a.trace && threadIdx.x == 0) {
            a.trace[8 * (int64_t)sidx + 0] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 3] = (uint64_t)blockIdx.x | ((uint64_t)__smid() << 32);
            if (NW_TRACE_EXT)
                a.trace[8 * (int64_t)sidx + 7] = (uint64_t)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15);   // XCC_ID
        }
        const int g0 = sidx * a.SQ + min(sidx, a.SR);                 // first pair stripe of the WG-stripe
        const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - g0);
        const int g = g0 + w;
        const bool real = w < nw;
        const int j0 = 1 + 128 * g;                // first row of the pair stripe
        const int ja = j0 + 2 * lane, jb = ja + 1; // this lane's rows
        int gav = 0;
        uint32_t bc = 0;

        if (pubw) {
            // ---------------- publisher wave ----------------
            // Drains the ring below the last compute wave into this
            // WG-stripe's bottom-row granules (for the next WG-stripe, or the
            // panel below), so the hand-off stores stay off the compute waves.
            const bool publish = sidx + 1 < a.NSW;
            // the panel's last row is row b of lane 63 of its last pair stripe (128*k rows)
            const bool xpublish = a.xout && g0 + nw - 1 == a.NG - 1;
            uint64_t* gout = a.gran + (int64_t)((sidx + 1) % a.nslot) * a.gpitch;
            const int* bot = &tring[nw * R * SLOT];
            int cd = 0;
            if (xpublish && !xcredit_wait(a, &sh_abort)) {
                if (lane == 0) __hip_atomic_store(&sh_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                cd = NC;
            }
            // Everything per chunk but the slot read, one add and the store is
            // scalar: the publisher shares a SIMD with a compute wave, and its
            // vector instructions come out of that wave's issue
            // (profiles/r02e_ab_chain_issue.txt).
            cd = uni(cd);
            const uint32_t tag = publish ? a.gtag | (uint32_t)(sidx + 1) : a.epoch;
            gu64* const gdst = (gu64*)(publish ? gout : a.xout);
            // (plain domain: H - d = G' - 128*nw*d - (i - base)d, i = CH*cd + lane + 1)
            int nklane = -(128 * nw * d + (lane + 1) * d);
            asm volatile("" : "+v"(nklane));                       // one v_add3 per granule
            const int* const botl = bot + lane;
            while ((publish || xpublish) && cd < NC) {
                const int p = uni(lds_ld(&ctr[2 * nw + 2]));          // prog of the last wave's ring
                if (p <= cd) {
                    if (uni(lds_ld(&sh_abort))) break;
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                lds_order();
                for (; cd < p; ++cd) {
                    const int n = (cd == NC - 1) ? nlast : CH;
                    const int nsv = -(CH * cd - chunk_base(cd)) * d;
                    gu64* const gp = gdst + CH * (int64_t)cd;
                    if (lane < n) {
                        const int v = botl[(cd % R) * SLOT] + nklane + nsv;
                        const uint64_t gr = ((uint64_t)tag << 32) | (uint32_t)v;
                        if (publish)   // put_granule (nw_kern.h) on the global address space
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
                if (NW_TRACE_EXT && a.trace && lane == 0 && cd > trace_mid_chunk(NC, R) && *trace_ext(a, TX_PUB, sidx) == 0)
                    *trace_ext(a, TX_PUB, sidx) = __builtin_amdgcn_s_memrealtime();
            }
        } else if (loader) {
            // ---------------- loader wave: ring 0 (as the one-row kernel's) ----------------
            // Nothing it waits for per chunk is a fresh global load unless the
            // granules are not there yet: the granule window (8 chunks, one lane
            // per granule) and the top-string window (2 dwords per chunk) are
            // prefetched one window ahead; a per-chunk
            // dependent load made the loader, not the producer, pace every
            // WG-stripe hop (+11% at 100k^2, tools/trace_lag.py).  Kept inline:
            // the same loop as a shared __device__ function compiled 5-10%
            // slower at 100k^2 (profiles/r02_ab_loader.txt).
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
            // lanes 8k and 8k+1 hold the two symbol words of chunk cf + k
            // (the other lanes duplicates), so the lanes that write chunk
            // cf + k's row-above values write its symbols in the same ds_write2
            auto sload = [&](int cf) -> uint32_t {
                const int64_t x = 2 * (int64_t)cf + 2 * wk + (wb & 1);
                return x < nsw ? s1w[x] : 0u;
            };
            // (H - d of the row above -> G' of row -1: + (i - base)*d, i = CH*c + wb + 1)
            int kwb = (wb + 1) * d;
            asm volatile("" : "+v"(kwb));
            const int dst0 = lds_addr(tring) + 4 * wb;
            // One window of CH chunks out of cur / scur, with the next window's
            // granules and symbols prefetched into nxt / snxt.  The two windows'
            // registers alternate (ping-pong, no copies): a copy of the
            // prefetched value into the loop-carried register made the
            // compiler wait for the prefetch right after issuing it, so every
            // window shift stalled the loader for a full load latency.
            auto window = [&](int cw, uint64_t& cur, uint64_t& nxt, uint32_t& scur, uint32_t& snxt) -> bool {
                // this window's loads were issued a window ago: take them now,
                // before the prefetch goes out, so no later wait covers it
                asm volatile("" ::"v"(cur), "v"(scur));
                if (!seeded) nxt = gload(cw + CH);
                snxt = sload(cw + CH);
                const int ce = min(cw + CH, NC);
                for (int c = cw; c < ce; ++c) {
                    const int n = (c == NC - 1) ? nlast : CH;
                    const bool tcm = NW_TRACE_EXT && a.trace && lane == 0 && c == trace_mid_chunk(NC, R);
                    if (tcm) *trace_ext(a, TX_REACH, sidx) = __builtin_amdgcn_s_memrealtime();
                    if (uni(lds_ld(&ctr[1])) < c - R + 1) {                      // ring slot not free yet
                        while (uni(lds_ld(&ctr[1])) < c - R + 1) {
                            if (uni(lds_ld(&sh_abort))) break;
                            __builtin_amdgcn_s_sleep(1);
                        }
                        if (uni(lds_ld(&sh_abort))) return false;
                    }
                    if (tcm) *trace_ext(a, TX_CREDIT, sidx) = __builtin_amdgcn_s_memrealtime();
                    const int k = c - cw;
                    const bool mine = wk == k;                                  // lanes 8k .. 8k+7
                    const int nbase = (CH * c - chunk_base(c)) * d;
                    int v;
                    if (seeded) {
                        // row 0: H[i][0] - d = -(i+1)*d (computation.c:102-110) -> G' = -(base+1)*d
                        v = -(chunk_base(c) + 1) * d;
                    } else {
                        // every granule of the chunk this loader needs carries the tag
                        const uint64_t need = ((n == CH ? 0xffull : (1ull << n) - 1)) << (8 * k);
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
                        if (tcm) *trace_ext(a, TX_LOAD, sidx) = __builtin_amdgcn_s_memrealtime();
                        v = (int)(uint32_t)cur + kwb + nbase;
                        if (xsrc && mine && wb < n) a.row0[CH * c + wb] = (int)(uint32_t)cur;
                    }
                    // lanes 8k..8k+7: slot[wb] = the row above, slot[8 + wb] = symbol
                    // word wb (wb < 2; the others land in the slot's unused tail)
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
            for (int cw = 0; cw < NC; cw += 2 * CH) {
                if (!window(cw, gA, gB, sA, sB)) break;
                if (cw + CH < NC && !window(cw + CH, gB, gA, sB, sA)) break;
            }
            if (xsrc) xcredit_post(a);
        } else if (real) {
            // ---------------- compute wave: its 128-row stripe, chunk by chunk ----
            // virtual 64-row stripes 2g (rows a) and 2g+1 (rows b): a.spitch = 1024*NC
            int32_t* tileA = a.H + (int64_t)g * a.spitch;
            int32_t* tileB = tileA + a.spitch / 2;
            uint32_t* dtileA = a.D + (int64_t)(2 * g) * (NC + 1) * 64;
            uint32_t* dtileB = dtileA + (int64_t)(NC + 1) * 64;
            const bool okA = ja <= a.L2, okB = jb <= a.L2;
            const int* tin = &tring[w * R * SLOT];
            int* tout = &tring[(w + 1) * R * SLOT];
            const int* cin = &ctr[2 * w + 1];          // {cons[w], prog[w], cons[w+1]}
            PairConst kc;
            kc.c2a = a.s2[ja - 1];
            kc.c2b = a.s2[jb - 1];
            kc.vcm = vcm;
            kc.vck = vck;
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                kc.kd[s] = -(s + 1) * d;
                asm volatile("" : "+v"(kc.kd[s]));     // keep the constants in VGPRs
            }
            asm volatile("" : "+v"(kc.c2a), "+v"(kc.c2b), "+v"(kc.vcm), "+v"(kc.vck));
            kc.pla = kc.pha = kc.plb = kc.phb = 0;
            if (PROF) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t ba = (uint32_t)((uint32_t)q == kc.c2a ? vcm : vck) & 0xffu;
                    const uint32_t bb = (uint32_t)((uint32_t)q == kc.c2b ? vcm : vck) & 0xffu;
                    if (q < 4) {
                        kc.pla |= ba << (8 * q);
                        kc.plb |= bb << (8 * q);
                    } else {
                        kc.pha |= ba << (8 * (q - 4));
                        kc.phb |= bb << (8 * (q - 4));
                    }
                }
            }
            kc.cb = lds_addr(&ctr[2 * w]);
            asm volatile("" : "+v"(kc.cb));
            // Ring writes of the block: lane 63 into the slot, the other lanes
            // into a per-lane dummy (conflict-free, no exec juggling).
            const int ring0 = lane == 63 ? lds_addr(tout) : lds_addr(&scratch[lane]);
            int ra[R], rd[R];
#pragma unroll
            for (int q = 0; q < R; ++q) {
                ra[q] = ring0 + q * SLOT * 4;
                rd[q] = lds_addr(tin) + q * SLOT * 4;
                asm volatile("" : "+v"(ra[q]), "+v"(rd[q]));
            }
            // column 0 (and the row above at column 0): G' = -(1 + row_base + 128*g0)*d
            const int C0 = -(1 + a.row_base + 128 * g0) * d;
            PairRegs r;
            r.ga = r.gb = r.sh = C0;
            r.gavA = r.gavB = 0;
            r.pq = 0;
            r.nloa = -(128 * w + 2 * lane) * d;       // H = G' + nlo - (s+1)d in chunk 0
            r.nlob = r.nloa - d;
            bool aborted = false;
            if (a.trace && lane == 0 && w == 0) {
                a.trace[8 * (int64_t)sidx + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * (int64_t)sidx + 4] = __builtin_amdgcn_s_memtime();
            }
            if (a.trace && lane == 0 && w == nw - 1) a.trace[8 * (int64_t)sidx + 6] = __builtin_amdgcn_s_memrealtime();
            // ---- the pipelined block's state (PIPE): `pend` = the chunk whose
            // column-7 flags, code words and scores of columns 4..7 are still
            // in registers (-1: none) ----
            r.qa1 = r.qb1 = v4i{0, 0, 0, 0};
            r.dga1 = r.dgb1 = 0;
            r.accA = r.accB = 0;
            int pend = -1;
            // byte offsets of this lane from the SGPR bases of the block's stores
            int voa = lane * 16, vob = voa + (int)((tileB - tileA) * 4);
            int vda = lane * 4, vdb = vda + (int)((dtileB - dtileA) * 4);
            asm volatile("" : "+v"(voa), "+v"(vob), "+v"(vda), "+v"(vdb));
            auto flush_pending = [&]() {
                if (PIPE && pend >= 0) {
                    auto eq = [](int x, int y) { return x == y ? 1u : 0u; };   // a candidate that attains the max
                    const int ga6 = r.qa1[2], ga7 = r.qa1[3], gb6 = r.qb1[2], gb7 = r.qb1[3];
                    const uint32_t accA = (r.accA << 3) | (eq(ga6, ga7) << 2) | (eq(r.sh, ga7) << 1) | eq(r.dga1, ga7);
                    const uint32_t accB = (r.accB << 3) | (eq(gb6, gb7) << 2) | (eq(ga7, gb7) << 1) | eq(r.dgb1, gb7);
                    __builtin_nontemporal_store(r.qa1, reinterpret_cast<v4i*>(tileA + (int64_t)pend * 512 + 256 + lane * 4));
                    __builtin_nontemporal_store(r.qb1, reinterpret_cast<v4i*>(tileB + (int64_t)pend * 512 + 256 + lane * 4));
                    __builtin_nontemporal_store(accA, dtileA + (int64_t)(pend + 1) * 64 + lane);
                    __builtin_nontemporal_store(accB, dtileB + (int64_t)(pend + 1) * 64 + lane);
                    r.ga = ga7;
                    r.gb = gb7;
                    pend = -1;
                }
            };
            auto rebase = [&](int c) {
                if (c > 0 && c % SUPER_CHUNKS == 0) {
                    flush_pending();
                    const int shv = SUPER_CHUNKS * CH * d;
                    r.ga -= shv;
                    r.gb -= shv;
                    r.sh -= shv;
                    r.nloa += shv;
                    r.nlob += shv;
                }
            };
            // ---- generic chunk (the last one: n = 1..8 columns) ----
            auto generic_chunk = [&](int c) -> bool {
                const int n = (c == NC - 1) ? nlast : CH;
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
                const uint64_t sym8 = (uint64_t)(uint32_t)slot[8] | ((uint64_t)(uint32_t)slot[9] << 32);
                lds_order();
                if (lane == 0) lds_publish(&ctr[2 * w + 1], c + 1);
                int* so = &tout[(c % R) * SLOT];
                int ha[CH], hb[CH];
                uint32_t accA = 0, accB = 0;
#pragma unroll
                for (int s = 0; s < CH; ++s) {
                    if (s < n) {
                        const uint32_t sym = (uint32_t)(sym8 >> (8 * s)) & 0xffu;
                        const int dga = r.sh + (sym == kc.c2a ? vcm : vck);
                        const int Xa = max(max(r.ga, dga), T[s]);
                        const int dgb = r.ga + (sym == kc.c2b ? vcm : vck);
                        const int Xb = max(max(r.gb, dgb), Xa);
                        const int Gbn = prefmax(Xb);
                        const int shn = shr1(T[s], Gbn);
                        const int Gan = max(Xa, shn);
                        const uint32_t ca = (dga == Gan ? 1u : 0u) | (shn == Gan ? 2u : 0u) | (r.ga == Gan ? 4u : 0u);
                        const uint32_t cb = (dgb == Gbn ? 1u : 0u) | (Gan == Gbn ? 2u : 0u) | (r.gb == Gbn ? 4u : 0u);
                        accA = (accA << 3) | ca;
                        accB = (accB << 3) | cb;
                        ha[s] = RAW ? Gan : Gan + r.nloa - (s + 1) * d;
                        hb[s] = RAW ? Gbn : Gbn + r.nlob - (s + 1) * d;
                        if (ST) {
                            r.gavA = max(r.gavA, ha[s] < 0 ? -ha[s] : ha[s]);
                            r.gavB = max(r.gavB, hb[s] < 0 ? -hb[s] : hb[s]);
                        }
                        if (lane == 63) so[s] = Gbn;
                        r.ga = Gan;
                        r.gb = Gbn;
                        r.sh = shn;
                    } else {
                        ha[s] = hb[s] = 0;
                    }
                }
                if (lane == 63) {                      // the chunk's symbols go down the ring (from
                    so[8] = (int)(uint32_t)sym8;       // registers: the input slot was released above)
                    so[9] = (int)(uint32_t)(sym8 >> 32);
                }
                if (n < CH) {
                    accA <<= 3 * (CH - n);
                    accB <<= 3 * (CH - n);
                }
                if (SH) {
                    pair_store_scores(ha, tileA + (int64_t)c * 512 + lane * 4);
                    pair_store_scores(hb, tileB + (int64_t)c * 512 + lane * 4);
                }
                if (SD) {
                    __builtin_nontemporal_store(accA, dtileA + (int64_t)(c + 1) * 64 + lane);
                    __builtin_nontemporal_store(accB, dtileB + (int64_t)(c + 1) * 64 + lane);
                }
                if (ST) {
                    bc += branch_codes(okA ? accA : 0u);
                    bc += branch_codes(okB ? accB : 0u);
                }
                if (!SH && c == NC - 1) {              // score-only: H[L1][*]
                    a.lastcol[ja] = ha[n - 1];
                    a.lastcol[jb] = hb[n - 1];
                }
                lds_order();
                if (lane == 0) lds_publish(&ctr[2 * w + 4], c + 1);
                r.nloa -= CH * d;
                r.nlob -= CH * d;
                return true;
            };
            // ---- full chunks: the generated block (nw_pair_chunk.inc) ----
            PairSlot tA, tB;
            auto wait_slot = [&](int c, PairSlot& tt) -> bool {
                for (;;) {
                    const uint64_t pq = pair_read_slot(kc.cb, rd[c % R], tt);
                    const int pin = uni((int)(uint32_t)pq), pout = uni((int)(pq >> 32));
                    if (pin > c && pout >= c - R + 1) return true;
                    if (uni(lds_ld(&sh_abort))) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            // (head: the first chunk of a run; mid: another full chunk follows --
            // constants at every call, so the checks they spare are compiled out)
            auto full_chunk = [&](int c, auto slotc, PairSlot& cur, PairSlot& nxt, bool head = false,
                                  bool mid = false) -> bool {
                constexpr int Q = decltype(slotc)::value;
                if constexpr (PIPE) {
                    // The block stores the pending chunk's second half and code
                    // words (the chunk before this one) and its own scores of
                    // columns 0..3.  With nothing pending those stores carry
                    // stale registers: they go to this chunk's own second half
                    // (rewritten by the next block or the flush, later in this
                    // wave's program order) and to the code tiles' padding row.
                    // (only a run's head chunk can have nothing pending)
                    const bool fresh = head && pend < 0;
                    const int32_t* hbs = tileA + (int64_t)c * 512;
                    const int32_t* hbp = fresh ? hbs : hbs - 512;
                    const uint32_t* dbp = fresh ? dtileA : dtileA + (int64_t)c * 64;
                    if (fresh) {
                        r.qa1[3] = r.ga;
                        r.qb1[3] = r.gb;
                    }
                    pair_chunk_pipe<PROF>(r, kc, cur, nxt, c + 1, ra[Q], rd[(Q + 1) % R], voa, vob, vda, vdb, hbs, hbp, dbp);
                    pend = c;
                    if (!mid && c + 2 >= NC) return true;
                    // (prog[w] > c + 1 and cons[w+1] >= c + 2 - R, as one sign test: the common case falls through)
                    if (__builtin_expect(((uni((int)(uint32_t)r.pq) - (c + 2)) | (uni((int)(r.pq >> 32)) - (c + 2 - R))) >= 0, 1))
                        return true;
                    return wait_slot(c + 1, nxt);
                } else if constexpr (RAW) {
                    pair_chunk_raw<SD, PROF>(r, kc, cur, nxt, c + 1, ra[Q], rd[(Q + 1) % R]);
                    r.ha[7] = r.ga;
                    r.hb[7] = r.gb;
                } else {
                    pair_chunk_asm<SH || ST, SD || ST, ST, PROF>(r, kc, cur, nxt, c + 1, ra[Q], rd[(Q + 1) % R]);
                }
                if (SH) {
                    pair_store_scores(r.ha, tileA + (int64_t)c * 512 + lane * 4);
                    pair_store_scores(r.hb, tileB + (int64_t)c * 512 + lane * 4);
                }
                if (SD) {
                    __builtin_nontemporal_store(r.accA, dtileA + (int64_t)(c + 1) * 64 + lane);
                    __builtin_nontemporal_store(r.accB, dtileB + (int64_t)(c + 1) * 64 + lane);
                }
                if (ST) {
                    bc += branch_codes(okA ? r.accA : 0u);
                    bc += branch_codes(okB ? r.accB : 0u);
                }
                if (!RAW) {
                    r.nloa -= CH * d;
                    r.nlob -= CH * d;
                }
                if (!mid && c + 2 >= NC) return true;  // the next chunk is the generic last one
                // (prog[w] > c + 1 and cons[w+1] >= c + 2 - R, as one sign test: the common case falls through)
                if (__builtin_expect(((uni((int)(uint32_t)r.pq) - (c + 2)) | (uni((int)(r.pq >> 32)) - (c + 2 - R))) >= 0, 1))
                    return true;
                return wait_slot(c + 1, nxt);
            };
            using S0 = std::integral_constant<int, 0>;
            using S1 = std::integral_constant<int, 1>;
            using S2 = std::integral_constant<int, 2>;
            using S3 = std::integral_constant<int, 3>;
            int c = 0;
            const int nfull = NC - 1;                  // chunks before the last one
            if (nfull > 0) aborted = !wait_slot(0, tA);
            while (c + R < nfull && !aborted) {
                rebase(c);
                // [8*NSW + g]: when this stripe reaches the middle of the table
                if (NW_TRACE_EXT && a.trace && lane == 0 && c == trace_mid_chunk(NC, R))
                    *trace_ext(a, TX_MID, g) = __builtin_amdgcn_s_memrealtime();
                aborted = !full_chunk(c, S0{}, tA, tB, true, true) || !full_chunk(c + 1, S1{}, tB, tA, false, true) ||
                          !full_chunk(c + 2, S2{}, tA, tB, false, true) || !full_chunk(c + 3, S3{}, tB, tA, false, true);
                c += R;
            }
            if (!aborted && c < nfull) {
                rebase(c);
                aborted = !full_chunk(c, S0{}, tA, tB, true);
                if (!aborted && c + 1 < nfull) aborted = !full_chunk(c + 1, S1{}, tB, tA);
                if (!aborted && c + 2 < nfull) aborted = !full_chunk(c + 2, S2{}, tA, tB);
                if (!aborted && c + 3 < nfull) aborted = !full_chunk(c + 3, S3{}, tB, tA);
                c = nfull;
            }
            if (!aborted) {
                flush_pending();
                rebase(c);
                aborted = !generic_chunk(c);
            }
            if (ST) gav = max(okA ? r.gavA : 0, okB ? r.gavB : 0);
        }
        if (a.trace && real && w == nw - 1 && lane == 0) {
            a.trace[8 * (int64_t)sidx + 2] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 5] = __builtin_amdgcn_s_memtime();
        }
        if (ST && real) {
            int gv = gav;
            uint32_t bv = bc;
            for (int o = 32; o > 0; o >>= 1) {
                gv = max(gv, __shfl_xor(gv, o));
                bv += __shfl_xor(bv, o);
            }
            if (lane == 0) {
                atomicMax(reinterpret_cast<int*>(&a.ctl[CTL_GAV]), gv);
                atomicAdd(&a.ctl[CTL_BC], bv);
            }
        }
        __syncthreads();
        if (sh_abort) break;
    }
}

template <int W, bool P>
KernelFn pick_flags(bool sh, bool sd, bool stt) {
    if (sh && sd) return stt ? nw_pair_kernel<W, true, true, true, P> : nw_pair_kernel<W, true, true, false, P>;
    if (sh) return stt ? nw_pair_kernel<W, true, false, true, P> : nw_pair_kernel<W, true, false, false, P>;
    if (sd) return stt ? nw_pair_kernel<W, false, true, true, P> : nw_pair_kernel<W, false, true, false, P>;
    return stt ? nw_pair_kernel<W, false, false, true, P> : nw_pair_kernel<W, false, false, false, P>;
}

template <int W>
KernelFn pick_prof(bool prof, bool sh, bool sd, bool stt) {
    return prof ? pick_flags<W, true>(sh, sd, stt) : pick_flags<W, false>(sh, sd, stt);
}

}  // namespace

KernelFn pick_pair(int W, bool prof, bool sh, bool sd, bool stt) {
    switch (W) {
        case 1: return pick_prof<1>(prof, sh, sd, stt);
        case 2: return pick_prof<2>(prof, sh, sd, stt);
        case 3: return pick_prof<3>(prof, sh, sd, stt);
        case 4: return pick_prof<4>(prof, sh, sd, stt);
        case 5: return pick_prof<5>(prof, sh, sd, stt);
        case 6: return pick_prof<6>(prof, sh, sd, stt);
        case 7: return pick_prof<7>(prof, sh, sd, stt);
        case 8: return pick_prof<8>(prof, sh, sd, stt);
        case 10: return pick_prof<10>(prof, sh, sd, stt);
        case 12: return pick_prof<12>(prof, sh, sd, stt);
        default: return nullptr;   // (W + 2 waves <= 16)
    }
}

}  // namespace nwk
