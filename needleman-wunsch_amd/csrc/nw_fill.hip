// nw_fill.hip -- MI355X (gfx950) Needleman-Wunsch score-table fill + C ABI.
//
// Replaces the reference hot path compute_table_scores()
// (needleman-wunsch.c:583-626 -> score_cell_column_set :557-574 ->
// score_cell_column :523-543 -> score_cell :418-510 -> max3 :395-404) and the
// table storage/seeding it relies on (score-table.c:60-81,
// walk-table.c:58-79, computation.c:75-125).  In short:
//
//  * A wave owns a 64-row stripe (lane l <-> row j0+l) and walks the columns
//    i = 1..L1.  All 64 lanes compute the SAME column per step, so the
//    vertical ("up") dependency H[i][j-1] is resolved by a max-plus prefix
//    scan over the lanes instead of a skewed wavefront:
//        H[i][j] = max_k<=j ( X_k - (j-k)*d ),  X_k = max(left_k, diag_k)
//    Working in the shifted domain G = H + r*d (r = row offset inside the
//    workgroup) turns it into a plain prefix MAX, done with six DPP
//    v_max_i32 (row_shr 1/2/4/8, row_bcast 15/31) -- no LDS, no skew, and
//    the column segment is written as one coalesced 256-byte store.
//  * A workgroup of W waves stacks W stripes; wave w runs one 8-column chunk
//    behind wave w-1 (barrier lockstep) and takes its top row through LDS.
//  * Workgroups take W*64-row "WG-stripes" from an atomic dequeue counter
//    and hand the bottom row of a WG-stripe to the next one through tagged
//    8-byte {tag, value} granules stored/loaded write-through (agent scope),
//    the hand-off form of the CDNA4 guide (Guideline 16, R2).
//  * Outputs: int32 scores (column-major, padded pitch), 4-bit direction
//    codes packed 8 columns per 32-bit word per lane (one coalesced 256-B
//    store per wave per chunk), optional stats.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nw_internal.h"
#include "nw_kern.h"

namespace {

using namespace nwk;

// Ring slot (scan kernel): 8 T' of a chunk + its 8 top-string bytes (2 words).
// In registers as the three vectors the block's wide LDS reads fill.


// ------------------------------------------------------------ column steps
// Domain.  A wave works on G' = H + r*d + (i - base)*d, r = row offset inside
// the workgroup (64*w + lane), i = column, base = the column where the current
// 4096-column "super-chunk" starts.  In it the left candidate H[i-1][j] - d is
// G'_{i-1} itself, the diagonal is wave_shr1(G'_{i-1}) + sub + 2d, and the up
// dependency becomes a prefix max over the lanes:
//     G'_i = prefmax( max3(G'_{i-1}, wave_shr1(G'_{i-1}) + sub'_i, T'_i) ),
//     sub' = match ? m + 2d : 2d - k,   T'_i = the row above, same domain.
// base moves every 512 chunks so |G'| stays within |H| + (64W + 4104)|d|.
// Cell recurrence = needleman-wunsch.c:429-465; direction flags :485-503.

struct RingSlot {
    v4i a, b;           // T' of steps 0..3, 4..7
    v2i c;              // top-string bytes of columns 1..4, 5..8 of the chunk
};

struct ChunkRegs {
    int g[6];           // out: G' after steps 0..5 (lane 63 -> the wave below)
    int gp6, gin;       // in: G' of the previous chunk's columns 7, 8; out: this chunk's
    int tm;             // in: T' of the previous column; out: T' of this chunk's last
    int dgA, dgB;       // diagonal candidates of even / odd steps (dgB: last step of a full chunk)
    int subA, subB;     // sub' of even / odd steps
    int h[8];           // out: H of steps 0..7 (partial chunks: the flush block adds the last)
    uint32_t accp;      // in: previous chunk's codes (missing the last); out: this chunk's so far
    uint32_t acc;       // out: previous chunk's complete codes word
    int gav;            // in/out: running max |H| (stats)
    uint64_t pq;        // out: {prog[w], cons[w+1]} read mid-chunk (NEXT blocks)
    int cv;             // in/out: chunk index + 1 (ring counter value of this chunk)
    int hv, dv;         // in/out: byte offsets of this lane in the score / code tiles
    int nlo;            // in/out: -(r*d) - (8c - base)*d: H = G' + nlo - (s+1)*d
};
struct ChunkConst {
    uint32_t c2;        // this lane's side-string byte
    int vcm, vck;       // sub' for match / mismatch
    int d8;             // 8*d (nlo step per chunk)
    int kd[8];          // -(s+1)*d
    int cb;             // LDS address of ctr[2w] (ring counters, see the kernel)
    int32_t* hb;        // score tile base (moves every super-chunk, with hv)
    uint32_t* db;       // code tile base (moves every super-chunk, with dv)
    uint32_t pl, ph;    // profile (P blocks): byte a = sub' of symbol code a (int8), a = 0..3 / 4..7
};

#include "nw_chunk.inc"

// Count 3-bit codes of a word (8 per word, bits 0..23) with >= 2 directions.
__device__ __forceinline__ uint32_t branch_codes(uint32_t x) {
    const uint32_t y = (x & (x >> 1)) | (x & (x >> 2)) | ((x >> 1) & (x >> 2));
    return __builtin_popcount(y & 0x249249u);
}

// G' of step s of the current chunk (steps 6, 7 live in the carried registers).
__device__ __forceinline__ int g_of(const ChunkRegs& r, int s) {
    switch (s) {
        case 0: return r.g[0];
        case 1: return r.g[1];
        case 2: return r.g[2];
        case 3: return r.g[3];
        case 4: return r.g[4];
        case 5: return r.g[5];
        case 6: return r.gp6;
        default: return r.gin;
    }
}

// The last chunk of a stripe (n = 1..8 columns): block + flush.  Returns H
// of the stripe's last column (for the score-only last column).
template <bool SH, bool SD, bool ST, bool P, int N>
__device__ __forceinline__ int run_last(ChunkRegs& r, const ChunkConst& k, RingSlot& t, int ra) {
    RingSlot n;
    chunk_asm<SH, SD, ST, P, N, false>(r, k, t, n, ra, 0);
    flush_asm<SH, SD, ST, N>(r, k, t, ra);
    if constexpr ((SH && !NW_SCORE_X4) || ST) return r.h[N - 1];
    else return g_of(r, N - 1) + r.nlo + k.kd[N - 1];
}
template <bool SH, bool SD, bool ST, bool P>
__device__ __forceinline__ int run_last_n(int n, ChunkRegs& r, const ChunkConst& k, RingSlot& t, int ra) {
    switch (n) {
        case 1: return run_last<SH, SD, ST, P, 1>(r, k, t, ra);
        case 2: return run_last<SH, SD, ST, P, 2>(r, k, t, ra);
        case 3: return run_last<SH, SD, ST, P, 3>(r, k, t, ra);
        case 4: return run_last<SH, SD, ST, P, 4>(r, k, t, ra);
        case 5: return run_last<SH, SD, ST, P, 5>(r, k, t, ra);
        case 6: return run_last<SH, SD, ST, P, 6>(r, k, t, ra);
        case 7: return run_last<SH, SD, ST, P, 7>(r, k, t, ra);
        default: return run_last<SH, SD, ST, P, 8>(r, k, t, ra);
    }
}

// Slow path of the ring: this wave's {prog, cons} counter pair, then the
// ring slot at LDS address rd (LDS is in order per wave: slot data read after
// a progress value that covers it is valid).  Same registers as the block's
// own reads of the next slot, and waited for here.
__device__ __forceinline__ uint64_t read_slot(int cb, int rd, RingSlot& s) {
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

#if NW_SCORE_X4
// Scores of one chunk from C++ (H = G' + nlo + kd, 8 v_add3): two 16-byte
// stores per lane into the quad tile (see score_index), 2 KB per wave.
__device__ __forceinline__ void store_chunk_scores(const ChunkRegs& r, const ChunkConst& k, int nl, bool have_h) {
    v4i qa, qb;
    if (have_h) {
        qa = v4i{r.h[0], r.h[1], r.h[2], r.h[3]};
        qb = v4i{r.h[4], r.h[5], r.h[6], r.h[7]};
    } else {
        qa = v4i{r.g[0] + nl + k.kd[0], r.g[1] + nl + k.kd[1], r.g[2] + nl + k.kd[2], r.g[3] + nl + k.kd[3]};
        qb = v4i{r.g[4] + nl + k.kd[4], r.g[5] + nl + k.kd[5], r.gp6 + nl + k.kd[6], r.gin + nl + k.kd[7]};
    }
    const int hv = r.hv;
    asm volatile(
        "global_store_dwordx4 %[hv], %[qa], %[hb]" NW_SCORE_HINT "\n\t"
        "global_store_dwordx4 %[hv], %[qb], %[hb] offset:1024" NW_SCORE_HINT
        :
        : [hv] "v"(hv), [qa] "v"(qa), [qb] "v"(qb), [hb] "s"(k.hb)
        : "memory");
}
#endif


// Workgroup = W compute waves (64-row stripes, stacked) + 1 loader wave, no
// barriers inside a stripe.  Wave w takes the top row of each 8-column chunk
// (and the chunk's top-string bytes) from an LDS ring tring[w] (R chunk
// slots) filled by its producer (the loader for w = 0, wave w-1 otherwise)
// and puts its own bottom row into tring[w+1].  Ring counters, interleaved so
// that a wave reads both of its own in one 8-byte LDS read:
//     ctr[2v+2] = prog[v]: chunks available in tring[v],
//     ctr[2v+1] = cons[v]: chunks wave v has taken out of tring[v]
// (cons of a wave that does not exist = "infinite").  A producer only waits
// when it is R chunks ahead.  The chunk block (nw_chunk.inc) issues all of a
// chunk's LDS traffic itself, including the next slot's reads; the C++ below
// only checks the progress values it read.  The loader feeds tring[0] from
// the previous WG-stripe's granules; it issues no stores, so its waits on the
// hand-off loads are exact, and the compute waves never wait on vmcnt.
// Granules (between workgroups and panels) carry H - d of the row above in
// the plain domain; ring slots carry G'.
template <int W, bool SH, bool SD, bool ST, bool PROF>
__global__ __launch_bounds__(64 * (W + 2)) void nw_fill_kernel(FillArgs a) {
    constexpr int R = 4;
    constexpr bool F = SD || ST;     // direction codes
    constexpr int NOCONS = 1 << 30;
    __shared__ __attribute__((aligned(16))) int tring[(W + 1) * R * SLOT];
    // Dummy target of the ring writes of lanes 0..62: lane-contiguous, so a
    // ds_write_b32 of the whole wave is bank-conflict free (an 8-dword lane
    // stride made every ring write a 16-way conflict).
    __shared__ int scratch[64 + R * SLOT];
    __shared__ __attribute__((aligned(8))) int ctr[2 * W + 4];
    __shared__ int sh_sidx;
    __shared__ int sh_abort;

    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6);
    const bool loader = (w == W);          // feeds ring 0
    const bool pubw = (w == W + 1);        // drains the last compute wave's ring into granules
    const int d = a.d;
    int vcm = a.m + 2 * a.d;
    int vck = 2 * a.d - a.k;
    const int NC = a.NC;
    const int nlast = a.L1 - CH * (NC - 1);   // steps in the last chunk (1..8)

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
        const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - g0);  // its stripes (<= W)
        const int g = g0 + w;                      // wave stripe (compute waves)
        const bool real = w < nw;                  // (the loader and the publisher are waves W, W+1)
        const int j0 = 1 + 64 * g;                 // first row of the wave stripe
        const int jrow = j0 + lane;
        int gav = 0;
        uint32_t bc = 0;

        if (pubw) {
            // ---------------- publisher wave ----------------
            // Drains the ring below the last compute wave into this
            // WG-stripe's bottom-row granules (for the next WG-stripe, or the
            // panel below), so the hand-off stores stay off the compute waves
            // (the stripe chain would otherwise move at the pace of each
            // WG-stripe's publishing wave).
            const bool publish = sidx + 1 < a.NSW;
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
            // (profiles/r02e_ab_chain_issue.txt; as nw_pair.hip).
            cd = uni(cd);
            const uint32_t tag = publish ? a.gtag | (uint32_t)(sidx + 1) : a.epoch;
            gu64* const gdst = (gu64*)(publish ? gout : a.xout);
            // (plain domain: H - d = G' - 128*nw*d - (i - base)d, i = CH*cd + lane + 1)
            int nklane = -(64 * nw * d + (lane + 1) * d);
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
            }
        } else if (loader) {
            // ---------------- loader wave: no stores, exact waits ----------------
            // Source of the WG-stripe's top row: the seeded row 0, the panel
            // above (xin, written by another agent: system-scope loads), or
            // the previous WG-stripe's granules (agent scope).  Lanes 8k..8k+7
            // write chunk cw + k's row above and its top-string words.
            // Nothing it waits for per chunk is a fresh global load unless the
            // granules are not there yet: the granule window (8 chunks, one lane
            // per granule) and the top-string window (2 dwords per chunk) are
            // prefetched one window ahead; a per-chunk
            // dependent load made the loader, not the producer, pace every
            // WG-stripe hop (+11% at 100k^2, tools/trace_lag.py).  Kept inline:
            // the same loop as a shared __device__ function compiled 5-10%
            // slower at 100k^2 (profiles/r02_ab_loader.txt; nw_pair.hip has the same loop).
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
            // ---------------- compute wave: its 64-row stripe, chunk by chunk ----
            int32_t* tile = a.H + (int64_t)g * a.spitch;
            // codes: row q+1 of the stripe's code tile holds chunk q (row 0 pads
            // the block's store of the word "before" chunk 0)
            uint32_t* dtile = a.D + (int64_t)g * (NC + 1) * 64;
            const bool out_lane = jrow <= a.L2;
            const int* tin = &tring[w * R * SLOT];
            const int* tout = &tring[(w + 1) * R * SLOT];
            ChunkConst kc;
            kc.c2 = a.s2[jrow - 1];
            asm volatile("" : "+v"(vcm), "+v"(vck));   // VGPR operands of v_cndmask
            kc.vcm = vcm;
            kc.vck = vck;
            kc.d8 = CH * d;
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                kc.kd[s] = -(s + 1) * d;
                asm volatile("" : "+v"(kc.kd[s]));     // keep the constants in VGPRs
            }
            kc.cb = lds_addr(&ctr[2 * w]);
            asm volatile("" : "+v"(kc.cb));
            kc.hb = tile;
            kc.db = dtile;
            // Profile (sequences coded 0..7 on the host): sub' of every
            // symbol for this lane's side symbol, one int8 per code; a v_perm
            // with the chunk's codes as selector looks up 4 columns at once.
            kc.pl = kc.ph = 0;
            if (PROF) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t b = (uint32_t)((uint32_t)q == kc.c2 ? vcm : vck) & 0xffu;
                    if (q < 4) kc.pl |= b << (8 * q);
                    else kc.ph |= b << (8 * (q - 4));
                }
            }
            ChunkRegs r;
            // column 0: H[0][j] = -j*d (computation.c:112-120) -> G' = -(1 + row_base + 64*g0)*d
            r.gin = -(1 + a.row_base + 64 * g0) * d;
            r.gp6 = r.gin;
            r.tm = r.gin;
            r.dgA = r.dgB = 0;
            r.subA = r.subB = 0;
            r.accp = 0;
            r.gav = 0;
            r.pq = 0;
            r.cv = 1;
            r.hv = NW_SCORE_X4 ? lane * 16 : lane * 4;
            r.dv = lane * 4;
            r.nlo = -(64 * w + lane) * d;
            // Ring writes: lane 63 into the slot, the other lanes into a
            // per-lane dummy, so no exec juggling per chunk.  One address per
            // ring slot (the chunk loop is unrolled by R).
            const int ring0 = lane == 63 ? lds_addr(tout) : lds_addr(&scratch[lane]);
            int ra[R], rd[R];
#pragma unroll
            for (int q = 0; q < R; ++q) {
                ra[q] = ring0 + q * SLOT * 4;
                rd[q] = lds_addr(tin) + q * SLOT * 4;
                asm volatile("" : "+v"(ra[q]), "+v"(rd[q]));
            }
            if (a.trace && lane == 0 && w == 0) {
                a.trace[8 * (int64_t)sidx + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * (int64_t)sidx + 4] = __builtin_amdgcn_s_memtime();
            }
            const bool trace_start = a.trace && lane == 0 && w == nw - 1;   // [6]: last wave's first block
            RingSlot tA, tB;
            // Slow path: wait until chunk c's ring slot is filled and our
            // consumer has room, re-reading the slot with every progress read.
            auto wait_slot = [&](int c, int rdq, RingSlot& tt) -> bool {
                for (int spins = 0;; ++spins) {
                    const uint64_t pq = read_slot(kc.cb, rdq, tt);
                    const int pin = uni((int)(uint32_t)pq), pout = uni((int)(pq >> 32));
                    if (pin > c && pout >= c - R + 1) return true;
                    if (uni(lds_ld(&sh_abort))) return false;
                    if (spins > 64) __builtin_amdgcn_s_sleep(1);
                }
            };
            auto rebase = [&](int c) {
                if (c > 0 && c % SUPER_CHUNKS == 0) {
                    // new super-chunk: rebase the carried G' values (and nlo) and
                    // move the tile bases so the lane offsets stay small
                    const int sh = SUPER_CHUNKS * CH * d;
                    r.gin -= sh;
                    r.gp6 -= sh;
                    r.dgB -= sh;
                    r.tm -= sh;
                    r.nlo += sh;
                    kc.hb += SUPER_CHUNKS * CH * 64;
                    r.hv -= SUPER_CHUNKS * CH * 64 * 4;
                    kc.db += SUPER_CHUNKS * 64;
                    r.dv -= SUPER_CHUNKS * 64 * 4;
                }
            };
            // After chunk c's block: stats of the previous chunk's codes,
            // the last chunk's code word, and the WG-stripe's bottom row
            // (last wave) out to the next WG-stripe / panel.
            auto after_chunk = [&](int c, int slot, int n, bool last) {
                if (ST && c > 0) bc += branch_codes(out_lane ? r.acc : 0u);
                if (F && last) {
                    const uint32_t dw = r.accp << (3 * (CH - n));
                    if (SD) dtile[(int64_t)(c + 1) * 64 + lane] = dw;
                    if (ST) bc += branch_codes(out_lane ? dw : 0u);
                }
                (void)slot;
            };
            // One full (non-final) chunk; SLOTC = c % R is a compile-time ring
            // slot.  The block reads the next slot into nxt; the slow path
            // re-reads it when the progress values it saw were too early.
            auto full_chunk = [&](int c, auto slotc, RingSlot& cur, RingSlot& nxt) -> bool {
                constexpr int Q = decltype(slotc)::value;
                constexpr int NQ = (Q + 1) % R;
#if NW_SCORE_X4
                const int nl = r.nlo;
#endif
                chunk_asm<SH, SD, ST, PROF, 8, true>(r, kc, cur, nxt, ra[Q], rd[NQ]);
#if NW_SCORE_X4
                if (SH) {
                    store_chunk_scores(r, kc, nl, ST);
                    r.hv += CH * 64 * 4;
                }
#endif
                after_chunk(c, Q, CH, false);
                // (wave-uniform: every lane read the same counters)
                // (prog[w] > c + 1 and cons[w+1] >= c + 2 - R, as one sign test: the common case falls through)
                if (__builtin_expect(((uni((int)(uint32_t)r.pq) - (c + 2)) | (uni((int)(r.pq >> 32)) - (c + 2 - R))) >= 0, 1))
                    return true;
                return wait_slot(c + 1, rd[NQ], nxt);
            };
            using S0 = std::integral_constant<int, 0>;
            using S1 = std::integral_constant<int, 1>;
            using S2 = std::integral_constant<int, 2>;
            using S3 = std::integral_constant<int, 3>;
            int c = 0;
            const int nfull = NC - 1;              // chunks before the last one
            bool aborted = !wait_slot(0, rd[0], tA);
            if (trace_start) a.trace[8 * (int64_t)sidx + 6] = __builtin_amdgcn_s_memrealtime();
            while (c + R <= nfull && !aborted) {
                rebase(c);
                aborted = !full_chunk(c, S0{}, tA, tB) || !full_chunk(c + 1, S1{}, tB, tA) ||
                          !full_chunk(c + 2, S2{}, tA, tB) || !full_chunk(c + 3, S3{}, tB, tA);
                c += R;
            }
            if (!aborted && c < nfull) {
                rebase(c);
                aborted = !full_chunk(c, S0{}, tA, tB);
                if (!aborted && c + 1 < nfull) aborted = !full_chunk(c + 1, S1{}, tB, tA);
                if (!aborted && c + 2 < nfull) aborted = !full_chunk(c + 2, S2{}, tA, tB);
                c = nfull;
            }
            // the last chunk (n = 1..8 columns), ring slot known only at run
            // time: re-read into tA (whichever array the loop left it in)
            if (!aborted && wait_slot(c, lds_addr(tin) + (c % R) * SLOT * 4, tA)) {
                rebase(c);
                const int slot = c % R;
#if NW_SCORE_X4
                const int nl = r.nlo;
#endif
                const int hl = run_last_n<SH, SD, ST, PROF>(nlast, r, kc, tA, ring0 + slot * SLOT * 4);
#if NW_SCORE_X4
                // (columns past the last one land in the tile's own padding)
                if (SH) store_chunk_scores(r, kc, nl, ST);
#endif
                if (!SH) a.lastcol[j0 + lane] = hl;   // score-only: H[L1][*]
                after_chunk(c, slot, nlast, true);
            }
            gav = r.gav;
        }
        if (a.trace && real && w == nw - 1 && lane == 0) {
            a.trace[8 * (int64_t)sidx + 2] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 5] = __builtin_amdgcn_s_memtime();
        }
        if (ST && real) {
            const bool rowok = jrow <= a.L2;
            int gv = rowok ? gav : 0;
            uint32_t bv = rowok ? bc : 0u;
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

// Mark granules [0, n) of a panel boundary as "the producer failed this fill".
__global__ void nw_poison_kernel(uint64_t* p, int64_t n, uint32_t epoch) {
    const uint64_t g = ((uint64_t)(epoch | POISON_BIT) << 32);
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + x, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Dense i-major copy of columns [i0, i1): out[(i-i0)*(L2+1) + j].
__global__ void nw_gather_scores_kernel(TableView v, int32_t L2, int64_t i0, int64_t i1, int32_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t n = (i1 - i0) * N;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = score_at(v, i0 + x / N, x % N);
}

// Dense nibble packing for nw_fill(): byte b = code(2b) | code(2b+1) << 4.
__global__ void nw_pack_nibbles_kernel(TableView v, int32_t L1, int32_t L2, uint8_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t ncell = ((int64_t)L1 + 1) * N;
    const int64_t nbyte = (ncell + 1) / 2;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbyte;
         b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c0 = 2 * b, c1 = 2 * b + 1;
        uint32_t x = code_at(v, c0 / N, c0 % N);
        if (c1 < ncell) x |= code_at(v, c1 / N, c1 % N) << 4;
        out[b] = (uint8_t)x;
    }
}

// One code byte per cell for columns [i0, i1).
__global__ void nw_codes_kernel(TableView v, int32_t L2, int64_t i0, int64_t i1, uint8_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t n = (i1 - i0) * N;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = (uint8_t)code_at(v, i0 + x / N, x % N);
}

// Per-column FNV-1a-64 of scores (int32 LE bytes) and codes (1 byte/cell)
// over rows j0..L2, continuing from the states in hcol / dcol (in place).  A
// whole table starts every column at the FNV offset basis with j0 = 0; a row
// panel continues the panel above's states from its first own row (j0 = 1).
__global__ void nw_colhash_kernel(TableView v, int32_t L1, int32_t L2, int32_t j0, uint64_t* hcol, uint64_t* dcol) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i > L1) return;
    const uint64_t P = 0x100000001b3ULL;
    uint64_t h = hcol[i], e = dcol[i];
    for (int64_t j = j0; j <= L2; ++j) {
        const uint32_t x = (uint32_t)score_at(v, i, j);
        h = (h ^ (x & 0xff)) * P;
        h = (h ^ ((x >> 8) & 0xff)) * P;
        h = (h ^ ((x >> 16) & 0xff)) * P;
        h = (h ^ (x >> 24)) * P;
        if (v.D) e = (e ^ code_at(v, i, j)) * P;
    }
    hcol[i] = h;
    dcol[i] = e;
}

// --------------------------------------------------------------- host side

template <int W, bool P>
KernelFn pick_flags(bool sh, bool sd, bool stt) {
    if (sh && sd) return stt ? nw_fill_kernel<W, true, true, true, P> : nw_fill_kernel<W, true, true, false, P>;
    if (sh) return stt ? nw_fill_kernel<W, true, false, true, P> : nw_fill_kernel<W, true, false, false, P>;
    if (sd) return stt ? nw_fill_kernel<W, false, true, true, P> : nw_fill_kernel<W, false, true, false, P>;
    return stt ? nw_fill_kernel<W, false, false, true, P> : nw_fill_kernel<W, false, false, false, P>;
}

template <int W>
KernelFn pick_prof(bool prof, bool sh, bool sd, bool stt) {
    return prof ? pick_flags<W, true>(sh, sd, stt) : pick_flags<W, false>(sh, sd, stt);
}

KernelFn pick_kernel(int W, bool prof, bool sh, bool sd, bool stt) {
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
        default: return nullptr;   // (W + loader + publisher <= 16 waves)
    }
}

// Resident fill workgroups per CU (the grid is at most this many per CU; one
// granule slot each, + 1).  Every plan that needs more than one WG-stripe per
// CU runs W >= 8 compute waves (+ loader + publisher), 1-2 workgroups per CU.
constexpr int kMaxWgPerCu = 4;

// Compute waves per workgroup (+1 loader wave; 16 waves = 1024 threads max).
const int kWaveChoices[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 15};

// How the NG stripes become workgroup stripes.  pack4 (scan and pair
// kernels): while every SIMD can have its own compute wave (NG <= 4 per CU),
// WG-stripes of 4 stripes (3 or 4, dealt evenly), even if CUs stay idle:
// a hop inside a workgroup costs ~0.7 us against 3-5 us through granules, and
// a fifth wave would double up a SIMD (profiles/r02_ab_loader.txt: 10k^2
// 1.10 -> 0.90 ms, 100k x 12.5k 7.06 -> 6.57 ms, 100k x 25k 7.20 -> 6.98 ms,
// 100k^2 pair 9.54 -> 9.45 ms).  Otherwise one WG-stripe per CU when that
// takes at most wmax waves, the stripes dealt as evenly as possible (SQ or
// SQ+1 each); beyond that fixed wfix-stripe WG-stripes taken in turn from the
// dequeue.
struct StripePlan {
    int W;              // kernel's compute waves per workgroup
    int64_t NSW;        // WG-stripes
    int SQ, SR;         // see FillArgs
};

// wmax: the most compute waves the kernel takes (the pair kernel adds a
// publisher wave to the loader, so it stops at 12); wfix: the WG-stripe
// height of the dequeued plan.
StripePlan plan_stripes(int64_t NG, int ncu, int wmax = 15, int wfix = 8, bool pack4 = false) {
    StripePlan p{wfix, (NG + wfix - 1) / wfix, wfix, 0};
    if (const char* e = getenv("NW_WAVES")) {
        const int w = atoi(e);
        for (int c : kWaveChoices)
            if (c == w && c <= wmax) return StripePlan{w, (NG + w - 1) / w, w, 0};
    }
    if (pack4 && NG <= 4 * (int64_t)ncu) {
        const int W = (int)std::min<int64_t>(4, NG);
        const int64_t NSW = (NG + W - 1) / W;
        return StripePlan{W, NSW, (int)(NG / NSW), (int)(NG % NSW)};
    }
    if (NG <= ncu) return StripePlan{1, NG, 1, 0};
    const int SQ = (int)(NG / ncu), SR = (int)(NG % ncu);
    const int need = SQ + (SR > 0);
    for (int c : kWaveChoices)
        if (c >= need && c <= wmax) return StripePlan{c, ncu, SQ, SR};
    return p;
}


double host_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- Host I/O
// Streamed slice copies.  A slice of columns [i0, i1)
// is gathered into dense column blocks of <= kStageBytes by a kernel on the
// table's stream, alternating between two device staging buffers, while the
// copy stream DMAs the previous block out: into the destination itself when
// it is pinned, else into one of two pinned bounce buffers that the host then
// copies out while the next DMA runs.
constexpr size_t kStageBytes = (size_t)64 << 20;

void release_io(nw_table* t) {
    if (t->copy_stream) (void)hipStreamSynchronize(t->copy_stream);
    for (auto& b : t->d_stage) {
        (void)hipFree(b);
        b = nullptr;
    }
    for (auto& b : t->h_stage) {
        if (b) (void)hipHostFree(b);
        b = nullptr;
    }
    t->stage_bytes = 0;
    for (auto& e : t->cev) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    if (t->copy_stream) (void)hipStreamDestroy(t->copy_stream);
    t->copy_stream = nullptr;
    if (t->h_seq) (void)hipHostFree(t->h_seq);
    t->h_seq = nullptr;
    t->h_seq_bytes = 0;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t at{};
    const hipError_t e = hipPointerGetAttributes(&at, p);
    (void)hipGetLastError();            // a pageable pointer is an error here, not a failure
    return e == hipSuccess && at.type == hipMemoryTypeHost;
}

template <class Gather>
int stream_columns(nw_table* t, int64_t i0, int64_t i1, size_t col_bytes, uint8_t* dst, Gather gather,
                   const char* who) {
    const double t0 = host_ms();
    const size_t stage = std::max(kStageBytes, col_bytes);
    const bool pinned = is_pinned(dst);
    if (t->stage_bytes < stage || (!pinned && !t->h_stage[0])) {
        for (auto& b : t->d_stage) {
            (void)hipFree(b);
            b = nullptr;
        }
        for (auto& b : t->h_stage) {
            if (b) (void)hipHostFree(b);
            b = nullptr;
        }
        t->stage_bytes = 0;
        for (auto& b : t->d_stage) NW_HIPCHK(hipMalloc(&b, stage));
        if (!pinned)
            for (auto& b : t->h_stage) NW_HIPCHK(hipHostMalloc(&b, stage, hipHostMallocDefault));
        t->stage_bytes = stage;
    }
    if (!t->copy_stream) NW_HIPCHK(hipStreamCreateWithFlags(&t->copy_stream, hipStreamNonBlocking));
    for (auto& e : t->cev)
        if (!e) NW_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const int64_t per = std::max<int64_t>(1, (int64_t)(t->stage_bytes / col_bytes));
    const int64_t nb = (i1 - i0 + per - 1) / per;
    hipEvent_t* gathered = &t->cev[0];
    hipEvent_t* copied = &t->cev[2];
    hipError_t e = hipSuccess;
    auto host_out = [&](int64_t b) {      // bounce path: block b is in h_stage[b & 1]
        const int64_t c0 = i0 + b * per, c1 = std::min(i1, c0 + per);
        if (e == hipSuccess) e = hipEventSynchronize(copied[b & 1]);
        if (e == hipSuccess)
            std::memcpy(dst + (size_t)(c0 - i0) * col_bytes, t->h_stage[b & 1], (size_t)(c1 - c0) * col_bytes);
    };
    for (int64_t b = 0; b < nb && e == hipSuccess; ++b) {
        const int k = (int)(b & 1);
        const int64_t c0 = i0 + b * per, c1 = std::min(i1, c0 + per);
        const size_t bytes = (size_t)(c1 - c0) * col_bytes;
        if (b >= 2) e = hipStreamWaitEvent(t->stream, copied[k], 0);   // d_stage[k] drained (block b-2)
        if (e == hipSuccess) {
            gather(c0, c1, t->d_stage[k]);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(gathered[k], t->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(t->copy_stream, gathered[k], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(pinned ? dst + (size_t)(c0 - i0) * col_bytes : t->h_stage[k], t->d_stage[k], bytes,
                               hipMemcpyDeviceToHost, t->copy_stream);
        if (e == hipSuccess) e = hipEventRecord(copied[k], t->copy_stream);
        if (!pinned && b >= 1) host_out(b - 1);   // overlaps block b's gather + DMA
    }
    if (!pinned && nb >= 1 && e == hipSuccess) host_out(nb - 1);
    if (e == hipSuccess) e = hipStreamSynchronize(t->copy_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    if (e != hipSuccess) return nwi::fail(NW_ERR_HIP, std::string(who) + ": " + hipGetErrorString(e));
    t->copy_ms = host_ms() - t0;
    t->copy_bytes = (int64_t)((size_t)(i1 - i0) * col_bytes);
    return NW_OK;
}

}  // namespace

namespace nwk {

TableView view_of(const nw_table* t) {
    TableView v{};
    v.tiles = t->H;
    v.spitch = t->spitch;
    v.D = (t->last_mask & NW_OUT_DIRS) ? t->D : nullptr;
    v.NC = (int32_t)t->lay_NC;
    v.skew = t->skew;
    v.pair = t->pair;
    v.raw = t->raw;
    v.SQ = t->SQ;
    v.SR = t->SR;
    v.d = t->last_d;
    v.row_base = (int32_t)t->row_base;
    v.top = t->row_base > 0 ? t->row0 : nullptr;
    return v;
}

}  // namespace nwk

namespace nwi {

thread_local std::string g_last_error;

int fail(int rc, const std::string& msg) {
    g_last_error = msg;
    return rc;
}

int fill_launch(nw_table* t, int32_t m, int32_t k, int32_t d, uint32_t out_mask) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_fill: NULL table");
    if (t->L1 < 0) return fail(NW_ERR_STATE, "nw_table_fill: no sequences set");
    if (t->launched) return fail(NW_ERR_STATE, "nw_table_fill: a fill is already in flight");
    if ((out_mask & ~t->cap_mask & (NW_OUT_SCORES | NW_OUT_DIRS)) != 0)
        return fail(NW_ERR_ARG, "nw_table_fill: output not allocated at creation");
    // Overflow guard: |H| <= (L1+L2)*max(|m|,|k|,|d|); the kernel's shifted
    // domain adds r*d + (i - base)*d <= (64*16 + 4096 + 8)*|d| and one more
    // candidate term (sub' = m + 2d or 2d - k).
    {
        const int64_t M = std::max({std::llabs(m), std::llabs(k), std::llabs(d)});
        const int64_t L2g = t->L2_total >= 0 ? t->L2_total : t->L2;
        const int64_t bound = (t->L1 + L2g) * M + 6144 * std::llabs(d) + 4 * M + 2;
        if (bound >= (int64_t)INT32_MAX)
            return fail(NW_ERR_RANGE, "nw_table_fill: |scores| could reach " + std::to_string(bound));
    }
    NW_HIPCHK(hipSetDevice(t->device));
    const bool sh = out_mask & NW_OUT_SCORES, sd = out_mask & NW_OUT_DIRS, stt = out_mask & NW_OUT_STATS;
    const int64_t L1 = t->L1, L2 = t->L2;
    const bool panel = t->xin || t->xout;
    t->filled = false;
    NW_HIPCHK(hipEventRecord(t->ev[0], t->stream));
    NW_HIPCHK(hipMemsetAsync(t->ctl, 0, CTL_WORDS * 4, t->stream));
    int W = 0;
    bool skew = false, pair = false, quad = false, autosel = false;
    int32_t pSQ = 0, pSR = 0;
    if (L1 > 0 && L2 > 0) {
        StripePlan plan = plan_stripes(t->NG, t->ncu, 12);
        W = plan.W;
        // Profile lookups when the sequences were coded to <= 8 symbols and
        // sub' fits a signed byte ($NW_PROF=0 forces the byte compares).
        const int64_t vcm = (int64_t)m + 2 * (int64_t)d, vck = 2 * (int64_t)d - k;
        const char* pe = getenv("NW_PROF");
        const bool prof = t->alpha > 0 && vcm >= -128 && vcm <= 127 && vck >= -128 && vck <= 127 &&
                          !(pe && atoi(pe) == 0);
        // Kernel: the column scan (nw_fill_kernel) or the skewed-stripe
        // wavefront (nw_skew.hip); they write different tile layouts
        // (TableView.skew).  The skew kernel's critical path is L1 + 72*NG
        // steps of ~110 cycles, the scan's L1 steps of ~150-230 cycles plus
        // ~1.2 us per stripe, so the skew kernel wins only on very wide tables
        // with few stripes (measured: 1M x 20k 61 vs 75 ms, 100k x 64 4.6 vs
        // 6.2 ms; 100k x 12.5k 8.0 vs 7.0 ms and 100k x 100k 22 vs 11 ms the
        // other way).  $NW_KERNEL = scan | skew | pair | quad | auto (default).
        const char* ke = getenv("NW_KERNEL");
        if (ke && std::strcmp(ke, "skew") == 0) skew = true;
        else if (ke && std::strcmp(ke, "scan") == 0) skew = false;
        else if (ke && std::strcmp(ke, "pair") == 0) pair = true;
        else if (ke && std::strcmp(ke, "quad") == 0) quad = true;
        else {
            // auto (profiles/r01_ab_skew_vs_scan_shapes.txt,
            // r01_ab_kernels_after_publisher.txt, r01_ab_pair_scoreonly.txt):
            // the pair kernel once the 64-row stripes outnumber the SIMDs (the
            // scan kernel then doubles up waves and runs at the two-wave
            // rate); the skew kernel for wide tables with few stripes; the
            // scan kernel otherwise.
            // (skew from L1 >= 32*L2: it won at 100k x 64 and 1M x 20k, lost
            // at 100k x 12.5k -- an 8-GPU row panel -- 8.03 vs 7.04 ms,
            // profiles/r02_ab_loader.txt)
            // (quad instead of scan wherever the fill needs no stats:
            // 100k x 12.5k 6.46 -> 5.92 ms, 100k x 50k 7.23 -> 6.92 ms, 10k^2
            // equal, profiles/r03m_ab_quad.txt)
            const int64_t simds = 4 * (int64_t)t->ncu;
            pair = t->NG > simds;
            // (against the quad kernel the skew kernel only wins on a single
            // stripe: 100k x 64 4.54 vs 5.15 ms, but 100k x 256 5.73 vs 5.16,
            // 1M x 20k 61.1 vs 53.2 ms, profiles/r05l_ab_skew_vs_quad.txt; fills
            // with stats choose between skew and scan as before)
            skew = !pair && t->NG <= simds && L1 >= 32 * L2 && (stt || t->NG == 1);
            autosel = true;
        }
        // a feeding panel's last row must be lane 63's row b of its last pair stripe
        if (pair && t->xout && L2 % 128 != 0) pair = false;
        if (autosel && !pair && !skew) quad = true;
        // The quad kernel (nw_quad.hip) has no stats variant and works in
        // G' = H + r*d + i*d without a moving column base: fall back to the
        // scan kernel where that could leave int32.
        if (quad) {
            const int64_t M = std::max({std::llabs(m), std::llabs(k), std::llabs(d)});
            const int64_t L2g = t->L2_total >= 0 ? t->L2_total : t->L2;
            if (stt || (t->L1 + L2g) * M + (L1 + 2048) * std::llabs(d) + 4 * M + 2 >= (int64_t)INT32_MAX) quad = false;
        }
        if (!skew && !pair) {
            plan = plan_stripes(t->NG, t->ncu, 12, 8, true);
            W = plan.W;
        }
        if (quad && !pick_quad(W, prof, sh, sd)) quad = false;   // (a wave count it is not built for)
        const int64_t NGk = pair ? (L2 + 127) / 128 : t->NG;
        if (pair) {
            // Dequeued WG-stripes (more than 15 pair stripes per CU): 12 high
            // for score-only fills, whose block fits 128 VGPRs, so three
            // compute waves share a SIMD (1M^2: 268 vs 292 ms at 8 high,
            // profiles/r02_ab_loader.txt); 8 when the block also makes
            // scores / codes (it would spill at 12).
            plan = plan_stripes(NGk, t->ncu, 12, (sh || sd || stt) ? 8 : 12, true);
            W = plan.W;
        }
        KernelFn fn = skew ? pick_skew(W, prof, sh, sd, stt)
                           : pair ? pick_pair(W, prof, sh, sd, stt)
                                  : quad ? pick_quad(W, prof, sh, sd) : pick_kernel(W, prof, sh, sd, stt);
        if (!fn) return fail(NW_ERR_ARG, "nw_table_fill: unsupported wave count");
        // chunks of 8 steps per stripe (quad: row group q runs q columns behind)
        const int64_t NCH = skew ? (L1 + 63 + CH - 1) / CH : quad ? (L1 + 3 + CH - 1) / CH : t->NC;
        t->spitch = 512 * NCH;          // per 64-row stripe (a pair stripe is two of them)
        FillArgs a{};
        a.s1 = t->s1;
        a.s2 = t->s2;
        a.L1 = (int32_t)L1;
        a.L2 = (int32_t)L2;
        a.m = m;
        a.k = k;
        a.d = d;
        a.NC = (int32_t)t->NC;
        a.NCH = (int32_t)NCH;
        a.NG = (int32_t)NGk;
        a.NSW = (int32_t)plan.NSW;
        a.SQ = pSQ = plan.SQ;
        a.SR = pSR = plan.SR;
        a.H = t->H;
        a.spitch = pair ? 2 * t->spitch : t->spitch;
        a.D = t->D;
        a.lastcol = t->lastcol;
        a.gran = t->gran;
        a.gpitch = CH * t->NC + CH;
        a.ctl = t->ctl;
        // A panel waits on another GPU (or process) that may start seconds
        // later; a plain fill only on itself.
        a.spin_ticks = (t->xin || t->xout) ? 30 * SPIN_TICKS : SPIN_TICKS;
        a.row_base = (int32_t)t->row_base;
        a.epoch = t->epoch;
        a.xin = t->xin;
        a.xout = t->xout;
        a.xflag = t->xflag;
        a.xblk = (int32_t)std::max<int64_t>(t->xblk, 1);
        a.row0 = t->row0;
        a.xin_credit = t->xin ? t->xin_credit : nullptr;
        a.xout_credit = t->xout ? t->xout_credit : nullptr;
        a.credit_want = t->credit_want;
        if (t->xout && (L2 % 64) != 0) return fail(NW_ERR_ARG, "nw_table_fill: a feeding panel needs 64*k rows");
        if (getenv("NW_TRACE")) {
            // header {NSW, stamps after the WG rows}, 8 words per WG-stripe, then
            // (pair kernel) one mid-table time per 128-row stripe
            const int64_t nmid = NGk + 4 * (int64_t)plan.NSW;   // + loader (+ pair: per-stripe, publisher) times
            const int64_t need = 8 + 8 * (int64_t)a.NSW + nmid;
            if (t->trace_n < need) {
                (void)hipFree(t->trace);
                t->trace = nullptr;
                t->trace_n = 0;
                NW_HIPCHK(hipMalloc(&t->trace, (size_t)need * 8));
                t->trace_n = need;
            }
            NW_HIPCHK(hipMemsetAsync(t->trace, 0, (size_t)need * 8, t->stream));
            t->trace_hdr[0] = (uint64_t)a.NSW;
            t->trace_hdr[1] = (uint64_t)nmid;
            NW_HIPCHK(hipMemcpyAsync(t->trace, t->trace_hdr, 16, hipMemcpyHostToDevice, t->stream));
            a.trace = t->trace + 8;
        }
        int occ = 1;
        const int wgw = W + (skew ? 1 : 2);   // + loader (+ publisher: scan, pair and quad kernels)
        NW_HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(fn), 64 * wgw, 0));
        occ = std::max(occ, 1);
        // A panel leaves room on every CU for the kernels of its neighbours
        // and of the transport (RCCL), which its hand-off waits on.
        const int per_cu = panel ? std::max(1, std::min(2, occ - 1)) : std::min(occ, kMaxWgPerCu);
        const int64_t grid = std::min<int64_t>(a.NSW, (int64_t)t->ncu * per_cu);
        a.nslot = (int32_t)std::min<int64_t>(grid + 1, (int64_t)(t->gran_bytes / 8 / a.gpitch));
        if (a.nslot < grid + 1) return fail(NW_ERR_ARG, "nw_table_fill: granule buffer too small");
        // Granule tags carry a 16-bit fill sequence above the WG-stripe index,
        // so a granule left by an earlier fill never matches and the slots
        // need clearing (205 MB at 100k^2, inside every timed step before)
        // only on a fresh buffer, once per 65535 fills, or when the indices
        // do not fit 16 bits.
        if (a.NSW > 1) {
            const size_t used = (size_t)a.nslot * a.gpitch * 8;
            t->gseq = (t->gseq + 1) & 0xffffu;
            if (t->gseq == 0 || used > t->gran_clean || a.NSW >= 0x10000) {
                NW_HIPCHK(hipMemsetAsync(t->gran, 0, used, t->stream));
                t->gran_clean = std::max(t->gran_clean, used);
                if (t->gseq == 0) t->gseq = 1;
            }
            a.gtag = a.NSW < 0x10000 ? t->gseq << 16 : 0u;
        }
        NW_HIPCHK(hipEventRecord(t->ev[1], t->stream));
        void* kargs[] = {&a};
        NW_HIPCHK(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3((unsigned)grid), dim3(64 * wgw), kargs,
                                  0, t->stream));
        NW_HIPCHK(hipGetLastError());
        NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    } else {
        NW_HIPCHK(hipEventRecord(t->ev[1], t->stream));
        // no kernel reads the row above: release it for the producer's next fill
        if (t->xin && t->xin_credit) NW_HIPCHK(hipMemsetD32Async(t->xin_credit, (int)t->epoch, 1, t->stream));
        NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    }
    t->launched = true;
    t->pend_mask = out_mask;
    t->pend_d = d;
    t->pend_W = W;
    t->pend_skew = skew ? 1 : quad ? 2 : 0;
    t->pend_pair = pair;
    // the pair kernel's fills with scores and without stats store G' (RAW in nw_pair.hip)
    t->pend_raw = (pair && sh && !stt) ? 1 : (quad && sh) ? 2 : 0;
    t->pend_SQ = pSQ;
    t->pend_SR = pSR;
    return NW_OK;
}

int poison(uint64_t* p, int64_t n, uint32_t epoch, hipStream_t s) {
    if (n <= 0) return NW_OK;
    nw_poison_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 1024), 256, 0, s>>>(p, n, epoch);
    NW_HIPCHK(hipGetLastError());
    return NW_OK;
}

int fill_finish(nw_table* t) {
    if (!t || !t->launched) return fail(NW_ERR_STATE, "nw_table_fill: no fill in flight");
    t->launched = false;
    NW_HIPCHK(hipSetDevice(t->device));
    const int64_t L1 = t->L1, L2 = t->L2;
    const bool sh = t->pend_mask & NW_OUT_SCORES, stt = t->pend_mask & NW_OUT_STATS;
    const int32_t d = t->pend_d;
    NW_HIPCHK(hipEventRecord(t->ev[3], t->stream));
    uint32_t ctl[CTL_WORDS];
    NW_HIPCHK(hipMemcpyAsync(ctl, t->ctl, sizeof ctl, hipMemcpyDeviceToHost, t->stream));
    int32_t corner = 0;
    if (L1 > 0 && L2 > 0) {
        const int64_t r = L2 - 1, q = L1 - 1;
        const int32_t* src = sh ? t->H + score_index(r, q, t->spitch, t->pend_skew, t->pend_pair) : t->lastcol + L2;
        NW_HIPCHK(hipMemcpyAsync(&corner, src, 4, hipMemcpyDeviceToHost, t->stream));
    }
    NW_HIPCHK(hipStreamSynchronize(t->stream));
    if (L1 > 0 && L2 > 0 && sh && t->pend_raw)
        corner = (int32_t)((uint32_t)corner - raw_offset(L1, L2, t->pend_SQ, t->pend_SR, d, t->pend_raw));
    if (ctl[CTL_ERR])
        return fail((int)ctl[CTL_ERR], (int)ctl[CTL_ERR] == NW_ERR_PEER
                                           ? "nw_table_fill: the panel above failed"
                                           : "nw_table_fill: in-kernel watchdog fired (hand-off timeout)");
    NW_HIPCHK(hipEventElapsedTime(&t->kernel_ms, t->ev[1], t->ev[2]));
    NW_HIPCHK(hipEventElapsedTime(&t->call_ms, t->ev[0], t->ev[3]));
    if (L1 == 0 || L2 == 0) corner = (int32_t)(-(L1 + L2 + t->row_base) * (int64_t)d);
    t->stats.corner = corner;
    t->stats.greatest_abs_interior = stt ? (int32_t)ctl[CTL_GAV] : 0;
    t->stats.branch_count = stt ? ctl[CTL_BC] : 0u;
    t->filled = true;
    ++t->fill_serial;
    t->last_mask = t->pend_mask;
    t->last_d = d;
    t->waves = t->pend_W;
    t->skew = t->pend_skew;
    t->pair = t->pend_pair;
    t->raw = t->pend_raw;
    t->SQ = t->pend_SQ;
    t->SR = t->pend_SR;
    t->lay_NC = t->spitch / 512;
    return NW_OK;
}

}  // namespace nwi

using nwi::fail;
#define HIPCHK NW_HIPCHK

extern "C" {

const char* nw_strerror(int rc) {
    switch (rc) {
        case NW_OK: return "success";
        case NW_ERR_ARG: return "invalid argument";
        case NW_ERR_NODEVICE: return "no usable gfx950 GPU";
        case NW_ERR_OOM: return "out of memory";
        case NW_ERR_HIP: return "HIP runtime error";
        case NW_ERR_RANGE: return "scores may overflow int32 for these inputs";
        case NW_ERR_TIMEOUT: return "device hand-off timed out";
        case NW_ERR_STATE: return "call out of order";
        case NW_ERR_PEER: return "a peer panel failed";
        default: return "unknown error";
    }
}

const char* nw_last_error(void) { return nwi::g_last_error.c_str(); }

void nw_table_destroy(nw_table* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    nwi::walk_release(t);
    (void)hipFree(t->s1);
    (void)hipFree(t->s2);
    (void)hipFree(t->H);
    (void)hipFree(t->D);
    (void)hipFree(t->lastcol);
    (void)hipFree(t->row0);
    (void)hipFree(t->gran);
    (void)hipFree(t->ctl);
    (void)hipFree(t->trace);
    for (auto& e : t->ev)
        if (e) (void)hipEventDestroy(e);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    release_io(t);
    delete t;
}

int nw_table_create(int device, int64_t max_L1, int64_t max_L2, uint32_t out_mask, nw_table** out) {
    if (!out || max_L1 < 0 || max_L2 < 0 || max_L1 > INT32_MAX - 64 || max_L2 > INT32_MAX - 4096)
        return fail(NW_ERR_ARG, "nw_table_create: bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(NW_ERR_NODEVICE, "nw_table_create: no HIP device visible");
    if (device < 0) {
        const char* e = getenv("NW_DEVICE");
        device = e ? atoi(e) : 0;
    }
    if (device >= ndev) return fail(NW_ERR_NODEVICE, "nw_table_create: device ordinal out of range");
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(NW_ERR_NODEVICE, std::string("nw_table_create: device is ") + prop.gcnArchName +
                                         ", this library is built for gfx950 only");
    nw_table* t = new nw_table;
    t->device = device;
    t->ncu = prop.multiProcessorCount;
    t->cap_mask = out_mask;
    t->max_L1 = max_L1;
    t->max_L2 = max_L2;
    auto bail = [&](int rc) {
        nw_table_destroy(t);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(fail(NW_ERR_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(NW_ERR_HIP, "hipStreamCreate failed"));
    for (auto& e : t->ev)
        if (hipEventCreate(&e) != hipSuccess) return bail(fail(NW_ERR_HIP, "hipEventCreate failed"));

    const int64_t NC = (max_L1 + CH - 1) / CH;
    const int64_t NG = (max_L2 + 63) / 64;
    auto alloc = [&](void** p, size_t bytes) -> int {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 256));
        if (e != hipSuccess)
            return fail(NW_ERR_OOM, "hipMalloc(" + std::to_string(bytes) + ") failed: " + hipGetErrorString(e));
        return 0;
    };
    int rc;
    if ((rc = alloc((void**)&t->s1, (size_t)(CH * NC + 64)))) return bail(rc);
    if ((rc = alloc((void**)&t->s2, (size_t)(64 * NG + 1024)))) return bail(rc);
    if (out_mask & NW_OUT_SCORES) {
        if ((rc = alloc((void**)&t->H, (size_t)(NG + 1) * (size_t)(NC + 8) * 2048)))
            return bail(rc);
    }
    if (out_mask & NW_OUT_DIRS) {
        if ((rc = alloc((void**)&t->D, (size_t)(NG + 1) * (NC + 9) * 256))) return bail(rc);
    }
    if ((rc = alloc((void**)&t->lastcol, (size_t)(64 * NG + 128) * 4))) return bail(rc);
    if ((rc = alloc((void**)&t->row0, (size_t)(max_L1 + 8) * 4))) return bail(rc);
    // Granule slots: one per concurrently running WG-stripe + 1.
    const int64_t gpitch = CH * NC + CH;
    const int64_t nslot = kMaxWgPerCu * (int64_t)t->ncu + 1;
    t->gran_bytes = (size_t)(gpitch * nslot * 8);
    if ((rc = alloc((void**)&t->gran, t->gran_bytes))) return bail(rc);
    if ((rc = alloc((void**)&t->ctl, CTL_WORDS * 4))) return bail(rc);
    *out = t;
    return NW_OK;
}

int nw_table_set_sequences(nw_table* t, const char* s1, int64_t L1, const char* s2, int64_t L2) {
    if (!t || L1 < 0 || L2 < 0 || L1 > t->max_L1 || L2 > t->max_L2 || (L1 && !s1) || (L2 && !s2))
        return fail(NW_ERR_ARG, "nw_table_set_sequences: bad arguments");
    const double t0 = host_ms();
    HIPCHK(hipSetDevice(t->device));
    t->L1 = L1;
    t->L2 = L2;
    t->NC = (L1 + CH - 1) / CH;
    t->NG = (L2 + 63) / 64;
    t->spitch = 512 * t->NC;
    t->filled = false;
    const size_t n1 = (size_t)(CH * t->NC + 64), n2 = (size_t)(64 * t->NG + 1024);
    HIPCHK(hipMemsetAsync(t->s1, 0, n1, t->stream));
    HIPCHK(hipMemsetAsync(t->s2, 0, n2, t->stream));
    // Only equality of symbols matters (needleman-wunsch.c:432), so when
    // s1 and s2 use at most 8 distinct bytes they are coded 0..7 (in order of
    // first appearance) and the fill looks sub' up in a per-lane profile.
    int code[256];
    std::fill(code, code + 256, -1);
    int alpha = 0;
    auto scan = [&](const char* p, int64_t n) {
        for (int64_t i = 0; i < n && alpha <= 8; ++i) {
            const uint8_t b = (uint8_t)p[i];
            if (code[b] < 0) code[b] = alpha++;
        }
    };
    scan(s1, L1);
    scan(s2, L2);
    t->alpha = (alpha >= 1 && alpha <= 8) ? alpha : 0;
    // The (coded) sequences are written straight into pinned staging, so
    // the upload runs at PCIe rate with no pageable bounce.
    const size_t need = (size_t)(t->max_L1 + t->max_L2 + 16);
    if (t->h_seq_bytes < need) {
        if (t->h_seq) (void)hipHostFree(t->h_seq);
        t->h_seq = nullptr;
        t->h_seq_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&t->h_seq, need, hipHostMallocDefault));
        t->h_seq_bytes = need;
    }
    uint8_t* h1 = t->h_seq;
    uint8_t* h2 = t->h_seq + L1;
    if (t->alpha) {
        for (int64_t i = 0; i < L1; ++i) h1[i] = (uint8_t)code[(uint8_t)s1[i]];
        for (int64_t i = 0; i < L2; ++i) h2[i] = (uint8_t)code[(uint8_t)s2[i]];
    } else {
        if (L1) std::memcpy(h1, s1, (size_t)L1);
        if (L2) std::memcpy(h2, s2, (size_t)L2);
    }
    if (L1) HIPCHK(hipMemcpyAsync(t->s1, h1, (size_t)L1, hipMemcpyHostToDevice, t->stream));
    if (L2) HIPCHK(hipMemcpyAsync(t->s2, h2, (size_t)L2, hipMemcpyHostToDevice, t->stream));
    HIPCHK(hipStreamSynchronize(t->stream));
    t->upload_ms = host_ms() - t0;
    t->upload_bytes = L1 + L2;
    return NW_OK;
}

int nw_table_fill(nw_table* t, int32_t m, int32_t k, int32_t d, uint32_t out_mask) {
    const int rc = nwi::fill_launch(t, m, k, d, out_mask);
    if (rc) return rc;
    return nwi::fill_finish(t);
}

int nw_table_stats(nw_table* t, nw_stats* st) {
    if (!t || !st) return fail(NW_ERR_ARG, "nw_table_stats: NULL argument");
    if (!t->filled) return fail(NW_ERR_STATE, "nw_table_stats: no completed fill");
    *st = t->stats;
    return NW_OK;
}

int nw_table_elapsed_ms(nw_table* t, float* kernel_ms, float* call_ms) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_elapsed_ms: NULL table");
    if (!t->filled) return fail(NW_ERR_STATE, "nw_table_elapsed_ms: no completed fill");
    if (kernel_ms) *kernel_ms = t->kernel_ms;
    if (call_ms) *call_ms = t->call_ms;
    return NW_OK;
}

int64_t nw_table_trace(nw_table* t, uint64_t* dst, int64_t n) {
    if (!t || !t->trace) return 0;
    const int64_t m = std::min(n, t->trace_n);
    if (m > 0 && dst) {
        if (hipMemcpy(dst, t->trace, (size_t)m * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    }
    return t->trace_n;
}

int64_t nw_table_score_pitch(const nw_table* t) { return t ? t->spitch : 0; }

int nw_table_layout(const nw_table* t, nw_layout* out) {
    if (!t || !out) return fail(NW_ERR_ARG, "nw_table_layout: NULL argument");
    if (!t->filled) return fail(NW_ERR_STATE, "nw_table_layout: no completed fill");
    nw_layout l{};
    l.score_pitch = t->spitch;
    l.NQ = t->lay_NC;
    l.pair = t->pair;
    l.skew = t->skew;
    l.raw = t->raw;
    l.SQ = t->SQ;
    l.SR = t->SR;
    l.d = t->last_d;
    l.has_scores = (t->last_mask & NW_OUT_SCORES) != 0;
    l.has_dirs = (t->last_mask & NW_OUT_DIRS) != 0;
    *out = l;
    return NW_OK;
}

int nw_table_device_buffers(const nw_table* t, const int32_t** scores, const uint32_t** dirs) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_device_buffers: NULL table");
    if (scores) *scores = t->H;
    if (dirs) *dirs = t->D;
    return NW_OK;
}
int nw_table_waves(const nw_table* t) { return t ? t->waves : 0; }

static int copy_scores_impl(nw_table* t, int64_t i0, int64_t i1, int32_t* dst) {
    const TableView v = view_of(t);
    const int32_t L2 = (int32_t)t->L2;
    return stream_columns(t, i0, i1, (size_t)(t->L2 + 1) * 4, reinterpret_cast<uint8_t*>(dst),
                          [&](int64_t c0, int64_t c1, void* buf) {
                              nw_gather_scores_kernel<<<1024, 256, 0, t->stream>>>(v, L2, c0, c1,
                                                                                   static_cast<int32_t*>(buf));
                          },
                          "nw_table_copy_scores");
}

int nw_table_copy_scores(nw_table* t, int64_t i0, int64_t i1, int32_t* dst) {
    if (!t || !dst || i0 < 0 || i1 < i0) return fail(NW_ERR_ARG, "nw_table_copy_scores: bad arguments");
    if (!t->filled || !(t->last_mask & NW_OUT_SCORES)) return fail(NW_ERR_STATE, "nw_table_copy_scores: no score table");
    if (i1 > t->L1 + 1) return fail(NW_ERR_ARG, "nw_table_copy_scores: column range");
    if (i1 == i0) return NW_OK;
    HIPCHK(hipSetDevice(t->device));
    return copy_scores_impl(t, i0, i1, dst);
}

int nw_table_copy_last_column(nw_table* t, int32_t* dst) {
    if (!t || !dst) return fail(NW_ERR_ARG, "nw_table_copy_last_column: bad arguments");
    if (!t->filled) return fail(NW_ERR_STATE, "nw_table_copy_last_column: no completed fill");
    HIPCHK(hipSetDevice(t->device));
    if (t->last_mask & NW_OUT_SCORES) return copy_scores_impl(t, t->L1, t->L1 + 1, dst);
    const int64_t d = t->last_d;
    if (t->L1 == 0) {
        for (int64_t j = 0; j <= t->L2; ++j) dst[j] = (int32_t)(-(t->row_base + j) * d);
        return NW_OK;
    }
    // Row 0: the seed, or (panels) the last row of the panel above.
    if (t->row_base > 0) {
        int32_t g = 0;
        HIPCHK(hipMemcpyAsync(&g, t->row0 + (t->L1 - 1), 4, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(hipStreamSynchronize(t->stream));
        dst[0] = g + t->last_d;
    } else {
        dst[0] = (int32_t)(-t->L1 * d);
    }
    if (t->L2 > 0) {
        HIPCHK(hipMemcpyAsync(dst + 1, t->lastcol + 1, (size_t)t->L2 * 4, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(hipStreamSynchronize(t->stream));
    }
    return NW_OK;
}

int nw_table_copy_codes(nw_table* t, int64_t i0, int64_t i1, uint8_t* dst) {
    if (!t || !dst || i0 < 0 || i1 < i0) return fail(NW_ERR_ARG, "nw_table_copy_codes: bad arguments");
    if (!t->filled || !(t->last_mask & NW_OUT_DIRS)) return fail(NW_ERR_STATE, "nw_table_copy_codes: no direction codes");
    if (i1 > t->L1 + 1) return fail(NW_ERR_ARG, "nw_table_copy_codes: column range");
    if (i1 == i0) return NW_OK;
    HIPCHK(hipSetDevice(t->device));
    const TableView v = view_of(t);
    const int32_t L2 = (int32_t)t->L2;
    return stream_columns(t, i0, i1, (size_t)(t->L2 + 1), dst,
                          [&](int64_t c0, int64_t c1, void* buf) {
                              nw_codes_kernel<<<1024, 256, 0, t->stream>>>(v, L2, c0, c1, static_cast<uint8_t*>(buf));
                          },
                          "nw_table_copy_codes");
}

int nw_host_alloc(size_t bytes, void** p) {
    if (!p) return fail(NW_ERR_ARG, "nw_host_alloc: NULL argument");
    *p = nullptr;
    hipError_t e = hipHostMalloc(p, std::max<size_t>(bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) return fail(NW_ERR_OOM, std::string("nw_host_alloc: ") + hipGetErrorString(e));
    return NW_OK;
}

void nw_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int nw_table_io_stats(nw_table* t, double* upload_ms, int64_t* upload_bytes, double* copy_ms, int64_t* copy_bytes) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_io_stats: NULL table");
    if (upload_ms) *upload_ms = t->upload_ms;
    if (upload_bytes) *upload_bytes = t->upload_bytes;
    if (copy_ms) *copy_ms = t->copy_ms;
    if (copy_bytes) *copy_bytes = t->copy_bytes;
    return NW_OK;
}

int nw_table_hash_columns(nw_table* t, int64_t j0, uint64_t* hstate, uint64_t* dstate) {
    if (!t || !hstate || !dstate || j0 < 0) return fail(NW_ERR_ARG, "nw_table_hash_columns: bad arguments");
    if (!t->filled || !(t->last_mask & NW_OUT_SCORES))
        return fail(NW_ERR_STATE, "nw_table_hash_columns: no score table");
    HIPCHK(hipSetDevice(t->device));
    const int64_t ncol = t->L1 + 1;
    uint64_t* dh = nullptr;
    HIPCHK(hipMalloc(&dh, (size_t)ncol * 16));
    TableView v = view_of(t);
    if (!(t->last_mask & NW_OUT_DIRS)) v.D = nullptr;
    hipError_t e = hipMemcpyAsync(dh, hstate, (size_t)ncol * 8, hipMemcpyHostToDevice, t->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dh + ncol, dstate, (size_t)ncol * 8, hipMemcpyHostToDevice, t->stream);
    if (e == hipSuccess) {
        nw_colhash_kernel<<<(unsigned)((ncol + 255) / 256), 256, 0, t->stream>>>(v, (int32_t)t->L1, (int32_t)t->L2,
                                                                                  (int32_t)std::min<int64_t>(j0, t->L2 + 1),
                                                                                  dh, dh + ncol);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(hstate, dh, (size_t)ncol * 8, hipMemcpyDeviceToHost, t->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dstate, dh + ncol, (size_t)ncol * 8, hipMemcpyDeviceToHost, t->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    (void)hipFree(dh);
    if (e != hipSuccess) return fail(NW_ERR_HIP, std::string("nw_table_hash_columns: ") + hipGetErrorString(e));
    return NW_OK;
}

uint64_t nw_hash_fold(const uint64_t* state, int64_t n) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (int64_t i = 0; state && i < n; ++i)
        for (int b = 0; b < 8; ++b) h = (h ^ ((state[i] >> (8 * b)) & 0xff)) * 0x100000001b3ULL;
    return h;
}

int nw_table_hash(nw_table* t, uint64_t* hH, uint64_t* hD) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_hash: NULL table");
    if (!t->filled || !(t->last_mask & NW_OUT_SCORES)) return fail(NW_ERR_STATE, "nw_table_hash: no score table");
    const int64_t ncol = t->L1 + 1;
    std::vector<uint64_t> hs((size_t)ncol, 0xcbf29ce484222325ULL), ds((size_t)ncol, 0xcbf29ce484222325ULL);
    const int rc = nw_table_hash_columns(t, 0, hs.data(), ds.data());
    if (rc) return fail(rc, std::string("nw_table_hash: ") + nw_last_error());
    if (hH) *hH = nw_hash_fold(hs.data(), ncol);
    if (hD) *hD = (t->last_mask & NW_OUT_DIRS) ? nw_hash_fold(ds.data(), ncol) : 0;
    return NW_OK;
}

int nw_fill(const char* s1, int64_t L1, const char* s2, int64_t L2, int32_t m, int32_t k, int32_t d,
            uint32_t out_mask, int device, int32_t* H, uint8_t* dirs, nw_stats* stats) {
    if (L1 < 0 || L2 < 0 || (L1 && !s1) || (L2 && !s2)) return fail(NW_ERR_ARG, "nw_fill: bad arguments");
    uint32_t mask = out_mask & NW_OUT_STATS;
    if (H) mask |= NW_OUT_SCORES;
    if (dirs) mask |= NW_OUT_DIRS;
    nw_table* t = nullptr;
    int rc = nw_table_create(device, L1, L2, mask, &t);
    if (rc) return rc;
    rc = nw_table_set_sequences(t, s1, L1, s2, L2);
    if (!rc) rc = nw_table_fill(t, m, k, d, mask);
    if (!rc && H) rc = nw_table_copy_scores(t, 0, L1 + 1, H);
    if (!rc && dirs) {
        const int64_t ncell = (L1 + 1) * (L2 + 1);
        const size_t nbyte = (size_t)((ncell + 1) / 2);
        uint8_t* buf = nullptr;
        if (hipMalloc(&buf, nbyte) != hipSuccess) rc = fail(NW_ERR_OOM, "nw_fill: hipMalloc(dirs)");
        if (!rc) {
            hipLaunchKernelGGL(nw_pack_nibbles_kernel, dim3(1024), dim3(256), 0, t->stream, view_of(t), (int32_t)L1,
                               (int32_t)L2, buf);
            hipError_t e = hipGetLastError();
            if (e == hipSuccess) e = hipMemcpyAsync(dirs, buf, nbyte, hipMemcpyDeviceToHost, t->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
            if (e != hipSuccess) rc = fail(NW_ERR_HIP, std::string("nw_fill: ") + hipGetErrorString(e));
        }
        (void)hipFree(buf);
    }
    if (!rc && stats) rc = nw_table_stats(t, stats);
    nw_table_destroy(t);
    return rc;
}

}  // extern "C"

// ------------------------------------------------------------------ no-alloc
// nw_fill_noalloc (include/nw_fill.h): the fill for callers that cannot
// allocate.  Everything the fill kernel needs beyond the caller's inputs and
// outputs -- the padded copies of the two sequences, the control words, the
// last-column staging of a score-only fill and the WG-stripe hand-off
// granules -- lives in one file-scope device array, `scratch`.  Every GPU the
// library runs on holds its own copy of the array at its own address; host
// code only ever uses the address hipGetSymbolAddress returned for that GPU
// (na_state.ptr), never the array's name.
namespace {

constexpr int64_t kNaMaxL1 = NW_NOALLOC_MAX_L1, kNaMaxL2 = NW_NOALLOC_MAX_L2;
constexpr int64_t kNaNC = (kNaMaxL1 + CH - 1) / CH, kNaNG = (kNaMaxL2 + 63) / 64;
constexpr int kNaW = 4;                                       // stripes per workgroup
constexpr int64_t kNaSlots = (kNaNG + kNaW - 1) / kNaW + 1;   // one per WG-stripe + 1
constexpr size_t na_align(size_t x) { return (x + 255) & ~(size_t)255; }
constexpr size_t kNaCtl = 0;                                              // CTL_WORDS uint32
constexpr size_t kNaS1 = na_align(kNaCtl + CTL_WORDS * 4);                // CH*NC + 64 bytes
constexpr size_t kNaS2 = na_align(kNaS1 + (size_t)(CH * kNaNC + 64));     // 64*NG + 1024 bytes
constexpr size_t kNaLast = na_align(kNaS2 + (size_t)(64 * kNaNG + 1024)); // (64*NG + 128) int32
constexpr size_t kNaGran = na_align(kNaLast + (size_t)(64 * kNaNG + 128) * 4);
constexpr size_t kNaBytes = na_align(kNaGran + (size_t)(kNaSlots * (CH * kNaNC + CH)) * 8);
static_assert(kNaBytes <= NW_NOALLOC_SCRATCH_BYTES, "scratch layout exceeds its stated size");

static __device__ __align__(256) unsigned char scratch[NW_NOALLOC_SCRATCH_BYTES];

struct NaState {
    unsigned char* ptr = nullptr;   // this device's copy of `scratch` (hipGetSymbolAddress)
    int ncu = 0;
    int rc = NW_OK;
    bool ready = false;
};
constexpr int kNaMaxDev = 64;
NaState g_na[kNaMaxDev];
std::atomic_flag g_na_lock = ATOMIC_FLAG_INIT;

// Once per device, with that device current.
const NaState& na_state(int device) {
    while (g_na_lock.test_and_set(std::memory_order_acquire)) {
    }
    NaState& st = g_na[device];
    if (!st.ready) {
        st.ready = true;
        hipDeviceProp_t prop;
        void* p = nullptr;
        hipError_t e = hipGetDeviceProperties(&prop, device);
        if (e == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            st.rc = fail(NW_ERR_NODEVICE, std::string("nw_fill_noalloc: device is ") + prop.gcnArchName +
                                              ", this library is built for gfx950 only");
        } else {
            if (e == hipSuccess) e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
            if (e != hipSuccess || !p)
                st.rc = fail(NW_ERR_HIP, std::string("nw_fill_noalloc: hipGetSymbolAddress(scratch): ") +
                                             hipGetErrorString(e));
            else {
                st.ptr = static_cast<unsigned char*>(p);
                st.ncu = prop.multiProcessorCount;
            }
        }
    }
    g_na_lock.clear(std::memory_order_release);
    return st;
}

// Padded copies of the sequences (the fill kernel reads whole chunks and whole
// stripes), the control words and the granule slots this fill uses start at
// zero.  A kernel, not hipMemsetAsync: the call may be recorded into a graph.
__global__ void nw_na_prep_kernel(unsigned char* sc, const char* s1, int32_t L1, const char* s2, int32_t L2,
                                  int64_t n1, int64_t n2, int64_t ngran) {
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
    if (tid < CTL_WORDS) reinterpret_cast<uint32_t*>(sc + kNaCtl)[tid] = 0u;
    for (int64_t x = tid; x < n1; x += nth) sc[kNaS1 + x] = x < L1 ? (unsigned char)s1[x] : 0;
    for (int64_t x = tid; x < n2; x += nth) sc[kNaS2 + x] = x < L2 ? (unsigned char)s2[x] : 0;
    uint64_t* g = reinterpret_cast<uint64_t*>(sc + kNaGran);
    for (int64_t x = tid; x < ngran; x += nth) g[x] = 0ull;
}

// Results: status + stats, and the last column H[L1][0..L2].
__global__ void nw_na_finish_kernel(const unsigned char* sc, TableView v, int32_t L1, int32_t L2, int32_t d, int sh,
                                    int stt, int32_t* last, nw_noalloc_result* res) {
    const uint32_t* ctl = reinterpret_cast<const uint32_t*>(sc + kNaCtl);
    const int32_t* lc = reinterpret_cast<const int32_t*>(sc + kNaLast);
    auto cell = [&](int64_t j) -> int32_t {
        if (L1 == 0 || j == 0) return (int32_t)(-(L1 + j) * (int64_t)d);
        return sh ? score_at(v, L1, j) : lc[j];
    };
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
    if (last)
        for (int64_t j = tid; j <= L2; j += nth) last[j] = cell(j);
    if (tid == 0 && res) {
        res->status = (int32_t)ctl[CTL_ERR];
        res->stats.corner = cell(L2);
        res->stats.greatest_abs_interior = stt ? (int32_t)ctl[CTL_GAV] : 0;
        res->stats.branch_count = stt ? ctl[CTL_BC] : 0u;
    }
}

}  // namespace

extern "C" int nw_fill_noalloc(int device, void* stream, const char* s1_dev, int64_t L1, const char* s2_dev,
                               int64_t L2, int32_t m, int32_t k, int32_t d, uint32_t out_mask,
                               int32_t* score_tiles_dev, uint32_t* dir_words_dev, int32_t* last_column_dev,
                               nw_noalloc_result* result_dev) {
    if (L1 < 0 || L2 < 0 || (L1 && !s1_dev) || (L2 && !s2_dev) || device < 0 || device >= kNaMaxDev)
        return fail(NW_ERR_ARG, "nw_fill_noalloc: bad arguments");
    if (L1 > kNaMaxL1 || L2 > kNaMaxL2)
        return fail(NW_ERR_ARG, "nw_fill_noalloc: " + std::to_string(L1) + " x " + std::to_string(L2) +
                                    " is beyond the scratch array's limit of " + std::to_string(kNaMaxL1) + " x " +
                                    std::to_string(kNaMaxL2) + " (use nw_table_fill)");
    if (((out_mask & NW_OUT_SCORES) && !score_tiles_dev) || ((out_mask & NW_OUT_DIRS) && !dir_words_dev))
        return fail(NW_ERR_ARG, "nw_fill_noalloc: an output in out_mask has no buffer");
    {
        const int64_t M = std::max({std::llabs(m), std::llabs(k), std::llabs(d)});
        const int64_t bound = (L1 + L2) * M + 6144 * std::llabs(d) + 4 * M + 2;   // as nwi::fill_launch
        if (bound >= (int64_t)INT32_MAX)
            return fail(NW_ERR_RANGE, "nw_fill_noalloc: |scores| could reach " + std::to_string(bound));
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)
        return fail(NW_ERR_NODEVICE, "nw_fill_noalloc: device ordinal out of range");
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != device) HIPCHK(hipSetDevice(device));
    struct Restore {
        int cur, device;
        ~Restore() {
            if (cur != device) (void)hipSetDevice(cur);
        }
    } restore{cur, device};
    const NaState& st = na_state(device);
    if (st.rc != NW_OK) return st.rc;
    unsigned char* const sc = st.ptr;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool sh = out_mask & NW_OUT_SCORES, sd = out_mask & NW_OUT_DIRS, stt = out_mask & NW_OUT_STATS;
    const int64_t NC = (L1 + CH - 1) / CH, NG = (L2 + 63) / 64;
    TableView v{};
    v.tiles = score_tiles_dev;
    v.spitch = 512 * NC;
    v.D = sd ? dir_words_dev : nullptr;
    v.NC = (int32_t)NC;
    v.d = d;
    if (L1 > 0 && L2 > 0) {
        // WG-stripes of up to 4 stripes, dealt evenly (every SIMD its own
        // compute wave), taken in order from the dequeue: any grid completes.
        const int W = (int)std::min<int64_t>(kNaW, NG);
        const int64_t NSW = (NG + W - 1) / W;
        KernelFn fn = pick_kernel(W, false, sh, sd, stt);
        if (!fn) return fail(NW_ERR_ARG, "nw_fill_noalloc: unsupported wave count");
        const int64_t grid = std::min<int64_t>(NSW, (int64_t)st.ncu * 2);
        FillArgs a{};
        a.s1 = sc + kNaS1;
        a.s2 = sc + kNaS2;
        a.L1 = (int32_t)L1;
        a.L2 = (int32_t)L2;
        a.m = m;
        a.k = k;
        a.d = d;
        a.NC = a.NCH = (int32_t)NC;
        a.NG = (int32_t)NG;
        a.NSW = (int32_t)NSW;
        a.SQ = (int32_t)(NG / NSW);
        a.SR = (int32_t)(NG % NSW);
        a.H = score_tiles_dev;
        a.spitch = 512 * NC;
        a.D = dir_words_dev;
        a.lastcol = reinterpret_cast<int32_t*>(sc + kNaLast);
        a.gran = reinterpret_cast<uint64_t*>(sc + kNaGran);
        a.gpitch = CH * NC + CH;
        a.nslot = (int32_t)(grid + 1);
        a.ctl = reinterpret_cast<uint32_t*>(sc + kNaCtl);
        a.spin_ticks = SPIN_TICKS;
        a.xblk = 1;
        a.gtag = 1u << 16;
        const int64_t ngran = NSW > 1 ? (int64_t)a.nslot * a.gpitch : 0;
        if ((size_t)ngran * 8 > kNaBytes - kNaGran) return fail(NW_ERR_ARG, "nw_fill_noalloc: granule scratch too small");
        nw_na_prep_kernel<<<256, 256, 0, s>>>(sc, s1_dev, (int32_t)L1, s2_dev, (int32_t)L2, CH * NC + 64,
                                              64 * NG + 1024, ngran);
        HIPCHK(hipGetLastError());
        void* kargs[] = {&a};
        HIPCHK(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3((unsigned)grid), dim3(64 * (W + 2)), kargs, 0, s));
        HIPCHK(hipGetLastError());
    } else {
        nw_na_prep_kernel<<<1, 64, 0, s>>>(sc, s1_dev, 0, s2_dev, 0, 0, 0, 0);   // the control words only
        HIPCHK(hipGetLastError());
    }
    if (last_column_dev || result_dev) {
        nw_na_finish_kernel<<<64, 256, 0, s>>>(sc, v, (int32_t)L1, (int32_t)L2, d, sh ? 1 : 0, stt ? 1 : 0,
                                               last_column_dev, result_dev);
        HIPCHK(hipGetLastError());
    }
    return NW_OK;
}
