// nw_skew.hip -- the skewed-stripe fill kernel (the default fill; launched
// by nwi::fill_launch in nw_fill.hip, which also holds the column-scan
// kernel; both share FillArgs, the ring counters and the hand-off helpers of
// nw_kern.h).
//
// Same hot path as nw_fill_kernel -- compute_table_scores()
// (needleman-wunsch.c:583-626 -> score_cell :418-510) -- organised as a
// wavefront INSIDE each wave instead of a prefix scan over the lanes:
//
//  * A wave owns a 64-row stripe (lane l <-> row j0 + l) and runs steps
//    t = 0 .. L1 + 62; at step t lane l computes column i = t - l + 1.  Lane
//    l - 1 computed (i, j-1) at step t-1 and (i-1, j-1) at step t-2, so
//    both vertical neighbours arrive with ONE wave_shr:1 DPP of the previous
//    step's values -- no 6-level scan, no serial chain across the lanes.
//  * Domain E = H + (t + 1 - base)*d (base moves by 4096 every 512 chunks):
//        left = E(l, t-1),  up = E(l-1, t-1),  diag = E(l-1, t-2) + m' (+2d)
//        E(l, t) = max3(left, up, diag)          (needleman-wunsch.c:429-465)
//    Column 0 is one constant C0 = -(row_base + j0 + base)*d in this domain.
//  * Lane 0's up comes from the row above (the stripe above's lane 63, or
//    the seeded row 0 / the WG-stripe above's granules via the loader) as
//    plain H through the LDS ring; one v_add converts it.  Lane 63 writes its
//    plain H into the ring of the wave below, 8 columns per slot.
//  * Top-string symbols come from a per-workgroup LDS window filled by the
//    loader wave: 8 copies, copy k shifted by k bytes, so that every lane's
//    8 symbols of a chunk (columns 8c+1-l .. 8c+8-l) are one aligned
//    ds_read_b64 (copy (-l) & 7).
//
// Layout (the "skewed" layout, nw_table.skew = 1): a lane's values are
// stored by STEP, so each wave-instruction stays one coalesced block:
//   scores: stripe g tile, step t, lane l -> g*spitch + ((t>>2)*64 + l)*4 + (t&3),
//           spitch = 512*NCH, NCH = ceil((L1 + 63) / 8) chunks of 8 steps;
//   codes : word (g*(NCH+1) + (t>>3) + 1)*64 + l, code of step t at bits
//           [21 - 3(t&7), 23 - 3(t&7)] (row 0 of each stripe pads).
// Cell (i, j): g = (j-1)/64, l = (j-1)%64, t = i - 1 + l.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "nw_kern.h"

namespace nwk {
namespace {

constexpr int SWN = 2048;   // LDS string window: bytes per copy (power of 2)

// The loader writes the window position of column 8c+1..8c+8 when it
// publishes ring slot c; a wave reads chunk c's symbols only after it read
// ring slot >= c (or finished the ring), so the bytes are there.  The loader
// runs at most R chunks ahead of wave 0 and wave w at most R + 7 chunks ahead
// of wave w + 1 (ring room), so for W <= 15 the oldest column still needed
// is < 8*(R + 14*(R + 7)) + 71 < SWN columns behind the loader.
static_assert(8 * (4 + 14 * (4 + 7)) + 71 < SWN, "string window too small for 15 waves");

// Count 3-bit codes of a word (8 per word, bits 0..23) with >= 2 directions.
__device__ __forceinline__ uint32_t branch_codes(uint32_t x) {
    const uint32_t y = (x & (x >> 1)) | (x & (x >> 2)) | ((x >> 1) & (x >> 2));
    return __builtin_popcount(y & 0x249249u);
}

// Operands of the generated chunk block (nw_skew_chunk.inc).
struct SkewSlot {
    v4i a, b;           // T (plain H of the row above) of steps 0..3, 4..7
    v2i w;              // this lane's 8 symbols of the chunk (window)
};
struct SkewRegs {
    int e[7];           // out: E after steps 0..6
    int ein;            // in: E of the previous step; out: E after step 7
    int upc;            // in: u of the previous step; out: u of step 7
    int h[8];           // out: H of steps 0..7
    uint32_t acc;       // out: the chunk's code word
    int gav;            // in/out: running max |H| (stats)
    uint64_t pq;        // out: {prog[w], cons[w+1]} read mid-chunk
};
struct SkewConst {
    int sd[8];          // s*d (lane-0 pre-fill)
    int kd[8];          // -(s+1)*d (H)
    uint32_t c2;        // this lane's side symbol (byte compares)
    int vcm, vck;       // sub' for match / mismatch (byte compares)
    uint32_t pl, ph;    // profile: byte a = sub' of symbol a (int8), a = 0..3 / 4..7
    int cb;             // LDS address of ctr[2w]
};

#include "nw_skew_chunk.inc"

// Slow path: {prog[w], cons[w+1]}, then slot data and this lane's window
// symbols (LDS is in order per wave: data read after a progress value that
// covers it is valid).  Waited for here.
__device__ __forceinline__ uint64_t skew_read_slot(int cb, int rd, int wa, SkewSlot& s) {
    uint64_t pq;
    asm volatile(
        "ds_read_b64 %[pq], %[cb] offset:8\n\t"
        "ds_read_b128 %[a], %[rd]\n\t"
        "ds_read_b128 %[b], %[rd] offset:16\n\t"
        "ds_read_b64 %[w], %[wa]\n\t"
        "s_waitcnt lgkmcnt(0)"
        : [pq] "=&v"(pq), [a] "=&v"(s.a), [b] "=&v"(s.b), [w] "=&v"(s.w)
        : [cb] "v"(cb), [rd] "v"(rd), [wa] "v"(wa)
        : "memory");
    return pq;
}

// Two 16-byte nt stores of a chunk's 8 scores (2 KB per wave) / one code word.
__device__ __forceinline__ void skew_store_scores(const int* h, int32_t* hb, int hv) {
    const v4i qa = v4i{h[0], h[1], h[2], h[3]}, qb = v4i{h[4], h[5], h[6], h[7]};
    asm volatile(
        "global_store_dwordx4 %[hv], %[qa], %[hb] nt\n\t"
        "global_store_dwordx4 %[hv], %[qb], %[hb] offset:1024 nt"
        :
        : [hv] "v"(hv), [qa] "v"(qa), [qb] "v"(qb), [hb] "s"(hb)
        : "memory");
}
__device__ __forceinline__ void skew_store_code(uint32_t x, uint32_t* db, int dv) {
    asm volatile("global_store_dword %[dv], %[x], %[db] nt" : : [dv] "v"(dv), [x] "v"(x), [db] "s"(db) : "memory");
}

template <int W, bool SH, bool SD, bool ST, bool PROF>
__global__ __launch_bounds__(64 * (W + 1)) void nw_skew_kernel(FillArgs a) {
    constexpr int R = 4;
    constexpr int NOCONS = 1 << 30;
    __shared__ __attribute__((aligned(16))) int tring[(W + 1) * R * SLOT];
    __shared__ __attribute__((aligned(16))) uint8_t swin_raw[8 * SWN + SWN];   // 8 copies, SWN-aligned inside
    __shared__ __attribute__((aligned(8))) int ctr[2 * W + 4];
    __shared__ int scratch[64 + R * SLOT];     // dummy target of the block's ring writes (lanes 0..62)
    __shared__ int sh_sidx;
    __shared__ int sh_abort;

    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6);
    const bool loader = (w == W);
    const int d = a.d;
    const int vcm = a.m + 2 * a.d;
    const int vck = 2 * a.d - a.k;
    const int NC1 = a.NC;                       // 8-column ring slots
    const int NCH = a.NCH;                      // 8-step chunks of a stripe
    const int nlast = a.L1 - CH * (NC1 - 1);    // columns in the last slot (1..8)
    // window copies start on an SWN boundary of the LDS address space, so a
    // lane's address wraps with one v_bfi
    const int swin0 = (lds_addr(swin_raw) + SWN - 1) & ~(SWN - 1);
    uint8_t* const swin = swin_raw + (swin0 - lds_addr(swin_raw));

    for (;;) {
        if (threadIdx.x == 0) {
            const int sidx = (int)atomicAdd(&a.ctl[CTL_NEXT], 1u);
            sh_sidx = sidx;
            sh_abort = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - (sidx * a.SQ + min(sidx, a.SR)));
            for (int v = 0; v <= W; ++v) {
                ctr[2 * v + 2] = 0;
                ctr[2 * v + 1] = v < nw ? 0 : NOCONS;
            }
        }
        __syncthreads();
        const int sidx = uni(sh_sidx);
        if (sidx >= a.NSW || sh_abort) break;
        if (a.trace && threadIdx.x == 0) {
            a.trace[8 * (int64_t)sidx + 0] = __builtin_amdgcn_s_memrealtime();
            a.trace[8 * (int64_t)sidx + 3] = (uint64_t)blockIdx.x | ((uint64_t)__smid() << 32);
        }
        const int g0 = sidx * a.SQ + min(sidx, a.SR);
        const int nw = min(a.SQ + (sidx < a.SR ? 1 : 0), a.NG - g0);
        const int g = g0 + w;
        const bool real = !loader && w < nw;
        const int j0 = 1 + 64 * g;
        const int jrow = j0 + lane;
        int gav = 0;
        uint32_t bc = 0;

        if (loader) {
            // ---------------- loader wave: ring 0 + the string window ----------------
            const bool seeded = sidx == 0 && !a.xin;
            const bool xsrc = sidx == 0 && a.xin;
            const uint64_t* gin = xsrc ? a.xin : a.gran + (int64_t)(sidx % a.nslot) * a.gpitch;
            const uint32_t want = xsrc ? a.epoch : a.gtag | (uint32_t)sidx;
            const int wk = lane >> 3, wb = lane & 7;   // window copy, byte of the chunk
            // Granule window: lane l holds granule (cw + l/8, column l%8), so
            // one load covers 8 chunks; pn prefetches the next 8.  A poll
            // reloads only the lanes of chunks >= c that are not valid yet.
            const int64_t ngr = (int64_t)CH * NC1;
            auto gload = [&](int cf) -> uint64_t {
                const int64_t x = (int64_t)CH * cf + lane;
                return x < ngr ? ld_gran(gin + x, xsrc) : 0ull;
            };
            // Top-string window (lanes 0..15: the 16 dwords of chunks cw..cw+7),
            // prefetched one window ahead like the granules: no per-chunk
            // dependent global load paces the loader (see the pair kernel's loader).
            const int64_t nsw = 2 * (int64_t)NC1 + 16;
            auto sload = [&](int cf) -> uint32_t {
                const int64_t x = 2 * (int64_t)cf + lane;
                return lane < 16 && x < nsw ? reinterpret_cast<const uint32_t*>(a.s1)[x] : 0u;
            };
            int cw = 0;
            uint64_t pf = 0, pn = 0;
            uint32_t sw = sload(0), swn = sload(CH);
            if (!seeded) {
                pf = gload(0);
                pn = gload(CH);
            }
            for (int c = 0; c < NC1; ++c) {
                const int n = (c == NC1 - 1) ? nlast : CH;
                if (c == cw + CH) {
                    cw += CH;
                    pf = pn;
                    sw = swn;
                    if (!seeded) pn = gload(cw + CH);
                    swn = sload(cw + CH);
                }
                while (lds_ld(&ctr[1]) < c - R + 1) __builtin_amdgcn_s_sleep(1);
                int* dst = &tring[(c % R) * SLOT];
                if (seeded) {
                    if (lane < CH) dst[lane] = -(CH * c + lane + 1) * d;   // H[i][0] = -i*d (computation.c:102-110)
                } else {
                    const bool mine = wk == c - cw;           // this lane carries chunk c
                    bool ok = !mine || wb >= n || (uint32_t)(pf >> 32) == want;
                    if (!__all(ok)) {
                        const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
                        for (;;) {
                            __builtin_amdgcn_s_sleep(1);
                            if (wk >= c - cw && (uint32_t)(pf >> 32) != want) pf = gload(cw);
                            ok = !mine || wb >= n || (uint32_t)(pf >> 32) == want;
                            if (__all(ok)) break;
                            const int64_t now = (int64_t)__builtin_amdgcn_s_memrealtime();
                            const uint32_t ab = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
                            const bool peer = xsrc && __any(mine && wb < n && (uint32_t)(pf >> 32) == (want | POISON_BIT));
                            if (ab || peer || now - t0 > a.spin_ticks) {
                                if (lane == 0) {
                                    __hip_atomic_store(&a.ctl[CTL_ABORT], 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                                    if (!ab)
                                        atomicCAS(&a.ctl[CTL_ERR], 0u,
                                                  (uint32_t)(peer ? NW_ERR_PEER : NW_ERR_TIMEOUT));
                                    __hip_atomic_store(&sh_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                                break;
                            }
                        }
                    }
                    if (lds_ld(&sh_abort)) break;
                    if (mine) dst[wb] = (int)(uint32_t)pf + d;                 // granules carry H - d
                    if (xsrc && mine && wb < n && CH * c + wb < a.L1) a.row0[CH * c + wb] = (int)(uint32_t)pf;
                }
                // window: copy k holds column p + 1 + k at position p
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)sw, 2 * (c - cw));
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)sw, 2 * (c - cw) + 1);
                const uint8_t pc = (uint8_t)((wb < 4 ? lo : hi) >> (8 * (wb & 3)));
                swin[wk * SWN + ((CH * c + wb - wk) & (SWN - 1))] = pc;
                lds_order();
                if (lane == 0) lds_publish(&ctr[2], c + 9);   // prog = slots done + 8
            }
            if (xsrc) xcredit_post(a);
        } else if (real) {
            // ---------------- compute wave: its 64-row stripe, 8 steps per chunk ----
            uint64_t* gout = a.gran + (int64_t)((sidx + 1) % a.nslot) * a.gpitch;
            int32_t* hb = a.H + (int64_t)g * a.spitch;                 // moves every super-chunk
            uint32_t* db = a.D + (int64_t)g * (NCH + 1) * 64 + 64;     // (row 0 of the code tile pads)
            int hv = lane * 16, dv = lane * 4;                         // byte offsets from hb / db
            const bool publish = (w == nw - 1) && sidx + 1 < a.NSW;
            const bool xpublish = a.xout && g == a.NG - 1;
            if (xpublish && !xcredit_wait(a, &sh_abort) && lane == 0)
                __hip_atomic_store(&sh_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const bool out_lane = jrow <= a.L2;
            const int* tin = &tring[w * R * SLOT];
            int* tout = &tring[(w + 1) * R * SLOT];
            const int* cin = &ctr[2 * w + 1];          // {cons[w], prog[w], cons[w+1]}
            SkewConst kc;
            kc.c2 = a.s2[jrow - 1];
            kc.vcm = vcm;
            kc.vck = vck;
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                kc.sd[s] = s * d;
                kc.kd[s] = -(s + 1) * d;
                asm volatile("" : "+v"(kc.sd[s]), "+v"(kc.kd[s]));   // keep the constants in VGPRs
            }
            asm volatile("" : "+v"(kc.c2), "+v"(kc.vcm), "+v"(kc.vck));
            kc.pl = kc.ph = 0;
            if (PROF) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t b = (uint32_t)((uint32_t)q == kc.c2 ? vcm : vck) & 0xffu;
                    if (q < 4) kc.pl |= b << (8 * q);
                    else kc.ph |= b << (8 * (q - 4));
                }
            }
            kc.cb = lds_addr(&ctr[2 * w]);
            asm volatile("" : "+v"(kc.cb));
            // this lane's window: copy (-l) & 7, its chunks lag ceil(l / 8)
            const int wbase = lds_addr(&swin[((-lane) & 7) * SWN]);
            const int wo = (lane + 7) >> 3;
            auto waddr = [&](int c) { return wbase + ((CH * (c - wo)) & (SWN - 1)); };
            // Ring writes of the generated block: lane 63 into the slot, the
            // other lanes into a per-lane dummy (conflict-free, no exec juggling).
            const int ring0 = lane == 63 ? lds_addr(tout) : lds_addr(&scratch[lane]);
            int ra[R], rd[R];
#pragma unroll
            for (int q = 0; q < R; ++q) {
                ra[q] = ring0 + q * SLOT * 4;
                rd[q] = lds_addr(tin) + q * SLOT * 4;
                asm volatile("" : "+v"(ra[q]), "+v"(rd[q]));
            }
            const int C0 = -(a.row_base + j0) * d;     // column 0 (and row j0-1 at column 0)
            SkewRegs r;
            r.ein = C0;
            r.upc = C0;
            r.gav = 0;
            int base = 0;
            int done = 0;                              // ring slots published to the wave below
            bool aborted = false;
            if (a.trace && lane == 0 && w == 0) {
                a.trace[8 * (int64_t)sidx + 1] = __builtin_amdgcn_s_memrealtime();
                a.trace[8 * (int64_t)sidx + 4] = __builtin_amdgcn_s_memtime();
            }
            // Granules of ring slot q (the WG-stripe's / panel's bottom row).
            auto publish_slot = [&](int q) {     // (q >= 0; only the publishing waves call it)
                const int n = (q == NC1 - 1) ? nlast : CH;
                if (lane < n) {
                    const int v = tout[(q & (R - 1)) * SLOT + lane] - d;        // granules carry H - d
                    const uint64_t tag = publish ? a.gtag | (uint32_t)(sidx + 1) : a.epoch;
                    const uint64_t gr = (tag << 32) | (uint32_t)v;
                    if (publish)
                        put_granule(gout, CH * (int64_t)q + lane, gr);
                    else
                        __hip_atomic_store(a.xout + CH * (int64_t)q + lane, gr, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (xpublish && a.xflag && ((q + 1) % a.xblk == 0 || q == NC1 - 1)) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0)
                        __hip_atomic_store(&a.xflag[q / a.xblk], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            };
            // Per-chunk state of the middle run: Pc = (8c - base)*d (lane-0
            // pre-fill offset, -Pc the score offset), cv = c + 1, wa = this
            // lane's window address of chunk c + 1.
            int Pc = 0, cv = 0, wa = 0;
            auto rebase = [&](int c) {
                if (c > 0 && c % SUPER_CHUNKS == 0) {
                    const int sh = SUPER_CHUNKS * CH * d;
                    r.ein -= sh;
                    r.upc -= sh;
                    Pc -= sh;
                    base += SUPER_CHUNKS * CH;
                    hb += SUPER_CHUNKS * 512;
                    hv -= SUPER_CHUNKS * 2048;
                    db += SUPER_CHUNKS * 64;
                    dv -= SUPER_CHUNKS * 256;
                }
            };
            // ---- generic chunk (prologue / epilogue, every lane checked) ----
            auto generic_chunk = [&](int c) -> bool {
                const bool need_in = c < NC1;
                for (;;) {
                    const int pin = uni(lds_ld(&cin[1]));
                    const int pout = uni(lds_ld(&cin[2]));
                    if ((!need_in || pin > c + 8) && pout >= c - 6 - R) break;
                    if (uni(lds_ld(&sh_abort))) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
                lds_order();
                int T[CH];
#pragma unroll
                for (int s = 0; s < CH; ++s) T[s] = need_in ? tin[(c % R) * SLOT + s] : 0;
                lds_order();
                if (need_in && lane == 0) lds_publish(&ctr[2 * w + 1], c + 1);
                const uint64_t wv = *reinterpret_cast<const uint64_t*>(&swin[0] + (waddr(c) - lds_addr(&swin[0])));
                const int off = (CH * c + 1 - base) * d;     // E - H at step 8c
                int h[CH];
                uint32_t acc = 0;
#pragma unroll
                for (int s = 0; s < CH; ++s) {
                    const int t = CH * c + s;
                    const int up0 = T[s] + off + (s - 1) * d;                          // H(row above) - d, in E
                    const int up = __builtin_amdgcn_update_dpp(up0, r.ein, 0x138, 0xf, 0xf, false);   // wave_shr:1
                    const uint32_t sym = (uint32_t)(wv >> (8 * s)) & 0xffu;
                    const int dg = r.upc + (sym == kc.c2 ? vcm : vck);
                    int En = max(max(r.ein, up), dg);
                    const int i = t - lane + 1;
                    if (c < 8 && i < 1) En = C0;                                       // column 0 (prologue)
                    const uint32_t code = (dg == En ? 1u : 0u) | (up == En ? 2u : 0u) | (r.ein == En ? 4u : 0u);
                    acc = (acc << 3) | code;
                    const int H = En - off - s * d;
                    h[s] = H;
                    const bool valid = i >= 1 && i <= a.L1;
                    if (ST && valid && out_lane) {
                        r.gav = max(r.gav, H < 0 ? -H : H);
                        bc += (code & (code - 1)) ? 1u : 0u;
                    }
                    if (lane == 63 && valid) tout[(((i - 1) >> 3) % R) * SLOT + ((i - 1) & 7)] = H;
                    if (!SH && i == a.L1) a.lastcol[jrow] = H;
                    r.upc = up;
                    r.ein = En;
                }
                if (SH) skew_store_scores(h, hb, hv);
                if (SD) skew_store_code(acc, db, dv);
                // ring slots completed by lane 63 (column 8c - 55 after this chunk)
                const int ndone = (CH * c - 55 >= a.L1) ? NC1 : min(NC1, max(0, c - 7));
                if (publish || xpublish)
                    for (int q = done; q < ndone; ++q) publish_slot(q);
                if (ndone > done) {
                    done = ndone;
                    lds_order();
                    if (lane == 0) lds_publish(&ctr[2 * w + 4], done + 8);
                }
                return true;
            };
            // ---- middle chunks: every lane has a real cell in all 8 steps ----
            // (8 <= c and 8c + 8 <= L1): the generated block.  cv = c + 1 is
            // both cons[w] (slot c taken) and prog[w+1] (slots done + 8).
            const int cmid = NC1 - 1;   // the chunk where lane 0 reaches column L1 stays generic (last column)
            SkewSlot tA, tB;
            auto wait_slot = [&](int c, SkewSlot& tt) -> bool {
                for (;;) {
                    const uint64_t pq = skew_read_slot(kc.cb, rd[c % R], waddr(c), tt);
                    const int pin = uni((int)(uint32_t)pq), pout = uni((int)(pq >> 32));
                    if (pin > c + 8 && pout >= c - 6 - R) return true;
                    if (uni(lds_ld(&sh_abort))) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            auto mid_chunk = [&](int c, auto slotc, const SkewSlot& cur, SkewSlot& nxt) -> bool {
                constexpr int Q = decltype(slotc)::value;
                skew_chunk_asm<ST, PROF>(r, kc, cur, nxt, Pc, -Pc, cv, ra[Q], ra[(Q + 1) % R], rd[(Q + 1) % R], wa);
                if (SH) skew_store_scores(r.h, hb, hv);
                if (SD) skew_store_code(r.acc, db, dv);
                hv += 2048;
                dv += 256;
                Pc += CH * d;
                cv += 1;
                wa = (wa & ~(SWN - 1)) | ((wa + CH) & (SWN - 1));
                if (ST) bc += branch_codes(out_lane ? r.acc : 0u);
                if (publish || xpublish) publish_slot(c - 8);
                if (c + 1 >= cmid) return true;      // the next chunk is generic: it waits itself
                // (prog[w] > c + 9 and cons[w+1] >= c - 5 - R, as one sign test: the common case falls through)
                if (__builtin_expect(((uni((int)(uint32_t)r.pq) - (c + 10)) | (uni((int)(r.pq >> 32)) - (c - 5 - R))) >= 0, 1))
                    return true;
                return wait_slot(c + 1, nxt);
            };
            using S0 = std::integral_constant<int, 0>;
            using S1 = std::integral_constant<int, 1>;
            using S2 = std::integral_constant<int, 2>;
            using S3 = std::integral_constant<int, 3>;
            if (a.trace && lane == 0 && w == nw - 1) a.trace[8 * (int64_t)sidx + 6] = __builtin_amdgcn_s_memrealtime();
            int c = 0;
            for (; c < min(8, NCH) && !aborted; ++c) {
                aborted = !generic_chunk(c);
                hv += 2048;
                dv += 256;
            }
            if (!aborted && c < cmid) {
                aborted = !wait_slot(c, tA);
                Pc = uni((CH * c - base) * d);
                cv = c + 1;
                wa = waddr(c + 1);
                // c = 8: c % R == 0, so the unrolled slots line up
                while (c + R <= cmid && !aborted) {
                    rebase(c);
                    aborted = !mid_chunk(c, S0{}, tA, tB) || !mid_chunk(c + 1, S1{}, tB, tA) ||
                              !mid_chunk(c + 2, S2{}, tA, tB) || !mid_chunk(c + 3, S3{}, tB, tA);
                    c += R;
                }
                if (!aborted && c < cmid) {
                    rebase(c);
                    aborted = !mid_chunk(c, S0{}, tA, tB);
                    if (!aborted && c + 1 < cmid) aborted = !mid_chunk(c + 1, S1{}, tB, tA);
                    if (!aborted && c + 2 < cmid) aborted = !mid_chunk(c + 2, S2{}, tA, tB);
                    c = cmid;
                }
                done = cmid - 8;     // slots the middle run published (prog = cmid = done + 8)
            }
            for (; c < NCH && !aborted; ++c) {
                rebase(c);
                aborted = !generic_chunk(c);
                hv += 2048;
                dv += 256;
            }
            gav = r.gav;
        }
        if (a.trace && !loader && w == nw - 1 && lane == 0) {
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

template <int W, bool P>
KernelFn pick_flags(bool sh, bool sd, bool stt) {
    if (sh && sd) return stt ? nw_skew_kernel<W, true, true, true, P> : nw_skew_kernel<W, true, true, false, P>;
    if (sh) return stt ? nw_skew_kernel<W, true, false, true, P> : nw_skew_kernel<W, true, false, false, P>;
    if (sd) return stt ? nw_skew_kernel<W, false, true, true, P> : nw_skew_kernel<W, false, true, false, P>;
    return stt ? nw_skew_kernel<W, false, false, true, P> : nw_skew_kernel<W, false, false, false, P>;
}

template <int W>
KernelFn pick_prof(bool prof, bool sh, bool sd, bool stt) {
    return prof ? pick_flags<W, true>(sh, sd, stt) : pick_flags<W, false>(sh, sd, stt);
}

}  // namespace

KernelFn pick_skew(int W, bool prof, bool sh, bool sd, bool stt) {
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
        case 15: return pick_prof<15>(prof, sh, sd, stt);
        default: return nullptr;
    }
}

}  // namespace nwk
