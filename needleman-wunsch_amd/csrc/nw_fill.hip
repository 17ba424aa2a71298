// nw_fill.hip -- MI355X (gfx950) Needleman-Wunsch score-table fill + C ABI.
//
// Replaces the reference hot path compute_table_scores()
// (needleman-wunsch.c:583-626 -> score_cell_column_set :557-574 ->
// score_cell_column :523-543 -> score_cell :418-510 -> max3 :395-404) and the
// table storage/seeding it relies on (score-table.c:60-81,
// walk-table.c:58-79, computation.c:75-125).  See DESIGN.md for the full
// derivation; in short:
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
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nw_internal.h"

namespace {

constexpr int CH = 8;                 // columns per chunk (= codes per dirs word)
constexpr int64_t SPIN_TICKS = 200000000;  // 2 s of s_memrealtime (100 MHz)
// Panel boundary granule tags: the fill's epoch (1 .. 2^31-1), or the epoch
// with bit 31 set when the panel above failed that fill (per-epoch, so a stale
// poison never trips a later fill).
constexpr uint32_t POISON_BIT = 0x80000000u;

enum CtlWord { CTL_NEXT = 0, CTL_ABORT = 1, CTL_GAV = 2, CTL_BC = 3, CTL_ERR = 4, CTL_WORDS = 16 };

struct FillArgs {
    const uint8_t* s1;      // device, zero-padded to >= 8*NC + 8 bytes (s1[i-1] = column i)
    const uint8_t* s2;      // device, zero-padded to >= 64*NG + 64 bytes
    int32_t L1, L2;
    int32_t m, k, d;
    int32_t NC;             // chunks = ceil(L1 / 8)
    int32_t NG;             // wave stripes = ceil(L2 / 64)
    int32_t NSW;            // workgroup stripes = ceil(NG / W)
    int32_t* H;             // score tiles, see score_at()
    int64_t spitch;         // 512*NC: elements per 64-row stripe
    uint32_t* D;            // codes: word ((g*NC + q)*64 + lane)
    int32_t* lastcol;       // score-only: H[L1][j] at lastcol[63 + j]
    uint64_t* gran;         // boundary granules, slot s at gran + s*gpitch
    int64_t gpitch;
    int32_t nslot;
    uint32_t* ctl;          // CtlWord
    uint64_t* trace;        // optional timeline: 4 words per WG-stripe (see nw_table_trace)
    int64_t spin_ticks;     // hand-off watchdog (s_memrealtime ticks)
    // Row panels (multi-GPU, nw_panel.h).  The table holds global rows
    // row_base+1 .. row_base+L2; row 0 is the boundary row of the panel above.
    int32_t row_base;
    uint32_t epoch;         // tag of this fill's panel hand-off granules
    const uint64_t* xin;    // top boundary row {epoch, H-d} per column, or null (= seeded row 0)
    uint64_t* xout;         // bottom row granules for the panel below, or null
    uint32_t* xflag;        // host-visible: xflag[b] = epoch once block b of xout is written
    int32_t xblk;           // chunks per block
};

// ---------------------------------------------------------------- DPP helpers
// wave_shr:1 -- lane l receives lane l-1; lane 0 keeps `old`.
__device__ __forceinline__ int wave_shr1(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false);
}

typedef const __attribute__((address_space(4))) uint64_t* cptr64;

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t u32x4(int a, int b, int c, int d) {
    return u32x4_t{(unsigned)a, (unsigned)b, (unsigned)c, (unsigned)d};
}

__device__ __forceinline__ int iabs(int v) { return v < 0 ? -v : v; }

// Count nibbles of a codes word that have >= 2 of their 3 direction bits.
__device__ __forceinline__ uint32_t branch_nibbles(uint32_t x) {
    uint32_t y = (x & (x >> 1)) | (x & (x >> 2)) | ((x >> 1) & (x >> 2));
    return __builtin_popcount(y & 0x11111111u);
}

// Wave-uniform copies of per-wave values (so address math stays scalar).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------ per-wave state
struct WaveState {
    int G;          // shifted score of this lane's row at the last column
    int Tprev;      // lane -1 (row above the stripe) shifted score, last column
    uint32_t c2;    // this lane's side-string byte
    int laneoff;    // (64*w + lane) * d: H = G - laneoff
    int gav;        // running max |H| (stats)
    uint32_t bc;    // running branch count (stats)
};

// One 8-column chunk of one wave.  NSTEP is 8 except for the last chunk.
// Cell recurrence = needleman-wunsch.c:429-465; direction flags :485-503.
// ----------------------------------------------------------- step kernels
// One column step of one wave, hand-scheduled.  The loop-carried chain is
//   G --dpp wave_shr:1--> sh --add--> dg --max3(lf,dg,top)--> Y --6 x dpp max--> G'
// and every DPP read of a VGPR written by the previous VALU needs two wait
// states.  Instead of s_nop, those slots carry the *previous* step's
// independent outputs: its direction code (3 compares, shifted into `acc`
// with v_addc: acc = 16*acc + diag + 2*up + 4*left), its score H = G - laneoff
// and (stats) the running max |H|.  The previous step's up candidate is this
// step's `sh` (wave_shr:1 of G with lane 0 = row above), so it comes free.
#define NW_STEP_HEAD                                                   \
    "v_cmp_eq_u32_e32 vcc, %[ch], %[c2]\n\t"                           \
    "v_cndmask_b32_e32 %[sub], %[ck], %[cm], vcc\n\t"                  \
    "v_mov_b32_dpp %[sh], %[G] wave_shr:1 row_mask:0xf bank_mask:0xf\n\t" \
    "v_subrev_u32_e32 %[lf], %[d], %[G]\n\t"                           \
    "v_add_u32_e32 %[dg], %[sh], %[sub]\n\t"                           \
    "v_max3_i32 %[Y], %[lf], %[dg], %[top]\n\t"
#define NW_DPP(CTRL) "v_max_i32_dpp %[Y], %[Y], %[Y] " CTRL "\n\t"
#define NW_FILL_A                                                      \
    "v_cmp_eq_i32_e64 %[sa], %[pG], %[pdg]\n\t"                        \
    "v_cmp_eq_i32_e64 %[sb], %[pG], %[sh]\n\t"
#define NW_FILL_B                                                      \
    "v_cmp_eq_i32_e32 vcc, %[pG], %[plf]\n\t"                          \
    "v_lshlrev_b32_e32 %[acc], 1, %[acc]\n\t"
#define NW_FILL_C                                                      \
    "v_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], vcc\n\t"       \
    "v_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], %[sb]\n\t"
#define NW_FILL_D                                                      \
    "v_addc_co_u32_e64 %[acc], %[junk], %[acc], %[acc], %[sa]\n\t"     \
    "v_sub_u32_e32 %[Hp], %[pG], %[lo]\n\t"
#define NW_FILL_E                                                      \
    "v_sub_u32_e32 %[tmp], 0, %[Hp]\n\t"                               \
    "v_max3_i32 %[gav], %[gav], %[Hp], %[tmp]\n\t"
#define NW_NOP2 "s_nop 1\n\t"
#define NW_SCAN_FILLED(E)                                              \
    NW_FILL_A NW_DPP("row_shr:1 row_mask:0xf bank_mask:0xf")           \
    NW_FILL_B NW_DPP("row_shr:2 row_mask:0xf bank_mask:0xf")           \
    NW_FILL_C NW_DPP("row_shr:4 row_mask:0xf bank_mask:0xf")           \
    NW_FILL_D NW_DPP("row_shr:8 row_mask:0xf bank_mask:0xf")           \
    E         NW_DPP("row_bcast:15 row_mask:0xa bank_mask:0xf")        \
    NW_NOP2   "v_max_i32_dpp %[Y], %[Y], %[Y] row_bcast:31 row_mask:0xc bank_mask:0xf"
#define NW_SCAN_BARE                                                   \
    NW_NOP2 NW_DPP("row_shr:1 row_mask:0xf bank_mask:0xf")             \
    NW_NOP2 NW_DPP("row_shr:2 row_mask:0xf bank_mask:0xf")             \
    NW_NOP2 NW_DPP("row_shr:4 row_mask:0xf bank_mask:0xf")             \
    NW_NOP2 NW_DPP("row_shr:8 row_mask:0xf bank_mask:0xf")             \
    NW_NOP2 NW_DPP("row_bcast:15 row_mask:0xa bank_mask:0xf")          \
    NW_NOP2 "v_max_i32_dpp %[Y], %[Y], %[Y] row_bcast:31 row_mask:0xc bank_mask:0xf"

struct StepIO {
    int G, sh, dg, lf;      // this step: new G (out), shift / diag / left candidates
    int pG, pdg, plf;       // previous step (inputs of the filled outputs)
    int Hp;                 // previous step's score (out)
    uint32_t acc;           // direction codes accumulator
    int gav;                // running max |H|
};

// MODE 0: first step of a chunk (nothing pending), 1: fill with the previous
// step's code + score, 2: also its |H| for the stats.
template <int MODE>
__device__ __forceinline__ void step_asm(StepIO& io, int Tprev, int top, uint32_t ch, uint32_t c2, int vck, int vcm,
                                         int d, int laneoff) {
    int Y, sub, tmp;
    uint64_t sa, sb, junk;
    int sh = Tprev;  // DPP lane 0 keeps the old value: the row above
#define NW_OPERANDS                                                                              \
    : [Y] "=&v"(Y), [sh] "+v"(sh), [sub] "=&v"(sub), [dg] "=&v"(io.dg), [lf] "=&v"(io.lf),        \
      [Hp] "=&v"(io.Hp), [acc] "+v"(io.acc), [gav] "+v"(io.gav), [tmp] "=&v"(tmp), [sa] "=&s"(sa), \
      [sb] "=&s"(sb), [junk] "=&s"(junk)                                                          \
    : [G] "v"(io.G), [ch] "s"(ch), [c2] "v"(c2), [ck] "v"(vck), [cm] "v"(vcm), [d] "s"(d),       \
      [top] "v"(top), [pG] "v"(io.pG), [pdg] "v"(io.pdg), [plf] "v"(io.plf), [lo] "v"(laneoff)    \
    : "vcc"
    if constexpr (MODE == 0) {
        asm volatile(NW_STEP_HEAD NW_SCAN_BARE NW_OPERANDS);
    } else if constexpr (MODE == 1) {
        asm volatile(NW_STEP_HEAD NW_SCAN_FILLED(NW_NOP2) NW_OPERANDS);
    } else {
        asm volatile(NW_STEP_HEAD NW_SCAN_FILLED(NW_FILL_E) NW_OPERANDS);
    }
#undef NW_OPERANDS
    io.sh = sh;
    io.G = Y;
}

// One 8-column chunk of one wave.  NSTEP is 8 except for the last chunk.
// Cell recurrence = needleman-wunsch.c:429-465; direction flags :485-503.
// In the shifted domain G = H + r*d each column is a prefix max over lanes:
//     G_i = prefmax( max(G_{i-1} - d, G_{i-1}[l-1] + sub_i, T_i) ).
template <bool SH, bool SD, bool ST, bool LAST>
__device__ __forceinline__ void chunk_body(const FillArgs& a, WaveState& st, const int* T, uint64_t ch8, int c,
                                           int nstep, int lane, int64_t tile_off, int j0, int d, int vcm, int vck,
                                           int* bot_wr, uint32_t* dword_out) {
    // Buffer descriptor on this chunk's two column quads (2 KB contiguous in
    // the stripe-major quad layout): lane l stores its 4 consecutive columns
    // as one 16-byte buffer_store_dwordx4 at lane*16 (+1024 for the 2nd quad).
    int32_t* cb = a.H + tile_off + (int64_t)c * 512;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cb, 0, 0x7fffffff, 0x00020000);
    StepIO io;
    io.G = st.G;
    io.acc = 0;
    io.gav = st.gav;
    io.pG = io.pdg = io.plf = 0;
    int Tprev = st.Tprev;
    int h[CH];
#pragma unroll
    for (int s = 0; s < CH; ++s) {
        if (LAST && s >= nstep) break;
        const uint32_t ch = (uint32_t)(ch8 >> (8 * s)) & 0xffu;
        if (s == 0) step_asm<0>(io, Tprev, T[s], ch, st.c2, vck, vcm, d, st.laneoff);
        else if (ST) step_asm<2>(io, Tprev, T[s], ch, st.c2, vck, vcm, d, st.laneoff);
        else step_asm<1>(io, Tprev, T[s], ch, st.c2, vck, vcm, d, st.laneoff);
        if (s > 0) h[s - 1] = io.Hp;
        if (SH && !LAST && s == 4)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4(h[0], h[1], h[2], h[3]), rs, lane * 16, 0, 0);
        bot_wr[s] = io.G;   // lane 63 -> bottom-row slot, lanes 0..62 -> scratch
        io.pG = io.G;
        io.pdg = io.dg;
        io.plf = io.lf;
        Tprev = T[s];
    }
    // Outputs of the chunk's last step (not overlapped).
    const int slast = LAST ? nstep - 1 : CH - 1;
    const int up = wave_shr1(Tprev, io.G);
    const int Hv = io.G - st.laneoff;
    h[slast] = Hv;
    if (SH) {
        if (LAST) {
            // partial chunk: unused slots land in the quad padding
            __builtin_amdgcn_raw_buffer_store_b128(u32x4(h[0], nstep > 1 ? h[1] : 0, nstep > 2 ? h[2] : 0,
                                                             nstep > 3 ? h[3] : 0), rs, lane * 16, 0, 0);
            if (nstep > 4)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4(h[4], nstep > 5 ? h[5] : 0, nstep > 6 ? h[6] : 0,
                                                                 nstep > 7 ? h[7] : 0), rs, lane * 16 + 1024, 0, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4(h[4], h[5], h[6], h[7]), rs, lane * 16 + 1024, 0, 0);
        }
    }
    uint32_t acc = (io.acc << 4) | (uint32_t)(io.G == io.dg) | ((uint32_t)(io.G == up) << 1) |
                   ((uint32_t)(io.G == io.lf) << 2);
    if (ST) io.gav = max(io.gav, iabs(Hv));
    if (LAST && !SH) a.lastcol[j0 + lane] = Hv;            // score-only: H[L1][*]
    if (LAST && nstep < CH) acc <<= 4 * (CH - nstep);
    st.G = io.G;
    st.Tprev = Tprev;
    st.gav = io.gav;
    *dword_out = acc;
}

// Hand-off granule load: agent scope between workgroups of one fill, system
// scope (bypassing L2) for the panel boundary, which another agent writes.
__device__ __forceinline__ uint64_t ld_gran(const uint64_t* p, bool sys) {
    return sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
               : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS counters of the barrier-free intra-workgroup pipeline.
__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(int* p, int v) {
    // Every LDS write this wave issued before (ring data) completes first:
    // LDS is in-order per wave, and the wait makes the counter the last word.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup = W compute waves (64-row stripes, stacked) + 1 loader wave, no
// barriers inside a stripe.  Wave w takes the top row of each 8-column chunk
// from an LDS ring tring[w] (R chunk slots) filled by its producer (the
// loader for w = 0, wave w-1 otherwise) and puts its own bottom row into
// tring[w+1].  prog[w] = chunks available in tring[w], cons[w] = chunks wave w
// has taken out of it; a producer only waits when it is R chunks ahead.
// The loader feeds tring[0] from the previous WG-stripe's granules; it issues
// no stores, so its waits on the hand-off loads are exact, and the compute
// waves never wait on vmcnt.
template <int W, bool SH, bool SD, bool ST>
__global__ __launch_bounds__(64 * (W + 1)) void nw_fill_kernel(FillArgs a) {
    constexpr int R = 4;
    __shared__ __attribute__((aligned(16))) int tring[(W + 1) * R * CH];
    __shared__ int scratch[64 + CH];
    __shared__ int prog[W + 1];
    __shared__ int cons[W + 1];
    __shared__ int sh_sidx;
    __shared__ int sh_abort;

    const int lane = threadIdx.x & 63;
    const int w = uni(threadIdx.x >> 6);
    const bool loader = (w == W);
    const int d = a.d;
    int vcm = a.m + a.d;
    int vck = a.d - a.k;
    asm volatile("" : "+v"(vcm), "+v"(vck));   // keep both as VGPR operands of v_cndmask
    const int NC = a.NC;
    const int nlast = a.L1 - CH * (NC - 1);   // steps in the last chunk (1..8)

    for (;;) {
        if (threadIdx.x == 0) {
            sh_sidx = (int)atomicAdd(&a.ctl[CTL_NEXT], 1u);
            sh_abort = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        }
        if (threadIdx.x <= W) {
            prog[threadIdx.x] = 0;
            cons[threadIdx.x] = 0;
        }
        __syncthreads();
        const int sidx = uni(sh_sidx);
        if (sidx >= a.NSW || sh_abort) break;
        if (a.trace && threadIdx.x == 0) {
            a.trace[4 * (int64_t)sidx + 0] = __builtin_amdgcn_s_memrealtime();
            a.trace[4 * (int64_t)sidx + 3] = (uint64_t)blockIdx.x | ((uint64_t)__smid() << 32);
        }

        const int g = sidx * W + w;                // wave stripe (compute waves)
        const bool real = !loader && g < a.NG;
        const bool next_real = !loader && w + 1 < W && g + 1 < a.NG;
        const int j0 = 1 + 64 * g;                 // first row of the wave stripe
        const int jrow = j0 + lane;
        WaveState st;
        st.G = 0;
        st.gav = 0;
        st.bc = 0;

        if (loader) {
            // ---------------- loader wave: no stores, exact waits ----------------
            // Source of the WG-stripe's top row: the seeded row 0, the panel
            // above (xin, written by another agent: system-scope loads), or
            // the previous WG-stripe's granules (agent scope).
            const bool seeded = sidx == 0 && !a.xin;
            const bool xsrc = sidx == 0 && a.xin;
            const uint64_t* gin = xsrc ? a.xin : a.gran + (int64_t)(sidx % a.nslot) * a.gpitch;
            const uint32_t want = xsrc ? a.epoch : (uint32_t)sidx;
            uint64_t pf = 0;
            if (!seeded && lane < CH) pf = ld_gran(gin + lane, xsrc);
            for (int c = 0; c < NC; ++c) {
                const int n = (c == NC - 1) ? nlast : CH;
                while (lds_ld(&cons[0]) < c - R + 1) __builtin_amdgcn_s_sleep(1);   // ring slot free?
                int* dst = &tring[(c % R) * CH];
                if (seeded) {
                    // row 0: H[i][0] - d = -(i+1)*d   (computation.c:102-110)
                    if (lane < CH) dst[lane] = -(CH * c + 2 + lane) * d;
                } else {
                    bool ok = lane >= n || (uint32_t)(pf >> 32) == want;
                    if (!__all(ok)) {
                        const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
                        for (;;) {
                            __builtin_amdgcn_s_sleep(1);
                            if (!ok) pf = ld_gran(gin + CH * (int64_t)c + lane, xsrc);
                            ok = lane >= n || (uint32_t)(pf >> 32) == want;
                            if (__all(ok)) break;
                            const int64_t now = (int64_t)__builtin_amdgcn_s_memrealtime();
                            const uint32_t ab = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT);
                            // a failed panel above poisons its boundary row
                            const bool peer = xsrc && __any(lane < n && (uint32_t)(pf >> 32) == (want | POISON_BIT));
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
                    if (lane < CH) dst[lane] = (int)(uint32_t)pf;
                    if (c + 1 < NC && lane < CH)          // prefetch the next chunk
                        pf = ld_gran(gin + CH * (int64_t)(c + 1) + lane, xsrc);
                }
                if (lane == 0) lds_publish(&prog[0], c + 1);
            }
        } else if (real) {
            // ---------------- compute wave: its 64-row stripe, chunk by chunk ----
            uint64_t* gout = a.gran + (int64_t)((sidx + 1) % a.nslot) * a.gpitch;
            const int64_t tile_off = (int64_t)g * a.spitch;
            st.c2 = a.s2[jrow - 1];
            st.laneoff = (64 * w + lane) * d;
            // column 0: H[0][j] = -j*d  ->  G = -(1 + row_base + 64*sidx*W)*d for every lane.
            st.G = -(1 + a.row_base + 64 * sidx * W) * d;
            st.Tprev = st.G;
            const bool publish = (w == W - 1) && sidx + 1 < a.NSW;
            // The wave holding the panel's last row (lane 63: panels above the
            // last one have a multiple of 64 rows) feeds the panel below.
            const bool xpublish = a.xout && g == a.NG - 1;
            const int* tin = &tring[w * R * CH];
            if (a.trace && lane == 0 && w == 0) a.trace[4 * (int64_t)sidx + 1] = __builtin_amdgcn_s_memrealtime();
            // Chunk prologue, software-pipelined one chunk ahead: the s1 bytes
            // (s_load), our producer's progress, the ring slot and our
            // consumer's progress for chunk c+1 are all requested at the start
            // of chunk c and only checked at its end.  LDS is in order per
            // wave, so ring data read after a progress value that covers it is
            // valid.  (s_load shares lgkmcnt with LDS, so it is issued first.)
            uint64_t ch8 = *(cptr64)(a.s1);
            int pin = lds_ld(&prog[w]);
            int4 t03 = *reinterpret_cast<const int4*>(&tin[0]);
            int4 t47 = *reinterpret_cast<const int4*>(&tin[4]);
            int pout = next_real ? lds_ld(&cons[w + 1]) : (1 << 30);
            for (int c = 0; c < NC; ++c) {
                const int slot = (c % R) * CH;
                if (pin <= c || pout < c - R + 1) {
                    // slow path: producer behind (or ring full) -- wait, then re-read
                    for (;;) {
                        pin = lds_ld(&prog[w]);
                        pout = next_real ? lds_ld(&cons[w + 1]) : (1 << 30);
                        if ((pin > c && pout >= c - R + 1) || lds_ld(&sh_abort)) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (lds_ld(&sh_abort)) break;
                    t03 = *reinterpret_cast<const int4*>(&tin[slot]);
                    t47 = *reinterpret_cast<const int4*>(&tin[slot + 4]);
                }
                const int T[CH] = {t03.x, t03.y, t03.z, t03.w, t47.x, t47.y, t47.z, t47.w};
                const uint64_t ch8c = ch8;
                if (lane == 0) __hip_atomic_store(&cons[w], c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (c + 1 < NC) {
                    const int nslot = ((c + 1) % R) * CH;
                    ch8 = *(cptr64)(a.s1 + 8 * (int64_t)(c + 1));
                    pin = lds_ld(&prog[w]);
                    t03 = *reinterpret_cast<const int4*>(&tin[nslot]);
                    t47 = *reinterpret_cast<const int4*>(&tin[nslot + 4]);
                    if (next_real) pout = lds_ld(&cons[w + 1]);
                }
                int* bot_wr = (lane == 63) ? &tring[(w + 1) * R * CH + slot] : &scratch[lane];
                const int nstep = (c == NC - 1) ? nlast : CH;
                uint32_t dw;
                if (c == NC - 1)
                    chunk_body<SH, SD, ST, true>(a, st, T, ch8c, c, nstep, lane, tile_off, j0, d, vcm, vck, bot_wr, &dw);
                else
                    chunk_body<SH, SD, ST, false>(a, st, T, ch8c, c, CH, lane, tile_off, j0, d, vcm, vck, bot_wr, &dw);
                if (next_real && lane == 0) lds_publish(&prog[w + 1], c + 1);
                if (jrow > a.L2) dw = 0;
                if (SD) a.D[((int64_t)g * NC + c) * 64 + lane] = dw;
                if (ST) st.bc += branch_nibbles(dw);
                // Last wave of a non-final WG-stripe publishes its bottom row.
                if (publish) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane < nstep) {
                        const int v = tring[W * R * CH + slot + lane] - 64 * W * d;  // row-above domain
                        const uint64_t gr = ((uint64_t)(uint32_t)(sidx + 1) << 32) | (uint32_t)v;
                        __hip_atomic_store(gout + CH * (int64_t)c + lane, gr, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                if (xpublish) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane < nstep) {
                        const int v = tring[(w + 1) * R * CH + slot + lane] - 64 * (w + 1) * d;
                        const uint64_t gr = ((uint64_t)a.epoch << 32) | (uint32_t)v;
                        __hip_atomic_store(a.xout + CH * (int64_t)c + lane, gr, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    if (a.xflag && ((c + 1) % a.xblk == 0 || c == NC - 1)) {
                        // block complete: its granules are out before the flag
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0)
                            __hip_atomic_store(&a.xflag[c / a.xblk], a.epoch, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
        }
        if (a.trace && threadIdx.x == 64 * (W - 1)) a.trace[4 * (int64_t)sidx + 2] = __builtin_amdgcn_s_memrealtime();
        if (ST && real) {
            const bool rowok = jrow <= a.L2;
            int gv = rowok ? st.gav : 0;
            uint32_t bv = rowok ? st.bc : 0u;
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

// Device view of a filled table for the copy / hash kernels.
struct TableView {
    const int32_t* tiles;   // score tiles
    int64_t spitch;
    const uint32_t* D;      // codes, or null
    int32_t NC;
    int32_t d;
    int32_t row_base;       // panels: global row of local row 0
    const uint64_t* top;    // panels: boundary row granules (H - d), or null for row 0 = seed
};

// Score of cell (i, j) in the device layout.  Row 0 and column 0 are the
// reference's seeds (computation.c:93-120), computed, not stored; a panel's
// row 0 is the last row of the panel above, kept in its xin granules.
// Interior cells live in stripe-major quad tiles: stripe g = (j-1)/64, lane
// l = (j-1)%64, column quad q = (i-1)/4, r = (i-1)%4 at
//     g*spitch + (q*64 + l)*4 + r,   spitch = 512*NC,
// i.e. each lane's 4 consecutive columns are one 16-byte word and one quad of
// one stripe is 1 KB contiguous.
__device__ __forceinline__ int32_t score_at(const TableView& v, int64_t i, int64_t j) {
    if (i == 0) return (int32_t)(-(j + v.row_base) * (int64_t)v.d);
    if (j == 0) return v.top ? (int32_t)(uint32_t)v.top[i - 1] + v.d : (int32_t)(-i * (int64_t)v.d);
    const int64_t r = j - 1, c = i - 1;
    return v.tiles[(r >> 6) * v.spitch + (((c >> 2) * 64 + (r & 63)) << 2) + (c & 3)];
}

// Dense i-major copy of columns [i0, i1): out[(i-i0)*(L2+1) + j].
__global__ void nw_gather_scores_kernel(TableView v, int32_t L2, int64_t i0, int64_t i1, int32_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t n = (i1 - i0) * N;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = score_at(v, i0 + x / N, x % N);
}

// Direction code of cell (i, j).  A panel's row 0 belongs to the panel above
// and reads as 0 here.
__device__ __forceinline__ uint32_t code_at(const TableView& v, int64_t i, int64_t j) {
    if (j == 0 && v.row_base > 0) return 0u;
    if (i == 0) return j == 0 ? 0u : 2u;          // (0,0): none; (0,j): up
    if (j == 0) return 4u;                         // (i,0): left
    const int64_t g = (j - 1) >> 6, l = (j - 1) & 63, q = (i - 1) >> 3, s = (i - 1) & 7;
    return (v.D[(g * v.NC + q) * 64 + l] >> (28 - 4 * s)) & 0xfu;
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

// Per-column FNV-1a-64 of scores (int32 LE bytes) and codes (1 byte/cell).
__global__ void nw_colhash_kernel(TableView v, int32_t L1, int32_t L2, uint64_t* hcol, uint64_t* dcol) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i > L1) return;
    const uint64_t P = 0x100000001b3ULL;
    uint64_t h = 0xcbf29ce484222325ULL, e = 0xcbf29ce484222325ULL;
    for (int64_t j = 0; j <= L2; ++j) {
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
using KernelFn = void (*)(FillArgs);

template <int W>
KernelFn pick_flags(bool sh, bool sd, bool stt) {
    if (sh && sd) return stt ? nw_fill_kernel<W, true, true, true> : nw_fill_kernel<W, true, true, false>;
    if (sh) return stt ? nw_fill_kernel<W, true, false, true> : nw_fill_kernel<W, true, false, false>;
    if (sd) return stt ? nw_fill_kernel<W, false, true, true> : nw_fill_kernel<W, false, true, false>;
    return stt ? nw_fill_kernel<W, false, false, true> : nw_fill_kernel<W, false, false, false>;
}

KernelFn pick_kernel(int W, bool sh, bool sd, bool stt) {
    switch (W) {
        case 1: return pick_flags<1>(sh, sd, stt);
        case 2: return pick_flags<2>(sh, sd, stt);
        case 4: return pick_flags<4>(sh, sd, stt);
        case 6: return pick_flags<6>(sh, sd, stt);
        case 8: return pick_flags<8>(sh, sd, stt);
        case 12: return pick_flags<12>(sh, sd, stt);
        case 15: return pick_flags<15>(sh, sd, stt);
        default: return nullptr;
    }
}

// Compute waves per workgroup (+1 loader wave; 16 waves = 1024 threads max).
const int kWaveChoices[] = {1, 2, 4, 6, 8, 12, 15};

int choose_waves(int64_t NG, int ncu) {
    if (const char* e = getenv("NW_WAVES")) {
        const int w = atoi(e);
        for (int c : kWaveChoices)
            if (c == w) return w;
    }
    // One workgroup per CU when the stripes allow it, else the widest WG.
    for (int c : kWaveChoices)
        if ((NG + c - 1) / c <= ncu) return c;
    return 8;
}

TableView view_of(const nw_table* t) {
    TableView v{};
    v.tiles = t->H;
    v.spitch = t->spitch;
    v.D = (t->last_mask & NW_OUT_DIRS) ? t->D : nullptr;
    v.NC = (int32_t)t->NC;
    v.d = t->last_d;
    v.row_base = (int32_t)t->row_base;
    v.top = t->row_base > 0 ? t->xin : nullptr;
    return v;
}

}  // namespace

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
    // Overflow guard: |H| <= (L1+L2)*max(|m|,|k|,|d|); the shifted domain
    // adds up to 64*W*|d| (W <= 16) and one more candidate term.
    {
        const int64_t M = std::max({std::llabs(m), std::llabs(k), std::llabs(d)});
        const int64_t L2g = t->L2_total >= 0 ? t->L2_total : t->L2;
        const int64_t bound = (t->L1 + L2g) * M + 1024 * std::llabs(d) + 2 * M + 2;
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
    if (L1 > 0 && L2 > 0) {
        W = choose_waves(t->NG, t->ncu);
        KernelFn fn = pick_kernel(W, sh, sd, stt);
        if (!fn) return fail(NW_ERR_ARG, "nw_table_fill: unsupported wave count");
        FillArgs a{};
        a.s1 = t->s1;
        a.s2 = t->s2;
        a.L1 = (int32_t)L1;
        a.L2 = (int32_t)L2;
        a.m = m;
        a.k = k;
        a.d = d;
        a.NC = (int32_t)t->NC;
        a.NG = (int32_t)t->NG;
        a.NSW = (int32_t)((t->NG + W - 1) / W);
        a.H = t->H;
        a.spitch = t->spitch;
        a.D = t->D;
        a.lastcol = t->lastcol;
        a.gran = t->gran;
        a.gpitch = CH * t->NC + CH;
        a.ctl = t->ctl;
        // A panel waits on another GPU (or process) that may start seconds
        // later; a plain fill only on itself.
        a.spin_ticks = t->xin ? 30 * SPIN_TICKS : SPIN_TICKS;
        a.row_base = (int32_t)t->row_base;
        a.epoch = t->epoch;
        a.xin = t->xin;
        a.xout = t->xout;
        a.xflag = t->xflag;
        a.xblk = (int32_t)std::max<int64_t>(t->xblk, 1);
        if (t->xout && (L2 % 64) != 0) return fail(NW_ERR_ARG, "nw_table_fill: a feeding panel needs 64*k rows");
        if (getenv("NW_TRACE")) {
            const int64_t need = 4 * (int64_t)a.NSW;
            if (t->trace_n < need) {
                (void)hipFree(t->trace);
                t->trace = nullptr;
                t->trace_n = 0;
                NW_HIPCHK(hipMalloc(&t->trace, (size_t)need * 8));
                t->trace_n = need;
            }
            NW_HIPCHK(hipMemsetAsync(t->trace, 0, (size_t)need * 8, t->stream));
            a.trace = t->trace;
        }
        int occ = 1;
        NW_HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(fn), 64 * (W + 1), 0));
        occ = std::max(occ, 1);
        // A panel leaves room on every CU for the kernels of its neighbours
        // and of the transport (RCCL), which its hand-off waits on.
        const int per_cu = panel ? std::max(1, std::min(2, occ - 1)) : std::min(occ, 16);
        const int64_t grid = std::min<int64_t>(a.NSW, (int64_t)t->ncu * per_cu);
        a.nslot = (int32_t)std::min<int64_t>(grid + 1, (int64_t)(t->gran_bytes / 8 / a.gpitch));
        if (a.nslot < grid + 1) return fail(NW_ERR_ARG, "nw_table_fill: granule buffer too small");
        if (a.NSW > 1) NW_HIPCHK(hipMemsetAsync(t->gran, 0, (size_t)a.nslot * a.gpitch * 8, t->stream));
        NW_HIPCHK(hipEventRecord(t->ev[1], t->stream));
        void* kargs[] = {&a};
        NW_HIPCHK(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3((unsigned)grid), dim3(64 * (W + 1)), kargs,
                                  0, t->stream));
        NW_HIPCHK(hipGetLastError());
        NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    } else {
        NW_HIPCHK(hipEventRecord(t->ev[1], t->stream));
        NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    }
    t->launched = true;
    t->pend_mask = out_mask;
    t->pend_d = d;
    t->pend_W = W;
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
        const int32_t* src = sh ? t->H + (r >> 6) * t->spitch + (((q >> 2) * 64 + (r & 63)) << 2) + (q & 3)
                                : t->lastcol + L2;
        NW_HIPCHK(hipMemcpyAsync(&corner, src, 4, hipMemcpyDeviceToHost, t->stream));
    }
    NW_HIPCHK(hipStreamSynchronize(t->stream));
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
    t->last_mask = t->pend_mask;
    t->last_d = d;
    t->waves = t->pend_W;
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
    (void)hipFree(t->s1);
    (void)hipFree(t->s2);
    (void)hipFree(t->H);
    (void)hipFree(t->D);
    (void)hipFree(t->lastcol);
    (void)hipFree(t->gran);
    (void)hipFree(t->ctl);
    (void)hipFree(t->trace);
    for (auto& e : t->ev)
        if (e) (void)hipEventDestroy(e);
    if (t->stream) (void)hipStreamDestroy(t->stream);
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
        if ((rc = alloc((void**)&t->H, (size_t)std::max<int64_t>(NG, 1) * (size_t)std::max<int64_t>(NC, 1) * 2048)))
            return bail(rc);
    }
    if (out_mask & NW_OUT_DIRS) {
        if ((rc = alloc((void**)&t->D, (size_t)std::max<int64_t>(NG, 1) * std::max<int64_t>(NC, 1) * 256))) return bail(rc);
    }
    if ((rc = alloc((void**)&t->lastcol, (size_t)(64 * NG + 128) * 4))) return bail(rc);
    // Granule slots: one per concurrently running WG-stripe + 1.
    const int64_t gpitch = CH * NC + CH;
    const int64_t nslot = 16 * (int64_t)t->ncu + 1;
    t->gran_bytes = (size_t)(gpitch * nslot * 8);
    if ((rc = alloc((void**)&t->gran, t->gran_bytes))) return bail(rc);
    if ((rc = alloc((void**)&t->ctl, CTL_WORDS * 4))) return bail(rc);
    *out = t;
    return NW_OK;
}

int nw_table_set_sequences(nw_table* t, const char* s1, int64_t L1, const char* s2, int64_t L2) {
    if (!t || L1 < 0 || L2 < 0 || L1 > t->max_L1 || L2 > t->max_L2 || (L1 && !s1) || (L2 && !s2))
        return fail(NW_ERR_ARG, "nw_table_set_sequences: bad arguments");
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
    if (L1) HIPCHK(hipMemcpyAsync(t->s1, s1, (size_t)L1, hipMemcpyHostToDevice, t->stream));
    if (L2) HIPCHK(hipMemcpyAsync(t->s2, s2, (size_t)L2, hipMemcpyHostToDevice, t->stream));
    HIPCHK(hipStreamSynchronize(t->stream));
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
int nw_table_waves(const nw_table* t) { return t ? t->waves : 0; }

static int copy_scores_impl(nw_table* t, int64_t i0, int64_t i1, int32_t* dst) {
    const int64_t N = t->L2 + 1;
    // Gather the tiles into dense columns through a bounded staging buffer.
    const int64_t cols_per = std::max<int64_t>(1, ((int64_t)256 << 20) / (4 * N));
    int32_t* stage = nullptr;
    HIPCHK(hipMalloc(&stage, (size_t)(std::min(cols_per, i1 - i0) * N * 4)));
    hipError_t e = hipSuccess;
    for (int64_t c0 = i0; c0 < i1 && e == hipSuccess; c0 += cols_per) {
        const int64_t c1 = std::min(i1, c0 + cols_per);
        nw_gather_scores_kernel<<<1024, 256, 0, t->stream>>>(view_of(t), (int32_t)t->L2, c0, c1, stage);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(dst + (c0 - i0) * N, stage, (size_t)((c1 - c0) * N * 4), hipMemcpyDeviceToHost, t->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    }
    (void)hipFree(stage);
    if (e != hipSuccess) return fail(NW_ERR_HIP, std::string("nw_table_copy_scores: ") + hipGetErrorString(e));
    return NW_OK;
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
        uint64_t g = 0;
        HIPCHK(hipMemcpyAsync(&g, t->xin + (t->L1 - 1), 8, hipMemcpyDeviceToHost, t->stream));
        HIPCHK(hipStreamSynchronize(t->stream));
        dst[0] = (int32_t)(uint32_t)g + t->last_d;
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
    const size_t n = (size_t)((i1 - i0) * (t->L2 + 1));
    uint8_t* buf = nullptr;
    HIPCHK(hipMalloc(&buf, n));
    nw_codes_kernel<<<1024, 256, 0, t->stream>>>(view_of(t), (int32_t)t->L2, i0, i1, buf);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(dst, buf, n, hipMemcpyDeviceToHost, t->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(NW_ERR_HIP, std::string("nw_table_copy_codes: ") + hipGetErrorString(e));
    return NW_OK;
}

int nw_table_hash(nw_table* t, uint64_t* hH, uint64_t* hD) {
    if (!t) return fail(NW_ERR_ARG, "nw_table_hash: NULL table");
    if (!t->filled || !(t->last_mask & NW_OUT_SCORES)) return fail(NW_ERR_STATE, "nw_table_hash: no score table");
    HIPCHK(hipSetDevice(t->device));
    const int64_t ncol = t->L1 + 1;
    uint64_t* dh = nullptr;
    HIPCHK(hipMalloc(&dh, (size_t)ncol * 16));
    const bool have_d = (t->last_mask & NW_OUT_DIRS) != 0;
    TableView v = view_of(t);
    if (!have_d) v.D = nullptr;
    nw_colhash_kernel<<<(unsigned)((ncol + 255) / 256), 256, 0, t->stream>>>(v, (int32_t)t->L1, (int32_t)t->L2, dh,
                                                                              dh + ncol);
    std::vector<uint64_t> hv((size_t)ncol * 2);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(hv.data(), dh, (size_t)ncol * 16, hipMemcpyDeviceToHost, t->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    (void)hipFree(dh);
    if (e != hipSuccess) return fail(NW_ERR_HIP, std::string("nw_table_hash: ") + hipGetErrorString(e));
    auto fold = [](const uint64_t* v, int64_t n) {
        uint64_t h = 0xcbf29ce484222325ULL;
        for (int64_t i = 0; i < n; ++i)
            for (int b = 0; b < 8; ++b) h = (h ^ ((v[i] >> (8 * b)) & 0xff)) * 0x100000001b3ULL;
        return h;
    };
    if (hH) *hH = fold(hv.data(), ncol);
    if (hD) *hD = have_d ? fold(hv.data() + ncol, ncol) : 0;
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
