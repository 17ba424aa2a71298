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

#include "nw_fill.h"

namespace {

constexpr int CH = 8;                 // columns per chunk (= codes per dirs word)
constexpr int64_t SPIN_TICKS = 200000000;  // 2 s of s_memrealtime (100 MHz)

enum CtlWord { CTL_NEXT = 0, CTL_ABORT = 1, CTL_GAV = 2, CTL_BC = 3, CTL_ERR = 4, CTL_WORDS = 16 };

struct FillArgs {
    const uint8_t* s1;      // device, zero-padded to >= 8*NC + 8 bytes (s1[i-1] = column i)
    const uint8_t* s2;      // device, zero-padded to >= 64*NG + 64 bytes
    int32_t L1, L2;
    int32_t m, k, d;
    int32_t NC;             // chunks = ceil(L1 / 8)
    int32_t NG;             // wave stripes = ceil(L2 / 64)
    int32_t NSW;            // workgroup stripes = ceil(NG / W)
    int32_t* H;             // score tiles: (i, j>=1) at H[(g*(L1+1) + i)*64 + l], j-1 = 64g+l
    int64_t spitch;         // (L1+1)*64: elements per stripe
    uint32_t* D;            // codes: word ((g*NC + q)*64 + lane)
    int32_t* lastcol;       // score-only: H[L1][j] at lastcol[63 + j]
    uint64_t* gran;         // boundary granules, slot s at gran + s*gpitch
    int64_t gpitch;
    int32_t nslot;
    uint32_t* ctl;          // CtlWord
};

// ---------------------------------------------------------------- DPP helpers
// wave_shr:1 -- lane l receives lane l-1; lane 0 keeps `old`.
__device__ __forceinline__ int wave_shr1(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false);
}

// Inclusive prefix max over the 64 lanes (lane l gets max of lanes 0..l).
// Out-of-row sources leave the lane unchanged (bound_ctrl off), which is the
// identity for max; the compiler fuses each step into one v_max_i32_dpp.
__device__ __forceinline__ int wave_prefix_max(int y) {
    constexpr int NEG = (int)0x80000000;
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x111, 0xf, 0xf, false));  // row_shr:1
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x112, 0xf, 0xf, false));  // row_shr:2
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x114, 0xf, 0xf, false));  // row_shr:4
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x118, 0xf, 0xf, false));  // row_shr:8
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x142, 0xa, 0xf, false));  // row_bcast:15
    y = max(y, __builtin_amdgcn_update_dpp(NEG, y, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return y;
}

typedef const __attribute__((address_space(4))) uint64_t* cptr64;

__device__ __forceinline__ int iabs(int v) { return v < 0 ? -v : v; }

// Count nibbles of a codes word that have >= 2 of their 3 direction bits.
__device__ __forceinline__ uint32_t branch_nibbles(uint32_t x) {
    uint32_t y = (x & (x >> 1)) | (x & (x >> 2)) | ((x >> 1) & (x >> 2));
    return __builtin_popcount(y & 0x11111111u);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) and syncs.  Unlike __syncthreads() it carries no fence, so it
// never waits for the wave's in-flight global stores (vmcnt).
__device__ __forceinline__ void wg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
template <bool SH, bool SD, bool ST, bool LAST>
__device__ __forceinline__ void chunk_body(const FillArgs& a, WaveState& st, const int* T,
                                           int c, int nstep, int lane, int64_t tile_off, int j0,
                                           int d, int vcm, int vck, int* bot_wr, uint32_t* dword_out) {
    // s1[8c .. 8c+7]: one uniform 8-byte load through the constant address
    // space -> s_load_dwordx2 (lgkmcnt), never a vector load that would make
    // the wave wait for its own in-flight score stores.
    const uint64_t ch8 = *(cptr64)(a.s1 + 8 * (int64_t)c);
    uint32_t acc = 0;
    // Buffer descriptor on this chunk's 8 column segments (2 KB contiguous in
    // the stripe-major tile layout): per-step addresses are lane*4 (VGPR) +
    // s*256 (SGPR) -- no VALU address math.
    int32_t* cb = a.H + tile_off + (int64_t)(8 * c + 1) * 64;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cb, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int s = 0; s < CH; ++s) {
        if (LAST && s >= nstep) break;
        const uint32_t ch = (uint32_t)(ch8 >> (8 * s)) & 0xffu;
        const int sub = (ch == st.c2) ? vcm : vck;        // m+d or d-k
        const int sh = wave_shr1(st.Tprev, st.G);         // G[l-1], lane 0: row above
        const int dg = sh + sub;                          // diag candidate (shifted)
        const int lf = st.G - d;                          // left candidate (shifted)
        const int top = T[s];                             // up candidate of lane 0
        const int Y = max(max(lf, dg), top);
        const int G = wave_prefix_max(Y);                 // resolves all "up" terms
        const int Hv = G - st.laneoff;
        if (SH) __builtin_amdgcn_raw_buffer_store_b32(Hv, rs, lane * 4, s * 256, 0);
        if (SD || ST) {                                   // codes also feed branch_count
            const int up = wave_shr1(top, G);             // up candidate (shifted)
            acc = (acc << 4) | (uint32_t)(G == dg) | ((uint32_t)(G == up) << 1) |
                  ((uint32_t)(G == lf) << 2);
        }
        if (ST) st.gav = max(st.gav, iabs(Hv));
        bot_wr[s] = G;   // lane 63 -> bottom-row slot, lanes 0..62 -> scratch
        st.G = G;
        st.Tprev = top;
        if (LAST && !SH && s == nstep - 1) {
            // score-only: keep the last column H[L1][*].
            a.lastcol[j0 + lane] = Hv;
        }
    }
    if (LAST && nstep < CH) acc <<= 4 * (CH - nstep);
    *dword_out = acc;
}

// Workgroup = W compute waves (64-row stripes, stacked) + 1 loader wave.
// The loader feeds the top row of the WG-stripe for chunk t+1 into LDS while
// the compute waves run superstep t; it issues no stores, so its waits on
// the hand-off loads are exact, and the compute waves never wait on vmcnt.
template <int W, bool SH, bool SD, bool ST>
__global__ __launch_bounds__(64 * (W + 1)) void nw_fill_kernel(FillArgs a) {
    // xfer[w][par][8]: top row of wave w (w = 0: from the loader, else the
    // bottom row of wave w-1) for chunk parity par.  Then 72 scratch dwords.
    constexpr int XFER = (W + 1) * 2 * CH;
    __shared__ __attribute__((aligned(16))) int xfer[XFER + 64 + CH];
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
        __syncthreads();
        const int sidx = uni(sh_sidx);
        if (sidx >= a.NSW || sh_abort) break;

        const int g = sidx * W + w;                // wave stripe (compute waves)
        const bool real = !loader && g < a.NG;
        const int j0 = 1 + 64 * g;                 // first row of the wave stripe
        const int jrow = j0 + lane;
        const int64_t tile_off = (int64_t)g * a.spitch;
        WaveState st;
        st.c2 = real ? a.s2[jrow - 1] : 0u;
        st.laneoff = (64 * w + lane) * d;
        // column 0: H[0][j] = -j*d  ->  G = -(1 + 64*sidx*W)*d for every lane.
        st.G = -(1 + 64 * sidx * W) * d;
        st.Tprev = st.G;
        st.gav = 0;
        st.bc = 0;

        // ---- loader state: top row of this WG-stripe, one chunk ahead ----
        const uint64_t* gin = a.gran + (int64_t)(sidx % a.nslot) * a.gpitch;
        uint64_t* gout = a.gran + (int64_t)((sidx + 1) % a.nslot) * a.gpitch;
        uint64_t pf = 0;
        // Fill xfer[0][par(c)] with chunk c's top values (G domain of row "-1").
        auto loader_fill = [&](int c) {
            int* dst = &xfer[(c & 1) * CH];
            const int n = (c == NC - 1) ? nlast : CH;
            if (sidx == 0) {
                // row 0: H[i][0] - d = -(i+1)*d   (computation.c:102-110)
                if (lane < CH) dst[lane] = -(CH * c + 2 + lane) * d;
                return;
            }
            const uint32_t want = (uint32_t)sidx;
            bool ok = lane >= n || (uint32_t)(pf >> 32) == want;
            if (!__all(ok)) {
                const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
                for (;;) {
                    __builtin_amdgcn_s_sleep(1);
                    if (!ok)
                        pf = __hip_atomic_load(gin + CH * (int64_t)c + lane, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    ok = lane >= n || (uint32_t)(pf >> 32) == want;
                    if (__all(ok)) break;
                    const int64_t now = (int64_t)__builtin_amdgcn_s_memrealtime();
                    const uint32_t ab = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                    if (ab || now - t0 > SPIN_TICKS) {
                        if (lane == 0) {
                            __hip_atomic_store(&a.ctl[CTL_ABORT], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (!ab) atomicCAS(&a.ctl[CTL_ERR], 0u, (uint32_t)NW_ERR_TIMEOUT);
                            sh_abort = 1;
                        }
                        break;
                    }
                }
            }
            if (lane < CH) dst[lane] = (int)(uint32_t)pf;
            if (c + 1 < NC && lane < CH)          // prefetch the next chunk
                pf = __hip_atomic_load(gin + CH * (int64_t)(c + 1) + lane, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        };
        if (loader) {
            // ---------------- loader wave: no stores, exact waits ----------------
            if (sidx > 0 && lane < CH)
                pf = __hip_atomic_load(gin + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            loader_fill(0);
            wg_barrier();
            if (!sh_abort) {
                const int nsuper = NC + W - 1;
                for (int t = 0; t < nsuper; ++t) {
                    if (t + 1 < NC) loader_fill(t + 1);
                    wg_barrier();
                    if (sh_abort) break;
                }
            }
        } else {
            // ---------------- compute waves: one chunk per superstep ------------
            wg_barrier();
            if (!sh_abort) {
                const int nsuper = NC + W - 1;
                for (int t = 0; t < nsuper; ++t) {
                    const int c = t - w;
                    if (real && c >= 0 && c < NC) {
                        const int par = c & 1;
                        const int* top_lds = &xfer[(w * 2 + par) * CH];
                        // Bottom row goes to xfer[w+1][par]; lanes 0..62 hit scratch.
                        int* bot_wr = (lane == 63) ? &xfer[((w + 1) * 2 + par) * CH] : &xfer[XFER + lane];
                        const int nstep = (c == NC - 1) ? nlast : CH;
                        const int4 t03 = *reinterpret_cast<const int4*>(top_lds);
                        const int4 t47 = *reinterpret_cast<const int4*>(top_lds + 4);
                        const int T[CH] = {t03.x, t03.y, t03.z, t03.w, t47.x, t47.y, t47.z, t47.w};
                        uint32_t dw;
                        if (c == NC - 1)
                            chunk_body<SH, SD, ST, true>(a, st, T, c, nstep, lane, tile_off, j0, d, vcm, vck, bot_wr, &dw);
                        else
                            chunk_body<SH, SD, ST, false>(a, st, T, c, CH, lane, tile_off, j0, d, vcm, vck, bot_wr, &dw);
                        if (jrow > a.L2) dw = 0;
                        if (SD) a.D[((int64_t)g * NC + c) * 64 + lane] = dw;
                        if (ST) st.bc += branch_nibbles(dw);
                        // Last wave of a non-final WG-stripe publishes its bottom row.
                        if (w == W - 1 && sidx + 1 < a.NSW && lane < nstep) {
                            const int v = xfer[((w + 1) * 2 + par) * CH + lane] - 64 * W * d;  // row-above domain
                            const uint64_t gr = ((uint64_t)(uint32_t)(sidx + 1) << 32) | (uint32_t)v;
                            __hip_atomic_store(gout + CH * (int64_t)c + lane, gr, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                    wg_barrier();
                    if (sh_abort) break;
                }
            }
        }
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

// Boundary row/column seeding (computation.c:93-120): row 0, H[i][0] = -i*d,
// into row0[]; column 0, H[0][j] = -j*d, into slot i = 0 of every stripe.
// Directions of boundary cells are implicit (code_at).
__global__ void nw_seed_kernel(int32_t* row0, int32_t* tiles, int64_t spitch, int32_t L1, int32_t NG, int32_t d) {
    const int64_t n = (int64_t)L1 + 1 + 64 * (int64_t)NG;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        if (x <= L1) row0[x] = (int32_t)(-x * (int64_t)d);
        else {
            const int64_t r = x - L1 - 1;          // = j - 1
            tiles[(r >> 6) * spitch + (r & 63)] = (int32_t)(-(r + 1) * (int64_t)d);
        }
    }
}

__device__ __forceinline__ int32_t score_at(const int32_t* row0, const int32_t* tiles, int64_t spitch, int64_t i,
                                            int64_t j) {
    if (j == 0) return row0[i];
    const int64_t r = j - 1;
    return tiles[(r >> 6) * spitch + i * 64 + (r & 63)];
}

// Dense i-major copy of columns [i0, i1): out[(i-i0)*(L2+1) + j].
__global__ void nw_gather_scores_kernel(const int32_t* row0, const int32_t* tiles, int64_t spitch, int32_t L2,
                                        int64_t i0, int64_t i1, int32_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t n = (i1 - i0) * N;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = score_at(row0, tiles, spitch, i0 + x / N, x % N);
}

__device__ __forceinline__ uint32_t code_at(const uint32_t* D, int32_t NC, int64_t i, int64_t j) {
    if (i == 0) return j == 0 ? 0u : 2u;          // (0,0): none; (0,j): up
    if (j == 0) return 4u;                         // (i,0): left
    const int64_t g = (j - 1) >> 6, l = (j - 1) & 63, q = (i - 1) >> 3, s = (i - 1) & 7;
    return (D[(g * NC + q) * 64 + l] >> (28 - 4 * s)) & 0xfu;
}

// Dense nibble packing for nw_fill(): byte b = code(2b) | code(2b+1) << 4.
__global__ void nw_pack_nibbles_kernel(const uint32_t* D, int32_t NC, int32_t L1, int32_t L2, uint8_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t ncell = ((int64_t)L1 + 1) * N;
    const int64_t nbyte = (ncell + 1) / 2;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbyte;
         b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c0 = 2 * b, c1 = 2 * b + 1;
        uint32_t v = code_at(D, NC, c0 / N, c0 % N);
        if (c1 < ncell) v |= code_at(D, NC, c1 / N, c1 % N) << 4;
        out[b] = (uint8_t)v;
    }
}

// One code byte per cell for columns [i0, i1).
__global__ void nw_codes_kernel(const uint32_t* D, int32_t NC, int32_t L2, int64_t i0, int64_t i1, uint8_t* out) {
    const int64_t N = (int64_t)L2 + 1;
    const int64_t n = (i1 - i0) * N;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = (uint8_t)code_at(D, NC, i0 + x / N, x % N);
}

// Per-column FNV-1a-64 of scores (int32 LE bytes) and codes (1 byte/cell).
__global__ void nw_colhash_kernel(const int32_t* row0, const int32_t* tiles, int64_t spitch, const uint32_t* D,
                                  int32_t NC, int32_t L1,
                                  int32_t L2, uint64_t* hcol, uint64_t* dcol) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i > L1) return;
    const uint64_t P = 0x100000001b3ULL;
    uint64_t h = 0xcbf29ce484222325ULL, e = 0xcbf29ce484222325ULL;
    for (int64_t j = 0; j <= L2; ++j) {
        const uint32_t v = (uint32_t)score_at(row0, tiles, spitch, i, j);
        h = (h ^ (v & 0xff)) * P;
        h = (h ^ ((v >> 8) & 0xff)) * P;
        h = (h ^ ((v >> 16) & 0xff)) * P;
        h = (h ^ (v >> 24)) * P;
        if (D) e = (e ^ code_at(D, NC, i, j)) * P;
    }
    hcol[i] = h;
    dcol[i] = e;
}

// --------------------------------------------------------------- host side
thread_local std::string g_last_error;

int fail(int rc, const std::string& msg) {
    g_last_error = msg;
    return rc;
}

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(e_ == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP,                \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                 \
    } while (0)

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


}  // namespace

struct nw_table {
    int device = 0;
    int ncu = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t cap_mask = 0;
    int64_t max_L1 = 0, max_L2 = 0;
    // geometry for the current sequences
    int64_t L1 = -1, L2 = -1;
    int64_t NC = 0, NG = 0, spitch = 0;
    // device buffers
    uint8_t* s1 = nullptr;
    uint8_t* s2 = nullptr;
    int32_t* H = nullptr;       // score tiles
    int32_t* row0 = nullptr;    // H[i][0]
    uint32_t* D = nullptr;
    int32_t* lastcol = nullptr;
    uint64_t* gran = nullptr;
    size_t gran_bytes = 0;
    uint32_t* ctl = nullptr;
    // results of the last fill
    bool filled = false;
    uint32_t last_mask = 0;
    int32_t last_d = 0;
    nw_stats stats{};
    float kernel_ms = 0.f, call_ms = 0.f;
    int waves = 0;
};

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
        default: return "unknown error";
    }
}

const char* nw_last_error(void) { return g_last_error.c_str(); }

void nw_table_destroy(nw_table* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    (void)hipFree(t->s1);
    (void)hipFree(t->s2);
    (void)hipFree(t->H);
    (void)hipFree(t->row0);
    (void)hipFree(t->D);
    (void)hipFree(t->lastcol);
    (void)hipFree(t->gran);
    (void)hipFree(t->ctl);
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
        if ((rc = alloc((void**)&t->H, (size_t)std::max<int64_t>(NG, 1) * (size_t)(max_L1 + 1) * 256))) return bail(rc);
        if ((rc = alloc((void**)&t->row0, (size_t)(max_L1 + 1) * 4))) return bail(rc);
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
    t->spitch = 64 * (L1 + 1);
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
    if (!t) return fail(NW_ERR_ARG, "nw_table_fill: NULL table");
    if (t->L1 < 0) return fail(NW_ERR_STATE, "nw_table_fill: no sequences set");
    if ((out_mask & ~t->cap_mask & (NW_OUT_SCORES | NW_OUT_DIRS)) != 0)
        return fail(NW_ERR_ARG, "nw_table_fill: output not allocated at creation");
    // Overflow guard: |H| <= (L1+L2)*max(|m|,|k|,|d|); the shifted domain
    // adds up to 64*W*|d| (W <= 16) and one more candidate term.
    {
        const int64_t M = std::max({std::llabs(m), std::llabs(k), std::llabs(d)});
        const int64_t bound = (t->L1 + t->L2) * M + 1024 * std::llabs(d) + 2 * M + 2;
        if (bound >= (int64_t)INT32_MAX)
            return fail(NW_ERR_RANGE, "nw_table_fill: |scores| could reach " + std::to_string(bound));
    }
    HIPCHK(hipSetDevice(t->device));
    const bool sh = out_mask & NW_OUT_SCORES, sd = out_mask & NW_OUT_DIRS, stt = out_mask & NW_OUT_STATS;
    const int64_t L1 = t->L1, L2 = t->L2;
    HIPCHK(hipEventRecord(t->ev[0], t->stream));
    HIPCHK(hipMemsetAsync(t->ctl, 0, CTL_WORDS * 4, t->stream));
    if (sh) nw_seed_kernel<<<256, 256, 0, t->stream>>>(t->row0, t->H, t->spitch, (int32_t)L1, (int32_t)t->NG, d);
    HIPCHK(hipGetLastError());
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
        int occ = 1;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(fn), 64 * (W + 1), 0));
        occ = std::max(occ, 1);
        const int64_t grid = std::min<int64_t>(a.NSW, (int64_t)t->ncu * std::min(occ, 16));
        a.nslot = (int32_t)std::min<int64_t>(grid + 1, (int64_t)(t->gran_bytes / 8 / a.gpitch));
        if (a.nslot < grid + 1) return fail(NW_ERR_ARG, "nw_table_fill: granule buffer too small");
        if (a.NSW > 1)
            HIPCHK(hipMemsetAsync(t->gran, 0, (size_t)a.nslot * a.gpitch * 8, t->stream));
        HIPCHK(hipEventRecord(t->ev[1], t->stream));
        void* kargs[] = {&a};
        HIPCHK(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3((unsigned)grid), dim3(64 * (W + 1)), kargs, 0,
                               t->stream));
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(t->ev[2], t->stream));
    } else {
        HIPCHK(hipEventRecord(t->ev[1], t->stream));
        HIPCHK(hipEventRecord(t->ev[2], t->stream));
    }
    HIPCHK(hipEventRecord(t->ev[3], t->stream));
    uint32_t ctl[CTL_WORDS];
    HIPCHK(hipMemcpyAsync(ctl, t->ctl, sizeof ctl, hipMemcpyDeviceToHost, t->stream));
    int32_t corner = 0;
    if (L1 > 0 && L2 > 0) {
        const int64_t r = L2 - 1;
        const int32_t* src = sh ? t->H + (r >> 6) * t->spitch + L1 * 64 + (r & 63) : t->lastcol + L2;
        HIPCHK(hipMemcpyAsync(&corner, src, 4, hipMemcpyDeviceToHost, t->stream));
    }
    HIPCHK(hipStreamSynchronize(t->stream));
    if (ctl[CTL_ERR]) {
        t->filled = false;
        return fail((int)ctl[CTL_ERR], "nw_table_fill: in-kernel watchdog fired (hand-off timeout)");
    }
    HIPCHK(hipEventElapsedTime(&t->kernel_ms, t->ev[1], t->ev[2]));
    HIPCHK(hipEventElapsedTime(&t->call_ms, t->ev[0], t->ev[3]));
    if (L1 == 0 || L2 == 0) corner = (int32_t)(-(L1 + L2) * (int64_t)d);
    t->stats.corner = corner;
    t->stats.greatest_abs_interior = stt ? (int32_t)ctl[CTL_GAV] : 0;
    t->stats.branch_count = stt ? ctl[CTL_BC] : 0u;
    t->filled = true;
    t->last_mask = out_mask;
    t->last_d = d;
    t->waves = W;
    return NW_OK;
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
        nw_gather_scores_kernel<<<1024, 256, 0, t->stream>>>(t->row0, t->H, t->spitch, (int32_t)t->L2, c0, c1, stage);
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
    if (t->L2 == 0 || t->L1 == 0) {
        for (int64_t j = 0; j <= t->L2; ++j) dst[j] = (int32_t)(-(t->L1 + j) * (int64_t)t->last_d);
        return NW_OK;
    }
    HIPCHK(hipMemcpyAsync(dst + 1, t->lastcol + 1, (size_t)t->L2 * 4, hipMemcpyDeviceToHost, t->stream));
    HIPCHK(hipStreamSynchronize(t->stream));
    dst[0] = (int32_t)(-t->L1 * (int64_t)t->last_d);
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
    nw_codes_kernel<<<1024, 256, 0, t->stream>>>(t->D, (int32_t)t->NC, (int32_t)t->L2, i0, i1, buf);
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
    nw_colhash_kernel<<<(unsigned)((ncol + 255) / 256), 256, 0, t->stream>>>(
        t->row0, t->H, t->spitch, have_d ? t->D : nullptr, (int32_t)t->NC, (int32_t)t->L1, (int32_t)t->L2, dh, dh + ncol);
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
            hipLaunchKernelGGL(nw_pack_nibbles_kernel, dim3(1024), dim3(256), 0, t->stream, t->D, (int32_t)t->NC,
                               (int32_t)L1, (int32_t)L2, buf);
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
