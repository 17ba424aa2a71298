// nw_walk.hip -- walk services over a device-resident filled table.
//
// The reference walks its table on the host after the fill
// (construct_alignments, needleman-wunsch.c:356-388, iterating in
// construct_alignments_for_subtable, :209-331): a depth-first enumeration of
// every optimal alignment that prints each one and counts them
// (inc_solution_count, :250-255; print_summary, computation.c:271-281).  The
// enumeration is exponential, so at 100k x 100k the reference cannot even
// report `-s`.  Two of its results do not need the enumeration and run here on
// the device, straight from the direction codes the fill left in HBM:
//
//   * nw_table_count_alignments -- the number of optimal alignments is the
//     number of code paths from the corner to (0,0): a path-count DP
//     P(i,j) = [diag] P(i-1,j-1) + [left] P(i-1,j) + [up] P(i,j-1), P(0,0) = 1,
//     in uint32 (the reference's counter is an `unsigned` that wraps the
//     same way, walk-table.c:108-147).  Same stripe orientation as the fill:
//     a wave owns 64 rows and sweeps the columns; the up term is an affine
//     scan over the lanes (six DPP levels, like the fill's prefix max); the
//     stripe below takes the bottom row through tagged granules.
//   * nw_table_first_path -- the first alignment the reference prints is the
//     greedy walk diag > left > up from the corner (:296-322).  One wave
//     stages 64 rows x 64 columns of codes in LDS and walks them, O(L1 + L2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "nw_internal.h"
#include "nw_kern.h"

struct nw_walk_state {
    uint64_t* rows = nullptr;     // count hand-off granules {tag, P}, (NG-1) x L1
    size_t rows_bytes = 0;
    uint32_t epoch = 0;           // tag of the count in flight
    uint32_t* ctl = nullptr;      // [0] dequeue, [1] abort, [2] result, [3] path length lo, [4] hi / error
    uint8_t* moves = nullptr;     // first path, back to front
    size_t moves_bytes = 0;
    uint64_t* cnt = nullptr;      // enumeration: saturating path counts, i-major (L1+1)*(L2+1)
    size_t cnt_bytes = 0;
    uint64_t cnt_serial = 0;      // fill_serial the counts belong to (0: none)
    uint8_t* emoves = nullptr;    // enumeration batch: moves and lengths
    int32_t* elens = nullptr;
    size_t ebytes = 0, elens_n = 0;
    float count_ms = 0.f, path_ms = 0.f;
};

namespace {

constexpr int CBLK = 16;                       // columns per count hand-off block
constexpr int64_t WALK_SPIN = 1000000000;      // 10 s of s_memrealtime (100 MHz)
constexpr uint32_t POISON = 0x80000000u;

struct CountArgs {
    const uint32_t* D;    // codes, include/nw_fill.h layout
    int64_t NC;           // 8-step chunks per stripe of the table's layout
    int32_t skew;         // skewed layout: lane l's word index runs ahead by l steps
    int32_t pair;         // pair layout: rows permuted (nwi::pair_row)
    int32_t L1, L2, NG;
    uint64_t* rows;       // granule (g, i) at g*L1 + i-1: P(i, 64(g+1)) for stripe g < NG-1
    uint32_t* ctl;
    uint32_t epoch;
};

template <int CTRL, int ROWMASK>
__device__ __forceinline__ void scan_level(uint32_t& A, uint32_t& u) {
    const uint32_t Ap = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)A, CTRL, ROWMASK, 0xf, false);
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)u, CTRL, ROWMASK, 0xf, false);
    A += Ap & u;
    u &= up;
}

// One wave per 64-row stripe, stripes taken in order from a ticket counter,
// so a wave only ever waits for a stripe already held by a running wave.
__global__ __launch_bounds__(64) void nw_count_kernel(CountArgs a) {
    const int lane = threadIdx.x;
    const uint32_t tag = a.epoch;
    for (;;) {
        int g = 0;
        if (lane == 0) g = (int)atomicAdd(&a.ctl[0], 1u);
        g = __builtin_amdgcn_readfirstlane(g);
        if (g >= a.NG) return;
        if (__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;

        const int64_t rr = a.pair ? nwi::pair_row(64 * (int64_t)g + lane) : 64 * (int64_t)g + lane;
        const uint32_t* Dg = a.D + ((rr >> 6) * (a.NC + 1) + 1) * 64 + (rr & 63);
        const uint64_t* top = g > 0 ? a.rows + (int64_t)(g - 1) * a.L1 : nullptr;
        uint64_t* bot = g < a.NG - 1 ? a.rows + (int64_t)g * a.L1 : nullptr;
        uint32_t P = 1;         // column 0: (0,j) has only the up code, P = 1
        uint32_t Tprev = 1;     // P(0, 64g)
        // this lane's step of column i is t = i - 1 (+ lane in the skewed layout)
        const int toff = (int)nwk::skew_off(a.skew, lane);
        uint32_t w = 0, wn = a.NC > 0 ? Dg[(int64_t)(toff >> 3) * 64] : 0u;
        bool dead = false;
        for (int i0 = 1; i0 <= a.L1 && !dead; i0 += CBLK) {
            const int cnt = min(CBLK, a.L1 - i0 + 1);
            uint32_t Tv = 1;    // stripe 0: P(i, 0) = 1 (left codes)
            if (top) {
                uint64_t gv = 0;
                const int64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    if (lane < cnt)
                        gv = __hip_atomic_load(top + i0 - 1 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t gt = (uint32_t)(gv >> 32);
                    const bool ok = lane >= cnt || gt == tag;
                    const bool bad = lane < cnt && gt == (tag | POISON);
                    if (__builtin_amdgcn_ballot_w64(bad)) {
                        dead = true;
                        break;
                    }
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > WALK_SPIN) {
                        if (lane == 0) __hip_atomic_store(&a.ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        dead = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (dead) break;
                Tv = (uint32_t)gv;
            }
            uint32_t outv = 0;
            for (int c = 0; c < cnt; ++c) {
                const int i = i0 + c;
                const int t = i - 1 + toff;
                const int s = t & 7;
                if (s == 0 || i == 1) {
                    w = wn;
                    const int64_t qn = (t >> 3) + 1;
                    if (qn < a.NC) wn = Dg[qn * 64];
                }
                const uint32_t code = (w >> (21 - 3 * s)) & 7u;
                const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)Tv, c);
                const uint32_t diag = (uint32_t)__builtin_amdgcn_update_dpp((int)Tprev, (int)P, 0x138, 0xf, 0xf, false);
                uint32_t A = ((code & 1u) ? diag : 0u) + ((code & 4u) ? P : 0u);
                uint32_t u = (code & 2u) ? ~0u : 0u;
                scan_level<0x111, 0xf>(A, u);
                scan_level<0x112, 0xf>(A, u);
                scan_level<0x114, 0xf>(A, u);
                scan_level<0x118, 0xf>(A, u);
                scan_level<0x142, 0xa>(A, u);
                scan_level<0x143, 0xc>(A, u);
                P = A + (u & T);
                Tprev = T;
                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
                if (lane == c) outv = b;
            }
            if (bot && lane < cnt)
                __hip_atomic_store(bot + i0 - 1 + lane, ((uint64_t)tag << 32) | outv, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (dead) {
            // Tell the stripe below (and everything after it) to stop.
            if (bot)
                for (int x = lane; x < a.L1; x += 64)
                    __hip_atomic_store(bot + x, (uint64_t)(tag | POISON) << 32, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (g == (a.L2 - 1) / 64 && lane == (a.L2 - 1) % 64) a.ctl[2] = P;
    }
}

// Greedy walk diag > left > up from (i0, j0) (the corner for a whole
// table).  Moves are written back to front; ctl[3] = count, ctl[4] = 1 if a
// cell had no code, ctl[5] = the column where the walk left through row 0.
// top = 1: row 0 is the seeded first row, so the walk runs on along row 0 /
// column 0 to (0, 0); top = 0 (a band of rows below another): it stops on
// row 0, which is the band above's last row.
__global__ __launch_bounds__(64) void nw_first_path_kernel(const uint32_t* D, int64_t NC, int32_t skew, int32_t pair,
                                                           int32_t i0, int32_t j0, int32_t top, uint8_t* moves,
                                                           uint32_t* ctl) {
    __shared__ uint32_t blk[8][64];
    const int lane = threadIdx.x;
    int i = i0, j = j0;
    uint32_t n = 0;
    int gb = -1;
    int64_t qb = -1;
    while (i > 0 && j > 0) {
        const int g = (j - 1) >> 6;
        const int64_t t = (i - 1) + nwk::skew_off(skew, (j - 1) & 63);   // step of (i, j) in its stripe
        const int64_t q = t >> 3, q0 = q & ~(int64_t)7;
        if (g != gb || q0 != qb) {
            __syncthreads();
            const int64_t rr = pair ? nwi::pair_row(64 * (int64_t)g + lane) : 64 * (int64_t)g + lane;
#pragma unroll
            for (int x = 0; x < 8; ++x)
                blk[x][lane] = q0 + x < NC ? D[((rr >> 6) * (NC + 1) + q0 + x + 1) * 64 + (rr & 63)] : 0u;
            __syncthreads();
            gb = g;
            qb = q0;
        }
        const uint32_t code = (blk[q - q0][(j - 1) & 63] >> (21 - 3 * (int)(t & 7))) & 7u;
        uint8_t mv;
        if (code & 1u) {
            mv = 1;
            --i;
            --j;
        } else if (code & 4u) {
            mv = 4;
            --i;
        } else if (code & 2u) {
            mv = 2;
            --j;
        } else {
            if (lane == 0) ctl[4] = 1;
            return;
        }
        if (lane == 0) moves[n] = mv;
        ++n;
    }
    for (; j > 0; --j, ++n)      // column 0: up codes
        if (lane == 0) moves[n] = 2;
    if (top)
        for (; i > 0; --i, ++n)  // row 0: left codes
            if (lane == 0) moves[n] = 4;
    if (lane == 0) {
        ctl[3] = n;
        ctl[5] = (uint32_t)i;
    }
}

// ---------------------------------------------------------------- enumeration
// Every optimal alignment, in the reference's print order, each one computed
// on its own (the reference's "parallel traceback" future work, README:195-200).
// The reference prints alignments in the order of its depth-first walk, which
// tries diag, then left, then up at every cell (needleman-wunsch.c:296-322).
// With C(i,j) = the number of code paths from (i,j) to (0,0), alignment k
// (0-based, in that order) is found by walking from the corner: take diag if
// k < C(diag cell), else k -= C(diag cell) and try left, then up.  So a
// thread per alignment writes its moves independently; C is a saturating
// uint64 (cap 2^62: every k below the cap is unranked exactly).
constexpr uint64_t CNT_CAP = 1ull << 62;
constexpr int CT = 64;      // count tile: CT columns x 64 rows

__device__ __forceinline__ uint64_t sat_add(uint64_t a, uint64_t b) {
    const uint64_t s = a + b;              // a, b <= CNT_CAP: no wrap
    return s < CNT_CAP ? s : CNT_CAP;
}

// Row 0 and column 0: one path each (left / up codes, computation.c:102-120).
__global__ void nw_count_border_kernel(uint64_t* cnt, int64_t L1, int64_t L2) {
    const int64_t N = L2 + 1;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x <= L1 + L2;
         x += (int64_t)gridDim.x * blockDim.x) {
        if (x <= L2) cnt[x] = 1;                       // (0, j)
        else cnt[(x - L2) * N] = 1;                    // (i, 0)
    }
}

// One 64-row x CT-column tile per workgroup (a wave, lane = row), tiles of one
// tile anti-diagonal per launch.  The tile is swept in anti-diagonal order
// through LDS: cell (i, j) needs (i-1, j), (i, j-1), (i-1, j-1), all written
// by an earlier step or read into the halo (row j0-1, column i0-1).
__global__ __launch_bounds__(64) void nw_count_tiles_kernel(nwk::TableView v, uint64_t* cnt, int64_t L1, int64_t L2,
                                                            int diag, int ntj) {
    __shared__ uint64_t T[CT + 1][64 + 1];          // [column - i0 + 1][row - j0 + 1]
    const int lane = threadIdx.x;
    const int bj = max(0, diag - (int)((L1 + CT - 1) / CT - 1)) + (int)blockIdx.x;
    const int bi = diag - bj;
    if (bj >= ntj || bi < 0) return;
    const int64_t N = L2 + 1;
    const int64_t i0 = 1 + (int64_t)CT * bi, j0 = 1 + 64 * (int64_t)bj;
    const int64_t j = j0 + lane;
    // halo: row j0-1 over columns i0-1 .. i0+CT-1, column i0-1 over the tile's rows
    for (int c = lane; c <= CT; c += 64) {
        const int64_t i = i0 - 1 + c;
        T[c][0] = i <= L1 ? cnt[i * N + (j0 - 1)] : 0;
    }
    T[0][lane + 1] = j <= L2 ? cnt[(i0 - 1) * N + j] : 0;
    __syncthreads();
    for (int t = 0; t < CT + 63; ++t) {
        const int c = t - lane;                     // this lane's column in the tile
        const int64_t i = i0 + c;
        if (c >= 0 && c < CT && i <= L1 && j <= L2) {
            const uint32_t code = nwk::code_at(v, i, j);
            uint64_t x = 0;
            if (code & 1u) x = T[c][lane];                       // diag (i-1, j-1)
            if (code & 4u) x = sat_add(x, T[c][lane + 1]);       // left (i-1, j)
            if (code & 2u) x = sat_add(x, T[c + 1][lane]);       // up   (i, j-1)
            T[c + 1][lane + 1] = x;
        }
        __syncthreads();
    }
    for (int c = 0; c < CT; ++c) {
        const int64_t i = i0 + c;
        if (i <= L1 && j <= L2) cnt[i * N + j] = T[c + 1][lane + 1];
    }
}

// Alignment first + p for p = 0 .. count-1: its moves from the corner back to
// (0,0) -- the order the reference fills its X / Y buffers -- 1 = diag,
// 2 = up, 4 = left; lens[p] = number of moves (0 if there is no such path).
__global__ void nw_unrank_kernel(nwk::TableView v, const uint64_t* cnt, int64_t L1, int64_t L2, uint64_t first,
                                 uint64_t count, uint64_t total, uint8_t* moves, int64_t stride, int32_t* lens) {
    const int64_t N = L2 + 1;
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < count;
         p += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = first + p;
        uint8_t* out = moves + p * (uint64_t)stride;
        if (k >= total) {
            lens[p] = 0;
            continue;
        }
        int64_t i = L1, j = L2, n = 0;
        while (i > 0 || j > 0) {
            const uint32_t code = i == 0 ? 2u : (j == 0 ? 4u : nwk::code_at(v, i, j));
            uint8_t mv = 2;
            if (code & 1u) {
                const uint64_t c = cnt[(i - 1) * N + (j - 1)];
                if (k < c) mv = 1;
                else k -= c;
            }
            if (mv != 1 && (code & 4u)) {
                const uint64_t c = cnt[(i - 1) * N + j];
                if (k < c) mv = 4;
                else k -= c;
            }
            out[n++] = mv;
            if (mv != 4) --j;
            if (mv != 2) --i;
        }
        lens[p] = (int32_t)n;
    }
}

int check_walkable(nw_table* t, const char* who) {
    if (!t) return nwi::fail(NW_ERR_ARG, std::string(who) + ": NULL table");
    if (!t->filled || !(t->last_mask & NW_OUT_DIRS))
        return nwi::fail(NW_ERR_STATE, std::string(who) + ": no direction codes (fill with NW_OUT_DIRS first)");
    if (t->row_base > 0 || t->xout)
        return nwi::fail(NW_ERR_STATE, std::string(who) + ": a row panel is not a whole table");
    return NW_OK;
}

int walk_state(nw_table* t, nw_walk_state** out) {
    if (!t->walk) {
        t->walk = new nw_walk_state;
        NW_HIPCHK(hipMalloc(&t->walk->ctl, 64));
    }
    *out = t->walk;
    return NW_OK;
}

}  // namespace

namespace nwi {

void walk_release(nw_table* t) {
    if (!t || !t->walk) return;
    (void)hipFree(t->walk->rows);
    (void)hipFree(t->walk->ctl);
    (void)hipFree(t->walk->moves);
    (void)hipFree(t->walk->cnt);
    (void)hipFree(t->walk->emoves);
    (void)hipFree(t->walk->elens);
    delete t->walk;
    t->walk = nullptr;
}

}  // namespace nwi

extern "C" {

int nw_table_count_alignments(nw_table* t, uint32_t* count) {
    int rc = check_walkable(t, "nw_table_count_alignments");
    if (rc) return rc;
    if (!count) return nwi::fail(NW_ERR_ARG, "nw_table_count_alignments: NULL count");
    if (t->L1 == 0 || t->L2 == 0) {
        // One path along the seeded row or column -- or none for two empty
        // strings: the walk starts on (0,0), whose three directions are
        // already done (computation.c:96-99), so the loop never runs and no
        // solution is counted (needleman-wunsch.c:231-235).
        *count = (t->L1 == 0 && t->L2 == 0) ? 0u : 1u;
        return NW_OK;
    }
    NW_HIPCHK(hipSetDevice(t->device));
    nw_walk_state* w = nullptr;
    if ((rc = walk_state(t, &w))) return rc;
    const int64_t NG = t->NG;
    const size_t need = (size_t)std::max<int64_t>(NG - 1, 1) * (size_t)t->L1 * 8;
    if (need > w->rows_bytes) {
        (void)hipFree(w->rows);
        w->rows = nullptr;
        w->rows_bytes = 0;
        NW_HIPCHK(hipMalloc(&w->rows, need));
        NW_HIPCHK(hipMemsetAsync(w->rows, 0, need, t->stream));
        w->rows_bytes = need;
    }
    if (++w->epoch & POISON) w->epoch = 1;   // tags stay below the poison bit
    CountArgs a{};
    a.D = t->D;
    a.NC = t->lay_NC;
    a.skew = t->skew;
    a.pair = t->pair;
    a.L1 = (int32_t)t->L1;
    a.L2 = (int32_t)t->L2;
    a.NG = (int32_t)NG;
    a.rows = w->rows;
    a.ctl = w->ctl;
    a.epoch = w->epoch;
    NW_HIPCHK(hipMemsetAsync(w->ctl, 0, 64, t->stream));
    const int grid = (int)std::min<int64_t>(NG, 8 * (int64_t)t->ncu);
    NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    nw_count_kernel<<<grid, 64, 0, t->stream>>>(a);
    NW_HIPCHK(hipGetLastError());
    NW_HIPCHK(hipEventRecord(t->ev[3], t->stream));
    uint32_t ctl[8];
    NW_HIPCHK(hipMemcpyAsync(ctl, w->ctl, sizeof ctl, hipMemcpyDeviceToHost, t->stream));
    NW_HIPCHK(hipStreamSynchronize(t->stream));
    (void)hipEventElapsedTime(&w->count_ms, t->ev[2], t->ev[3]);
    if (ctl[1]) return nwi::fail(NW_ERR_TIMEOUT, "nw_table_count_alignments: stripe hand-off watchdog fired");
    *count = ctl[2];
    return NW_OK;
}

int nw_table_first_path(nw_table* t, uint8_t* moves, int64_t cap, int64_t* n) {
    int rc = check_walkable(t, "nw_table_first_path");
    if (rc) return rc;
    if (!n || (cap > 0 && !moves) || cap < 0) return nwi::fail(NW_ERR_ARG, "nw_table_first_path: bad arguments");
    const int64_t most = t->L1 + t->L2;
    if (cap < most) return nwi::fail(NW_ERR_ARG, "nw_table_first_path: cap < L1 + L2");
    NW_HIPCHK(hipSetDevice(t->device));
    nw_walk_state* w = nullptr;
    if ((rc = walk_state(t, &w))) return rc;
    if ((size_t)std::max<int64_t>(most, 1) > w->moves_bytes) {
        (void)hipFree(w->moves);
        w->moves = nullptr;
        w->moves_bytes = 0;
        NW_HIPCHK(hipMalloc(&w->moves, (size_t)std::max<int64_t>(most, 1)));
        w->moves_bytes = (size_t)std::max<int64_t>(most, 1);
    }
    NW_HIPCHK(hipMemsetAsync(w->ctl, 0, 64, t->stream));
    NW_HIPCHK(hipEventRecord(t->ev[2], t->stream));
    nw_first_path_kernel<<<1, 64, 0, t->stream>>>(t->D, t->lay_NC, t->skew, t->pair, (int32_t)t->L1, (int32_t)t->L2, 1,
                                                  w->moves, w->ctl);
    NW_HIPCHK(hipGetLastError());
    NW_HIPCHK(hipEventRecord(t->ev[3], t->stream));
    uint32_t ctl[8];
    NW_HIPCHK(hipMemcpyAsync(ctl, w->ctl, sizeof ctl, hipMemcpyDeviceToHost, t->stream));
    NW_HIPCHK(hipStreamSynchronize(t->stream));
    (void)hipEventElapsedTime(&w->path_ms, t->ev[2], t->ev[3]);
    if (ctl[4]) return nwi::fail(NW_ERR_STATE, "nw_table_first_path: a cell on the path has no direction code");
    const int64_t len = ctl[3];
    if (len > most) return nwi::fail(NW_ERR_HIP, "nw_table_first_path: path longer than L1 + L2");
    if (len > 0) {
        NW_HIPCHK(hipMemcpyAsync(moves, w->moves, (size_t)len, hipMemcpyDeviceToHost, t->stream));
        NW_HIPCHK(hipStreamSynchronize(t->stream));
    }
    std::reverse(moves, moves + len);
    *n = len;
    return NW_OK;
}

int nw_table_walk_elapsed_ms(nw_table* t, float* count_ms, float* path_ms) {
    if (!t) return nwi::fail(NW_ERR_ARG, "nw_table_walk_elapsed_ms: NULL table");
    if (count_ms) *count_ms = t->walk ? t->walk->count_ms : 0.f;
    if (path_ms) *path_ms = t->walk ? t->walk->path_ms : 0.f;
    return NW_OK;
}

// ---------------------------------------------------------------------------
// Banded checkpoint traceback: the first alignment the
// reference prints, for pairs whose full direction table does not fit.
//
//   1. Forward: the rows are cut into bands of `band_rows` (a multiple of 64).
//      Bands 0 .. K-2 are filled score-only, one after the other, each taking
//      its top row from the band above and handing its bottom row to the band
//      below through the panel boundary granules {epoch, H - d}
//      (fill_launch's xin / xout) -- K-1 rows of L1 granules are all that is
//      kept.
//   2. Backward: band K-1 .. 0 is refilled with direction codes (only columns
//      1 .. i_entry: a walk that entered at column i_entry never goes right)
//      and walked greedily diag > left > up from its entry cell until it
//      leaves through the band's top row; the exit column is the next band's
//      entry.  The greedy order is the reference's print order
//      (needleman-wunsch.c:296-322), so the result is nw_table_first_path's.
// Device memory: band_rows x L1 direction codes (0.5 B per cell) + the K-1
// boundary rows; time: about two fills of the table.
int nw_first_path_banded(int device, const char* s1, int64_t L1, const char* s2, int64_t L2, int32_t m, int32_t k,
                         int32_t d, int64_t band_rows, uint8_t* moves, int64_t cap, int64_t* n) {
    if (L1 < 0 || L2 < 0 || (L1 && !s1) || (L2 && !s2) || !n || cap < L1 + L2 || (cap > 0 && !moves) ||
        band_rows < 64 || band_rows % 64 != 0 || L1 > INT32_MAX - 64 || L2 > INT32_MAX - 4096)
        return nwi::fail(NW_ERR_ARG, "nw_first_path_banded: bad arguments (band_rows: a positive multiple of 64)");
    *n = 0;
    if (L1 == 0 || L2 == 0) {   // the seeded row / column
        for (int64_t x = 0; x < L2; ++x) moves[x] = 2;
        for (int64_t x = 0; x < L1; ++x) moves[L2 + x] = 4;
        *n = L1 + L2;
        return NW_OK;
    }
    const int64_t K = (L2 + band_rows - 1) / band_rows;
    const int64_t rows_max = std::min(band_rows, L2);
    nw_table* t = nullptr;
    int rc = nw_table_create(device, L1, rows_max, NW_OUT_DIRS, &t);
    if (rc) return rc;
    uint64_t* rows = nullptr;   // boundary b (below band b): rows[b * L1 ..]
    uint32_t* ctl = nullptr;
    uint8_t* dmoves = nullptr;
    std::vector<uint8_t> path;  // back to front
    path.reserve((size_t)(L1 + L2));
    auto done = [&](int r) {
        (void)hipFree(rows);
        (void)hipFree(ctl);
        (void)hipFree(dmoves);
        t->xin = nullptr;
        t->xout = nullptr;
        nw_table_destroy(t);
        return r;
    };
    auto hipchk = [&](hipError_t e, const char* what) {
        return e == hipSuccess ? NW_OK : nwi::fail(NW_ERR_HIP, std::string("nw_first_path_banded: ") + what + ": " +
                                                                   hipGetErrorString(e));
    };
    if ((rc = hipchk(hipMalloc(&rows, (size_t)std::max<int64_t>(K - 1, 1) * (size_t)L1 * 8), "hipMalloc(rows)")))
        return done(rc == NW_ERR_HIP ? NW_ERR_OOM : rc);
    if ((rc = hipchk(hipMalloc(&ctl, 64), "hipMalloc")) || (rc = hipchk(hipMalloc(&dmoves, (size_t)(L1 + band_rows)), "hipMalloc")))
        return done(rc);
    t->L2_total = L2;
    t->epoch = 1;            // one producer per boundary, bands run one after the other
    t->xblk = 1;
    auto setup = [&](int64_t b, int64_t cols) -> int {
        const int64_t r0 = b * band_rows, nr = std::min(band_rows, L2 - r0);
        t->row_base = r0;
        t->xin = b > 0 ? rows + (b - 1) * L1 : nullptr;
        t->xout = nullptr;
        return nw_table_set_sequences(t, s1, cols, s2 + r0, nr);
    };
    // 1. forward, score-only: bands 0 .. K-2 hand their bottom rows down
    for (int64_t b = 0; b + 1 < K; ++b) {
        if ((rc = setup(b, L1))) return done(rc);
        t->xout = rows + b * L1;
        if ((rc = nw_table_fill(t, m, k, d, 0u))) return done(rc);
    }
    // 2. backward: refill each band with codes, walk it bottom-up
    int64_t ie = L1;
    for (int64_t b = K - 1; b >= 0; --b) {
        const int64_t r0 = b * band_rows, nr = std::min(band_rows, L2 - r0);
        if (ie == 0) {       // on column 0: up moves to (0, 0)
            path.insert(path.end(), (size_t)nr, (uint8_t)2);
            continue;
        }
        if ((rc = setup(b, ie))) return done(rc);
        if ((rc = nw_table_fill(t, m, k, d, NW_OUT_DIRS))) return done(rc);
        if ((rc = hipchk(hipMemsetAsync(ctl, 0, 64, t->stream), "hipMemset"))) return done(rc);
        nw_first_path_kernel<<<1, 64, 0, t->stream>>>(t->D, t->lay_NC, t->skew, t->pair, (int32_t)ie, (int32_t)nr,
                                                      b == 0 ? 1 : 0, dmoves, ctl);
        if ((rc = hipchk(hipGetLastError(), "first path kernel"))) return done(rc);
        uint32_t hc[8];
        if ((rc = hipchk(hipMemcpyAsync(hc, ctl, sizeof hc, hipMemcpyDeviceToHost, t->stream), "hipMemcpy")))
            return done(rc);
        if ((rc = hipchk(hipStreamSynchronize(t->stream), "hipStreamSynchronize"))) return done(rc);
        if (hc[4]) return done(nwi::fail(NW_ERR_STATE, "nw_first_path_banded: a cell on the path has no direction code"));
        const size_t off = path.size();
        path.resize(off + hc[3]);
        if (hc[3] > 0 &&
            (rc = hipchk(hipMemcpy(path.data() + off, dmoves, hc[3], hipMemcpyDeviceToHost), "hipMemcpy(moves)")))
            return done(rc);
        ie = hc[5];
    }
    if ((int64_t)path.size() > L1 + L2) return done(nwi::fail(NW_ERR_HIP, "nw_first_path_banded: path too long"));
    std::reverse_copy(path.begin(), path.end(), moves);
    *n = (int64_t)path.size();
    return done(NW_OK);
}


int nw_table_enumerate_paths(nw_table* t, uint64_t first, uint64_t count, uint8_t* moves, int64_t stride,
                             int32_t* lens, uint64_t* n_out, uint64_t* total) {
    int rc = check_walkable(t, "nw_table_enumerate_paths");
    if (rc) return rc;
    const int64_t L1 = t->L1, L2 = t->L2;
    if ((count && (!moves || !lens)) || stride < L1 + L2)
        return nwi::fail(NW_ERR_ARG, "nw_table_enumerate_paths: bad arguments (stride >= L1 + L2)");
    NW_HIPCHK(hipSetDevice(t->device));
    nw_walk_state* w = nullptr;
    if ((rc = walk_state(t, &w))) return rc;
    const int64_t N = L2 + 1;
    const size_t need = (size_t)(L1 + 1) * (size_t)N * 8;
    if (w->cnt_serial != t->fill_serial) {
        if (w->cnt_bytes < need) {
            (void)hipFree(w->cnt);
            w->cnt = nullptr;
            w->cnt_bytes = 0;
            // The path-count table is 8 bytes per cell, ~20x the direction
            // codes: say so up front instead of failing inside hipMalloc
            // ($NW_ENUM_MAX_BYTES caps it, e.g. to exercise a caller's fallback).
            size_t free_b = 0, total_b = 0;
            NW_HIPCHK(hipMemGetInfo(&free_b, &total_b));
            if (const char* e = getenv("NW_ENUM_MAX_BYTES")) free_b = std::min<size_t>(free_b, (size_t)atoll(e));
            if (need > free_b)
                return nwi::fail(NW_ERR_OOM, "nw_table_enumerate_paths: the path-count table needs " +
                                                 std::to_string(need) + " bytes (8 per cell), " +
                                                 std::to_string(free_b) + " available on the device; copy the codes "
                                                 "(nw_table_copy_codes) and walk them on the host, or use "
                                                 "nw_table_first_path / nw_first_path_banded");
            NW_HIPCHK(hipMalloc(&w->cnt, need));
            w->cnt_bytes = need;
        }
        const nwk::TableView v = nwk::view_of(t);
        nw_count_border_kernel<<<256, 256, 0, t->stream>>>(w->cnt, L1, L2);
        NW_HIPCHK(hipGetLastError());
        const int nti = (int)((L1 + CT - 1) / CT), ntj = (int)((L2 + 63) / 64);
        for (int dg = 0; L1 > 0 && L2 > 0 && dg < nti + ntj - 1; ++dg) {
            const int lo = std::max(0, dg - (nti - 1)), hi = std::min(dg, ntj - 1);
            nw_count_tiles_kernel<<<hi - lo + 1, 64, 0, t->stream>>>(v, w->cnt, L1, L2, dg, ntj);
        }
        NW_HIPCHK(hipGetLastError());
        NW_HIPCHK(hipStreamSynchronize(t->stream));
        w->cnt_serial = t->fill_serial;
    }
    uint64_t tot = 0;
    if (L1 > 0 || L2 > 0)   // two empty strings: the reference's walk prints nothing (see count_alignments)
        NW_HIPCHK(hipMemcpy(&tot, w->cnt + L1 * N + L2, 8, hipMemcpyDeviceToHost));
    if (total) *total = tot;
    const uint64_t avail = first < tot ? tot - first : 0;
    const uint64_t todo = std::min(count, avail);
    // batches bounded by 64 MB of moves on the device
    const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, ((uint64_t)64 << 20) / (uint64_t)std::max<int64_t>(stride, 1)));
    const size_t mb = (size_t)(std::min(per, std::max<uint64_t>(todo, 1)) * (uint64_t)std::max<int64_t>(stride, 1));
    if (todo && (w->ebytes < mb || w->elens_n < std::min(per, todo))) {
        (void)hipFree(w->emoves);
        (void)hipFree(w->elens);
        w->emoves = nullptr;
        w->elens = nullptr;
        w->ebytes = w->elens_n = 0;
        NW_HIPCHK(hipMalloc(&w->emoves, mb));
        NW_HIPCHK(hipMalloc(&w->elens, (size_t)std::min(per, todo) * 4));
        w->ebytes = mb;
        w->elens_n = (size_t)std::min(per, todo);
    }
    const nwk::TableView v = nwk::view_of(t);
    for (uint64_t done = 0; done < todo;) {
        const uint64_t b = std::min(per, todo - done);
        nw_unrank_kernel<<<(unsigned)std::min<uint64_t>((b + 255) / 256, 4096), 256, 0, t->stream>>>(
            v, w->cnt, L1, L2, first + done, b, tot, w->emoves, stride, w->elens);
        NW_HIPCHK(hipGetLastError());
        NW_HIPCHK(hipMemcpyAsync(moves + done * (uint64_t)stride, w->emoves, (size_t)(b * (uint64_t)stride),
                                 hipMemcpyDeviceToHost, t->stream));
        NW_HIPCHK(hipMemcpyAsync(lens + done, w->elens, (size_t)b * 4, hipMemcpyDeviceToHost, t->stream));
        NW_HIPCHK(hipStreamSynchronize(t->stream));
        done += b;
    }
    for (uint64_t p = todo; p < count; ++p) lens[p] = 0;
    if (n_out) *n_out = todo;
    return NW_OK;
}

}  // extern "C"
