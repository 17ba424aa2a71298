// nw_kern.h -- definitions shared by the fill kernels (nw_fill.hip: the
// column-scan kernel; nw_skew.hip: the skewed-stripe kernel) and their
// launcher.  Device-side only; not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "nw_internal.h"

namespace nwk {

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
    int32_t NC;             // chunks = ceil(L1 / 8) (ring slots / granule chunks)
    int32_t NCH;            // skew kernel: 8-step chunks per stripe = ceil((L1 + 63) / 8)
    int32_t NG;             // wave stripes = ceil(L2 / 64)
    int32_t NSW;            // workgroup stripes (WG-stripes)
    int32_t SQ, SR;         // WG-stripe k holds stripes g0 = k*SQ + min(k, SR) .. + SQ + (k < SR) - 1
                            // (clipped to NG): the first SR WG-stripes hold one stripe more
    int32_t* H;             // score tiles, see score_at()
    int64_t spitch;         // 512*NC: elements per 64-row stripe
    uint32_t* D;            // codes: word ((g*NC + q)*64 + lane)
    int32_t* lastcol;       // score-only: H[L1][j] at lastcol[63 + j]
    uint64_t* gran;         // boundary granules, slot s at gran + s*gpitch (see put_granule)
    int64_t gpitch;
    int32_t nslot;
    uint32_t* ctl;          // CtlWord
    uint64_t* trace;        // optional timeline: 8 words per WG-stripe (see nw_table_trace)
    int64_t spin_ticks;     // hand-off watchdog (s_memrealtime ticks)
    // Row panels (multi-GPU, nw_panel.h).  The table holds global rows
    // row_base+1 .. row_base+L2; row 0 is the boundary row of the panel above.
    int32_t row_base;
    uint32_t epoch;         // tag of this fill's panel hand-off granules
    uint32_t gtag;          // WG-stripe granule tags of this fill: gtag | (consumer's WG-stripe index)
    const uint64_t* xin;    // top boundary row {epoch, H-d} per column, or null (= seeded row 0)
    uint64_t* xout;         // bottom row granules for the panel below, or null
    uint32_t* xflag;        // host-visible: xflag[b] = epoch once block b of xout is written
    int32_t xblk;           // chunks per block
    // Panel back-pressure (IPC / group transports; null otherwise).  The
    // consumer snapshots the row above into row0 (H - d per column) while its
    // loader reads xin, then posts this fill's epoch to xin_credit; the
    // producer's first xout store of a fill waits until xout_credit (the
    // consumer's xin_credit) reads credit_want, the epoch of its previous
    // fill -- so a producer never overwrites a row its consumer still reads.
    int32_t* row0;
    uint32_t* xin_credit;
    const uint32_t* xout_credit;
    uint32_t credit_want;
};

// ---------------------------------------------------------------- DPP helpers
typedef const __attribute__((address_space(4))) uint64_t* cptr64;
typedef __attribute__((address_space(1))) uint64_t gu64;   // global-address-space granule


// LDS byte address of a __shared__ object (for ds_* in inline asm).
__device__ __forceinline__ int lds_addr(const void* p) {
    return (int)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Wave-uniform copies of per-wave values (so address math stays scalar).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

constexpr int SUPER_CHUNKS = 512;     // chunks per super-chunk (4096 columns)

__device__ __forceinline__ int chunk_base(int c) { return (c / SUPER_CHUNKS) * (SUPER_CHUNKS * CH); }

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

// Ring slot stride (ints): 8 values of a chunk (+ the scan kernel's 8 top-string bytes).
constexpr int SLOT = 16;

// WG-stripe to WG-stripe granule: ONE aligned 8-byte write-through (sc1)
// store {tag, value}; the loader polls it with sc1 loads (R2 of the CDNA
// guide's Guideline 16: the data is the flag).  Measured at 100k^2: ~1.2 us
// from the producer wave starting a chunk to its granules stored, ~2.5 us
// more until the next WG-stripe's loader sees them, wherever the two
// WG-stripes sit (tools/trace_lag.py; an L2-resident second copy for
// same-XCD consumers and 128-byte padded lines were both slower; plain
// stores with one agent release per batch, 0.43 -> 1.2 us in isolation
// beside a store stream against 1.9 us for sc1 (tools/ubench_handoff.hip),
// made the 100k^2 fill 8x slower: the release writes back the L2 that the
// table stream keeps dirty).
__device__ __forceinline__ void put_granule(uint64_t* gout, int64_t idx, uint64_t gr) {
    __hip_atomic_store(gout + idx, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Hand-off granule load: agent scope between workgroups of one fill, system
// scope (bypassing L2) for the panel boundary, which another agent writes.
__device__ __forceinline__ uint64_t ld_gran(const uint64_t* p, bool sys) {
    return sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
               : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Epochs run 1 .. 2^31 - 1 and wrap to 1 (bit 31 is the poison bit); c is "at
// or after" want when it is less than half the ring ahead of it.
__host__ __device__ __forceinline__ bool epoch_reached(uint32_t c, uint32_t want) {
    return ((c - want) & 0x7fffffffu) < 0x40000000u;
}

// Producer side of the panel back-pressure (FillArgs.xout_credit): one wave
// waits until the consumer has read the previous fill's boundary row, i.e.
// until its credit word reads that fill's epoch or a later one (a consumer
// whose fill failed or never launched posts its credit from the host, so
// one failed panel does not stall its producer's next fill).  False when the
// fill is being aborted (another wave's failure, or this wait's watchdog:
// NW_ERR_TIMEOUT).
__device__ __forceinline__ bool xcredit_wait(const FillArgs& a, const int* sh_abort) {
    if (!a.xout_credit) return true;
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t c = __hip_atomic_load(a.xout_credit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (epoch_reached((uint32_t)__builtin_amdgcn_readfirstlane((int)c), a.credit_want)) return true;
        const uint32_t ab = __hip_atomic_load(&a.ctl[CTL_ABORT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ab || __hip_atomic_load(sh_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        if ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 > a.spin_ticks) {
            if ((threadIdx.x & 63) == 0) {
                __hip_atomic_store(&a.ctl[CTL_ABORT], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicCAS(&a.ctl[CTL_ERR], 0u, (uint32_t)NW_ERR_TIMEOUT);
            }
            return false;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// Consumer side: the row above is read (and kept in row0); release xin.
__device__ __forceinline__ void xcredit_post(const FillArgs& a) {
    if (a.xin_credit && (threadIdx.x & 63) == 0)
        __hip_atomic_store(a.xin_credit, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LDS counters of the barrier-free intra-workgroup pipeline.
__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(int* p, int v) {
    // Every LDS write this wave issued before (ring data) lands first: the
    // LDS executes one wave's DS instructions in order, so a reader that sees
    // the counter and then reads the ring sees the data.
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Compiler-only fence for the LDS ring handshakes written in C++: the LDS
// performs one wave's DS instructions in issue order, so keeping the plain
// slot reads / writes on their side of the relaxed counter accesses in the
// instruction stream is all the ordering they need.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// Extended trace stamps (tools/trace_lag.py) are compiled in only with
// -DNW_TRACE_EXT=1 (tools/ab_build.sh): even a never-taken stamp branch in
// the pair kernel's loops moved the 100k^2 fill by several percent.
#ifndef NW_TRACE_EXT
#define NW_TRACE_EXT 0
#endif

// Trace words after the 8 per WG-stripe (nw_fill.hip, $NW_TRACE; pair kernel):
// per 128-row stripe the time it starts the middle chunk cm, then per
// WG-stripe: publisher has stored cm's granules, loader has cm in ring 0,
// loader reaches cm, loader has a free ring slot for cm.
enum TraceExt { TX_MID = 0, TX_PUB = 1, TX_LOAD = 2, TX_REACH = 3, TX_CREDIT = 4 };
__device__ __forceinline__ uint64_t* trace_ext(const FillArgs& a, int kind, int idx) {
    const int64_t base = 8 * (int64_t)a.NSW;
    return a.trace + base + (kind == TX_MID ? idx : a.NG + (int64_t)(kind - 1) * a.NSW + idx);
}
__device__ __forceinline__ int trace_mid_chunk(int NC, int R) { return ((NC - 1) / 2) & ~(R - 1); }

// ---------------------------------------------------------------- table views
// (shared by the copy / hash kernels of nw_fill.hip and the walk services of
// nw_walk.hip)
#ifndef NW_SCORE_X4
#define NW_SCORE_X4 1
#endif

// Device view of a filled table for the copy / hash kernels.
struct TableView {
    const int32_t* tiles;   // score tiles
    int64_t spitch;
    const uint32_t* D;      // codes, or null
    int32_t NC;             // chunks per stripe of the layout (scan: ceil(L1/8); skew: ceil((L1+63)/8))
    int32_t skew;           // 0: column layout; 1: skewed by lane (nw_skew.hip); 2: by 16-lane row (nw_quad.hip)
    int32_t pair;           // 1: column layout with rows permuted (nw_pair.hip)
    int32_t raw;            // 1: the tiles hold the pair kernel's G', 2: the quad kernel's (see raw_offset)
    int32_t SQ, SR;         // raw: the fill's WG-stripe plan (FillArgs)
    int32_t d;
    int32_t row_base;       // panels: global row of local row 0
    const int32_t* top;     // panels: the row above (H - d, nw_table.row0), or null for row 0 = seed
};

// Score of cell (i, j) in the device layout.  Row 0 and column 0 are the
// reference's seeds (computation.c:93-120), computed, not stored; a panel's
// row 0 is the last row of the panel above, kept in row0 by the loader.
// Interior cells live in stripe tiles: stripe g = (j-1)/64, lane l =
// (j-1)%64, spitch = 512*NC elements per stripe.  Quad tiles (NW_SCORE_X4):
// column i = 4q + r + 1 at g*spitch + (q*64 + l)*4 + r, so a lane's 4
// consecutive columns are one 16-byte store and a chunk is 2 KB contiguous.
// Column tiles: g*spitch + (i-1)*64 + l, one 256-byte store per column.
// Skewed layouts: stored by step instead of by column, same quad tiles.
// skew = 1 (nw_skew.hip): step t = c + (r & 63), every lane one column behind
// the lane above; skew = 2 (nw_quad.hip): t = c + ((r & 63) >> 4), every
// 16-lane DPP row one column behind the row above.
// Pair layout (nw_pair.hip): the column layout of the permuted row
// nwi::pair_row(r).
__host__ __device__ __forceinline__ int64_t skew_off(int skew, int64_t lane) {
    return skew == 1 ? lane : skew == 2 ? lane >> 4 : 0;
}

__host__ __device__ __forceinline__ int64_t score_index(int64_t r, int64_t c, int64_t spitch, int skew = 0,
                                                         bool pair = false) {
    if (pair) r = nwi::pair_row(r);
    c += skew_off(skew, r & 63);
#if NW_SCORE_X4
    return (r >> 6) * spitch + ((c >> 2) * 64 + (r & 63)) * 4 + (c & 3);
#else
    return (r >> 6) * spitch + c * 64 + (r & 63);
#endif
}

// Code word and bit position of interior cell (i, j) (see include/nw_fill.h).
__host__ __device__ __forceinline__ int64_t code_word(int64_t i, int64_t j, int64_t NC, int skew, int* shift,
                                                      bool pair = false) {
    const int64_t rr = pair ? nwi::pair_row(j - 1) : j - 1;
    const int64_t g = rr >> 6, l = rr & 63;
    const int64_t t = (i - 1) + skew_off(skew, l);
    *shift = 21 - 3 * (int)(t & 7);
    return (g * (NC + 1) + (t >> 3) + 1) * 64 + l;
}

// Raw pair tiles (nw_pair.hip, RAW) hold G' = H + r*d + (i - base)*d of the
// kernel's domain: r = the row's offset inside its WG-stripe (pair stripes
// g0 = s*SQ + min(s, SR) .. of WG-stripe s, 128 rows each), base = the first
// column of the cell's 4096-column super-chunk.  H = G' - raw_offset (mod 2^32,
// as the kernel computes).
// The quad kernel (raw = 2) has 64-row stripes and no column base: G' = H + r*d + i*d.
__host__ __device__ __forceinline__ uint32_t raw_offset(int64_t i, int64_t j, int SQ, int SR, int32_t d, int raw = 1) {
    const int sh = raw == 2 ? 6 : 7;
    const int64_t rr = j - 1, g = rr >> sh;
    const int64_t big = (int64_t)SR * (SQ + 1);
    const int64_t s = g < big ? g / (SQ + 1) : SR + (g - big) / SQ;
    const int64_t g0 = s * SQ + (s < SR ? s : SR);
    const int64_t r = rr - (g0 << sh);
    const int64_t base = raw == 2 ? 0 : ((i - 1) >> 12) << 12;
    return (uint32_t)(r + (i - base)) * (uint32_t)d;
}

__device__ __forceinline__ int32_t score_at(const TableView& v, int64_t i, int64_t j) {
    if (i == 0) return (int32_t)(-(j + v.row_base) * (int64_t)v.d);
    if (j == 0) return v.top ? v.top[i - 1] + v.d : (int32_t)(-i * (int64_t)v.d);
    const int32_t x = v.tiles[score_index(j - 1, i - 1, v.spitch, v.skew, v.pair)];
    return v.raw ? (int32_t)((uint32_t)x - raw_offset(i, j, v.SQ, v.SR, v.d, v.raw)) : x;
}

// Direction code of cell (i, j).  A panel's row 0 belongs to the panel above
// and reads as 0 here.
__device__ __forceinline__ uint32_t code_at(const TableView& v, int64_t i, int64_t j) {
    if (j == 0 && v.row_base > 0) return 0u;
    if (i == 0) return j == 0 ? 0u : 2u;          // (0,0): none; (0,j): up
    if (j == 0) return 4u;                         // (i,0): left
    int sh;
    const int64_t wd = code_word(i, j, v.NC, v.skew, &sh, v.pair);
    return (v.D[wd] >> sh) & 7u;
}

// The device view of a table's last fill (nw_fill.hip).
TableView view_of(const nw_table* t);

using KernelFn = void (*)(FillArgs);

// nw_skew.hip: the skewed-stripe kernel for W compute waves per workgroup
// (nullptr for an unsupported W).
KernelFn pick_skew(int W, bool prof, bool sh, bool sd, bool stt);
// nw_pair.hip: the two-rows-per-lane scan kernel.
KernelFn pick_pair(int W, bool prof, bool sh, bool sd, bool stt);
// nw_quad.hip: the one-row scan kernel with 16-lane skewed row groups (no stats).
KernelFn pick_quad(int W, bool prof, bool sh, bool sd);

}  // namespace nwk
