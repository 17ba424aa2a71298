// nw_internal.h -- state shared by nw_fill.hip (single-GPU table) and
// nw_panel.hip (row panels across GPUs).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "nw_fill.h"

struct nw_walk_state;   // nw_walk.hip: count / first-path buffers

struct nw_table {
    int device = 0;
    int ncu = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t cap_mask = 0;
    int64_t max_L1 = 0, max_L2 = 0;
    // geometry for the current sequences
    int64_t L1 = -1, L2 = -1;
    int64_t NC = 0, NG = 0, spitch = 0;   // NC = ceil(L1/8) column chunks; spitch: see fill_launch
    int skew = 0;                   // layout of the tables: 1 = skewed (nw_skew.hip), 0 = column (scan)
    int pair = 0;                   // 1: column layout with rows permuted (nw_pair.hip, nwi::pair_row)
    int raw = 0;                    // 1: pair tiles hold G' (nwk::raw_offset) under plan SQ / SR
    int32_t SQ = 0, SR = 0;
    int64_t lay_NC = 0;             // chunks per stripe of that layout
    int alpha = 0;                  // s1/s2 coded to symbols 0..alpha-1 on the device (<= 8), 0: raw bytes
    // device buffers
    uint8_t* s1 = nullptr;
    uint8_t* s2 = nullptr;
    int32_t* H = nullptr;       // score tiles (score_at)
    uint32_t* D = nullptr;
    int32_t* lastcol = nullptr;
    uint64_t* gran = nullptr;
    size_t gran_bytes = 0;
    uint32_t* ctl = nullptr;
    uint64_t* trace = nullptr;      // $NW_TRACE: in-kernel timeline
    int64_t trace_n = 0;
    uint64_t trace_hdr[2] = {0, 0};
    // Row-panel hand-off (set by nw_panel.hip; all null for a plain table).
    int64_t row_base = 0;           // global row of local row 0
    int64_t L2_total = -1;          // global rows, for the overflow guard (-1: L2)
    const uint64_t* xin = nullptr;  // top boundary granules (device), or null
    uint64_t* xout = nullptr;       // bottom boundary granules (device, maybe a peer's xin)
    uint32_t* xflag = nullptr;      // host-visible block flags, or null
    int64_t xblk = 0;               // chunks per hand-off block
    uint32_t epoch = 0;             // tag of the fill in flight
    uint32_t gseq = 0;              // WG-stripe granule tag sequence (16 bits, fill_launch)
    size_t gran_clean = 0;          // bytes of the granule slots zeroed since allocation
    int32_t* row0 = nullptr;        // device: the row above (H - d per column), snapshot by the loader
    uint32_t* xin_credit = nullptr;       // consumer: where it posts "row above read" (FillArgs)
    const uint32_t* xout_credit = nullptr;// producer: its consumer's xin_credit
    uint32_t credit_want = 0;             // producer: the epoch xout_credit must read
    // fill in flight (between fill_launch and fill_finish)
    bool launched = false;
    uint32_t pend_mask = 0;
    int32_t pend_d = 0;
    int pend_W = 0;
    int pend_skew = 0;
    int pend_pair = 0;
    int pend_raw = 0;
    int32_t pend_SQ = 0, pend_SR = 0;
    // results of the last fill
    bool filled = false;
    uint64_t fill_serial = 0;       // completed fills (walk services cache per fill)
    uint32_t last_mask = 0;
    int32_t last_d = 0;
    nw_stats stats{};
    float kernel_ms = 0.f, call_ms = 0.f;
    int waves = 0;
    nw_walk_state* walk = nullptr;  // lazily created by the walk services
    // Host I/O (nw_fill.hip "Host I/O"): pinned upload staging, and the
    // double-buffered device/pinned staging of streamed slice copies.
    uint8_t* h_seq = nullptr;       // pinned: coded s1 | s2 for the upload
    size_t h_seq_bytes = 0;
    void* d_stage[2] = {nullptr, nullptr};
    void* h_stage[2] = {nullptr, nullptr};   // pinned bounce buffers (pageable destinations)
    size_t stage_bytes = 0;
    hipStream_t copy_stream = nullptr;
    hipEvent_t cev[4] = {nullptr, nullptr, nullptr, nullptr};   // gathered[2], copied[2]
    double upload_ms = 0.0, copy_ms = 0.0;
    int64_t upload_bytes = 0, copy_bytes = 0;
};

namespace nwi {

int fail(int rc, const std::string& msg);

// Enqueue one fill on t->stream (no host synchronisation), then complete it.
// nw_table_fill() is fill_launch + fill_finish; panels run their boundary
// transport in between.
int fill_launch(nw_table* t, int32_t m, int32_t k, int32_t d, uint32_t out_mask);
int fill_finish(nw_table* t);

// Write "producer failed" granules for `epoch` over p[0, n) (any device memory,
// including a peer's mapped boundary buffer), on stream s.
int poison(uint64_t* p, int64_t n, uint32_t epoch, hipStream_t s);

// Free the walk services' buffers (nw_walk.hip); called by nw_table_destroy.
void walk_release(nw_table* t);

constexpr int kChunk = 8;   // columns per chunk (hand-off granules per chunk)

// The pair kernel's row permutation: row r (0-based) of the table lives at
// row pair_row(r) of the 64-row column layout (lane (r%128)/2 of virtual
// stripe 2*(r/128) + r%2).
__host__ __device__ __forceinline__ int64_t pair_row(int64_t r) {
    return 64 * (2 * (r >> 7) + (r & 1)) + ((r & 127) >> 1);
}

}  // namespace nwi

#define NW_HIPCHK(expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return nwi::fail(e_ == hipErrorOutOfMemory ? NW_ERR_OOM : NW_ERR_HIP,           \
                             std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)
