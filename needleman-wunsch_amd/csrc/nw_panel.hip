// nw_panel.hip -- row panels of one score table across GPUs (include/nw_panel.h).
//
// The reference's only parallel schedule is the pthread column-cyclic fill of
// `-p` (needleman-wunsch.c:444-475 per-cell wait/signal, :557-574, :583-626).
// Here each GPU owns a contiguous band of whole 64-row stripes (a row panel)
// and runs the ordinary single-GPU fill kernel on it; the only exchange is
// the panel's bottom row, published by the kernel itself as tagged granules
// {epoch, H - d}, 8 columns per chunk, and consumed by the loader wave of the
// panel below exactly like the hand-off between two workgroup stripes.  Three
// transports (see the header):
//   GROUP  one process: the producer stores into the consumer's xin directly.
//   IPC    one process per GPU: the same stores, into the consumer's xin
//          mapped with hipIpcOpenMemHandle (xGMI between GPUs).
//   RCCL   one process per GPU: the producer's kernel fills its own xout and
//          raises a pinned host flag per block of columns; a host proxy
//          forwards each block with ncclSend, the consumer pre-posts every
//          ncclRecv into its xin.
// This file is host code only; the kernels live in nw_fill.hip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nw_internal.h"
#include "nw_kern.h"
#include "nw_panel.h"

using nwi::fail;
using nwi::kChunk;

namespace {

constexpr uint32_t kEpochMax = 0x7fffffffu;   // bit 31 is the poison bit

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Hand-off block size in chunks ($NW_XBLK columns, default 1024).  Only the
// RCCL transport uses blocks; all ranks must agree on it.
int64_t xblk_chunks() {
    int64_t cols = 1024;
    if (const char* e = getenv("NW_XBLK")) cols = std::max<int64_t>(atoll(e), kChunk);
    return std::max<int64_t>(1, cols / kChunk);
}

int nccl_fail(ncclResult_t r, const char* what) {
    return fail(NW_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

struct nw_panel {
    int transport = NW_PANEL_GROUP;
    int device = 0, rank = 0, nranks = 1;
    nw_table* t = nullptr;
    int64_t max_L1 = 0, max_L2 = 0;
    // current sequences
    bool have_seq = false;
    int64_t L1 = 0, L2 = 0, row_base = 0, rows = 0;
    int prev = -1, next = -1, pos = -1;
    // boundary buffers
    uint64_t* xin = nullptr;        // device: the row above, written by the panel above
    int64_t xcap = 0;               // granules in xin / xout
    uint64_t* xout = nullptr;       // RCCL: device staging of our bottom row
    uint32_t* xflag = nullptr;      // RCCL: pinned host block flags
    uint32_t* xflag_dev = nullptr;
    int64_t xblk = 1;               // RCCL: chunks per block
    std::vector<uint64_t*> peer_xin;   // IPC: every rank's mapped xin (own: null)
    bool connected = false;
    std::vector<nw_panel*> group;      // GROUP: the whole group, rank order
    ncclComm_t comm[2] = {nullptr, nullptr};
    hipStream_t s_send = nullptr, s_recv = nullptr;
    // last fill
    uint32_t epoch = 0;
    bool filled = false;
    int last_rc = NW_OK;
    int32_t last_d = 0;
    nw_stats stats{};               // whole table (GROUP)
    bool have_global = false;
    float call_ms = 0.f;
};

namespace {

int panel_alloc(nw_panel* p, int64_t max_L1, int64_t max_L2, uint32_t out_mask) {
    p->max_L1 = max_L1;
    p->max_L2 = max_L2;
    const int64_t NGmax = cdiv(max_L2, 128);
    const int64_t rows_cap = 128 * std::max<int64_t>(cdiv(NGmax, p->nranks), 1);
    int rc = nw_table_create(p->device, max_L1, std::min(rows_cap, std::max<int64_t>(max_L2, 0)), out_mask, &p->t);
    if (rc) return rc;
    NW_HIPCHK(hipSetDevice(p->device));
    const int64_t NC = cdiv(max_L1, kChunk);
    p->xcap = kChunk * NC + kChunk;
    // The boundary buffer is written by another agent (a peer GPU over xGMI,
    // another process, RCCL): uncached device memory, so the loader's polls
    // can never hit a stale L2 line.
    // One more 64-byte line after the granules: this panel's credit word
    // (credit_of), the back-pressure of the IPC / group transports.
    NW_HIPCHK(hipExtMallocWithFlags(reinterpret_cast<void**>(&p->xin), (size_t)p->xcap * 8 + 64, hipDeviceMallocUncached));
    NW_HIPCHK(hipMemset(p->xin, 0, (size_t)p->xcap * 8 + 64));
    NW_HIPCHK(hipStreamCreateWithFlags(&p->s_send, hipStreamNonBlocking));
    if (p->transport == NW_PANEL_RCCL) {
        p->xblk = xblk_chunks();
        const int64_t nblk = cdiv(std::max<int64_t>(NC, 1), p->xblk) + 1;
        NW_HIPCHK(hipMalloc(&p->xout, (size_t)p->xcap * 8));
        NW_HIPCHK(hipMemset(p->xout, 0, (size_t)p->xcap * 8));
        NW_HIPCHK(hipHostMalloc(&p->xflag, (size_t)nblk * 4, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(p->xflag, 0, (size_t)nblk * 4);
        NW_HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->xflag_dev), p->xflag, 0));
        NW_HIPCHK(hipStreamCreateWithFlags(&p->s_recv, hipStreamNonBlocking));
    }
    NW_HIPCHK(hipDeviceSynchronize());
    return NW_OK;
}

// Per-rank record: {err, has_corner, corner, gav, bc, seed_corner, rows, 0}.
void make_record(const nw_panel* p, int64_t* rec) {
    std::memset(rec, 0, sizeof(int64_t) * NW_PANEL_REC);
    rec[0] = p->last_rc;
    const bool ok = p->last_rc == NW_OK && p->t->filled;
    rec[1] = ok && p->rows > 0 && p->next < 0;
    rec[2] = ok ? p->t->stats.corner : 0;
    rec[3] = ok ? p->t->stats.greatest_abs_interior : 0;
    rec[4] = ok ? p->t->stats.branch_count : 0;
    rec[5] = -(p->L1 + p->L2) * (int64_t)p->last_d;
    rec[6] = p->rows;
}

// The credit word behind a boundary buffer of xcap granules: the epoch of
// the last fill whose row above its owner has finished reading.
uint32_t* credit_of(uint64_t* xin, int64_t xcap) { return reinterpret_cast<uint32_t*>(xin + xcap); }

// prev_epoch: the epoch of this panel's previous fill (0 before the first).
void configure(nw_panel* p, uint32_t epoch, uint32_t prev_epoch) {
    nw_table* t = p->t;
    const bool credits = p->transport != NW_PANEL_RCCL;   // RCCL's own send/recv pairing paces it
    t->epoch = epoch;
    t->xin = (p->prev >= 0 && p->rows > 0) ? p->xin : nullptr;
    t->xin_credit = credits ? credit_of(p->xin, p->xcap) : nullptr;
    t->xout = nullptr;
    t->xout_credit = nullptr;
    t->credit_want = prev_epoch;
    t->xflag = nullptr;
    t->xblk = p->xblk;
    if (p->next >= 0 && p->rows > 0) {
        if (p->transport == NW_PANEL_GROUP) t->xout = p->group[p->next]->xin;
        else if (p->transport == NW_PANEL_IPC) t->xout = p->peer_xin[p->next];
        else {
            t->xout = p->xout;
            t->xflag = p->xflag_dev;
        }
        if (credits) t->xout_credit = credit_of(t->xout, p->xcap);
    }
}

// Every panel posts its credit for every fill, on every path: a fill kernel
// that reads the row above posts it itself once read (xcredit_post);
// otherwise it is posted here, stream-ordered after this panel's work, so a
// producer never waits on a panel that has nothing to read (first panel,
// empty panel, L1 == 0) -- or that failed: a fill that did not launch, or
// whose kernel ended before its loader ran, gets its credit from here as
// well (`failed`: on the send stream and waited for, since the fill's own
// stream may be the thing that broke).  Posting an epoch twice is harmless.
int post_credit(nw_panel* p, bool kernel_posts, bool failed = false) {
    if (p->transport == NW_PANEL_RCCL || (kernel_posts && !failed)) return NW_OK;
    NW_HIPCHK(hipSetDevice(p->device));
    hipStream_t s = failed ? p->s_send : p->t->stream;
    NW_HIPCHK(hipMemsetD32Async(credit_of(p->xin, p->xcap), (int)p->epoch, 1, s));
    if (failed) NW_HIPCHK(hipStreamSynchronize(s));
    return NW_OK;
}

uint32_t next_epoch(uint32_t e) { return e >= kEpochMax ? 1u : e + 1u; }

int first_error(const std::vector<int>& rcs) {
    int peer = NW_OK;
    for (int rc : rcs) {
        if (rc == NW_ERR_PEER) peer = rc;
        else if (rc != NW_OK) return rc;
    }
    return peer;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// The RCCL transport's callbacks for nw_panel_proxy_run.
struct RcclProxy {
    nw_panel* p;
    nw_table* t;
    uint32_t epoch;
    static int recv(void* c, int64_t off, int64_t cnt) {
        auto* x = static_cast<RcclProxy*>(c);
        nw_panel* p = x->p;
        const ncclResult_t r = ncclRecv(p->xin + off, (size_t)cnt, ncclUint64, p->prev, p->comm[(p->pos - 1) & 1],
                                        p->s_recv);
        return r == ncclSuccess ? NW_OK : nccl_fail(r, "ncclRecv");
    }
    static int flag(void* c, int64_t b, uint64_t spin) {
        auto* x = static_cast<RcclProxy*>(c);
        volatile uint32_t* f = x->p->xflag;
        if (f[b] == x->epoch) return 1;
        __builtin_ia32_pause();
        if ((spin & 1023) == 1023 && hipEventQuery(x->t->ev[2]) == hipSuccess) return f[b] == x->epoch ? 1 : -1;
        return 0;
    }
    static int poison(void* c, int64_t off, int64_t cnt) {
        auto* x = static_cast<RcclProxy*>(c);
        return nwi::poison(x->p->xout + off, cnt, x->epoch, x->p->s_send);
    }
    static int send(void* c, int64_t off, int64_t cnt) {
        auto* x = static_cast<RcclProxy*>(c);
        nw_panel* p = x->p;
        const ncclResult_t r = ncclSend(p->xout + off, (size_t)cnt, ncclUint64, p->next, p->comm[p->pos & 1],
                                        p->s_send);
        return r == ncclSuccess ? NW_OK : nccl_fail(r, "ncclSend");
    }
};

extern "C" {

int nw_panel_partition(int64_t L2, int nranks, int rank, int64_t* row_base, int64_t* rows) {
    if (L2 < 0 || nranks < 1 || rank < 0 || rank >= nranks || !row_base || !rows)
        return fail(NW_ERR_ARG, "nw_panel_partition: bad arguments");
    // whole 128-row pair stripes, so every feeding panel can run the pair kernel
    const int64_t NG = cdiv(L2, 128);
    const int64_t g0 = NG * rank / nranks, g1 = NG * (rank + 1) / nranks;
    *row_base = std::min(128 * g0, L2);
    *rows = std::max<int64_t>(0, std::min(128 * g1, L2) - *row_base);
    return NW_OK;
}

int nw_panel_chain(int64_t L2, int nranks, int rank, int* prev, int* next, int* pos) {
    if (L2 < 0 || nranks < 1 || rank < 0 || rank >= nranks || !prev || !next || !pos)
        return fail(NW_ERR_ARG, "nw_panel_chain: bad arguments");
    auto rows_of = [&](int r) {
        int64_t b, n;
        nw_panel_partition(L2, nranks, r, &b, &n);
        return n;
    };
    *prev = *next = -1;
    *pos = -1;
    if (rows_of(rank) == 0) return NW_OK;
    int before = 0;
    for (int r = 0; r < rank; ++r)
        if (rows_of(r) > 0) {
            *prev = r;
            ++before;
        }
    for (int r = rank + 1; r < nranks; ++r)
        if (rows_of(r) > 0) {
            *next = r;
            break;
        }
    *pos = before;
    return NW_OK;
}

int nw_panel_get_id(uint8_t id[NW_PANEL_ID_BYTES]) {
    if (!id) return fail(NW_ERR_ARG, "nw_panel_get_id: NULL id");
    static_assert(2 * sizeof(ncclUniqueId) <= NW_PANEL_ID_BYTES, "id size");
    ncclUniqueId u[2];
    for (auto& x : u) {
        ncclResult_t r = ncclGetUniqueId(&x);
        if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    }
    std::memset(id, 0, NW_PANEL_ID_BYTES);
    std::memcpy(id, u, sizeof u);
    return NW_OK;
}

void nw_panel_destroy(nw_panel* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    if (p->s_send) (void)hipStreamSynchronize(p->s_send);
    if (p->s_recv) (void)hipStreamSynchronize(p->s_recv);
    for (auto& c : p->comm)
        if (c) (void)ncclCommDestroy(c);
    for (uint64_t* q : p->peer_xin)
        if (q) (void)hipIpcCloseMemHandle(q);
    nw_table_destroy(p->t);
    (void)hipFree(p->xin);
    (void)hipFree(p->xout);
    if (p->xflag) (void)hipHostFree(p->xflag);
    if (p->s_send) (void)hipStreamDestroy(p->s_send);
    if (p->s_recv) (void)hipStreamDestroy(p->s_recv);
    // a group member leaves the group
    for (nw_panel* q : p->group)
        if (q && q != p)
            for (auto& x : q->group)
                if (x == p) x = nullptr;
    delete p;
}

int nw_panel_create(int transport, int device, int rank, int nranks, const uint8_t* id, int64_t max_L1,
                    int64_t max_L2, uint32_t out_mask, nw_panel** out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || max_L1 < 0 || max_L2 < 0 ||
        (transport != NW_PANEL_IPC && transport != NW_PANEL_RCCL) || (transport == NW_PANEL_RCCL && !id))
        return fail(NW_ERR_ARG, "nw_panel_create: bad arguments");
    *out = nullptr;
    nw_panel* p = new nw_panel;
    p->transport = transport;
    p->rank = rank;
    p->nranks = nranks;
    p->peer_xin.assign((size_t)nranks, nullptr);
    if (device < 0) {
        const char* e = getenv("NW_DEVICE");
        device = e ? atoi(e) : 0;
    }
    p->device = device;
    int rc = panel_alloc(p, max_L1, max_L2, out_mask);
    if (!rc && transport == NW_PANEL_RCCL && nranks > 1) {
        ncclUniqueId u[2];
        std::memcpy(u, id, sizeof u);
        for (int c = 0; c < 2 && !rc; ++c) {
            ncclResult_t r = ncclCommInitRank(&p->comm[c], nranks, u[c], rank);
            if (r != ncclSuccess) rc = nccl_fail(r, "ncclCommInitRank");
        }
    }
    if (rc) {
        nw_panel_destroy(p);
        return rc;
    }
    *out = p;
    return NW_OK;
}

int nw_panel_ipc_handle(nw_panel* p, uint8_t handle[NW_PANEL_IPC_BYTES]) {
    if (!p || !handle || p->transport != NW_PANEL_IPC) return fail(NW_ERR_ARG, "nw_panel_ipc_handle: bad arguments");
    static_assert(sizeof(hipIpcMemHandle_t) == NW_PANEL_IPC_BYTES, "IPC handle size");
    NW_HIPCHK(hipSetDevice(p->device));
    hipIpcMemHandle_t h;
    NW_HIPCHK(hipIpcGetMemHandle(&h, p->xin));
    std::memcpy(handle, &h, sizeof h);
    return NW_OK;
}

int nw_panel_ipc_connect(nw_panel* p, const uint8_t* handles) {
    if (!p || !handles || p->transport != NW_PANEL_IPC) return fail(NW_ERR_ARG, "nw_panel_ipc_connect: bad arguments");
    NW_HIPCHK(hipSetDevice(p->device));
    for (int r = 0; r < p->nranks; ++r) {
        if (r == p->rank || p->peer_xin[(size_t)r]) continue;
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)r * NW_PANEL_IPC_BYTES, sizeof h);
        void* q = nullptr;
        NW_HIPCHK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
        p->peer_xin[(size_t)r] = static_cast<uint64_t*>(q);
    }
    p->connected = true;
    return NW_OK;
}

int nw_panel_group_create(int n, const int* devices, int64_t max_L1, int64_t max_L2, uint32_t out_mask,
                          nw_panel** out) {
    if (n < 1 || !devices || !out || max_L1 < 0 || max_L2 < 0)
        return fail(NW_ERR_ARG, "nw_panel_group_create: bad arguments");
    std::vector<nw_panel*> ps((size_t)n, nullptr);
    int rc = NW_OK;
    for (int r = 0; r < n && !rc; ++r) {
        nw_panel* p = new nw_panel;
        ps[(size_t)r] = p;
        p->transport = NW_PANEL_GROUP;
        p->rank = r;
        p->nranks = n;
        p->device = devices[r] < 0 ? 0 : devices[r];
        rc = panel_alloc(p, max_L1, max_L2, out_mask);
    }
    // producers store into their successor's xin: peer access between GPUs
    for (int r = 0; r + 1 < n && !rc; ++r) {
        const int a = ps[(size_t)r]->device, b = ps[(size_t)r + 1]->device;
        if (a == b) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
            rc = fail(NW_ERR_NODEVICE, "nw_panel_group_create: no peer access between devices");
            break;
        }
        (void)hipSetDevice(a);
        hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            rc = fail(NW_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
        (void)hipGetLastError();
    }
    for (nw_panel* p : ps)
        if (p) p->group = ps;
    if (rc) {
        for (nw_panel* p : ps) nw_panel_destroy(p);
        return rc;
    }
    for (int r = 0; r < n; ++r) out[r] = ps[(size_t)r];
    return NW_OK;
}

int nw_panel_set_sequences(nw_panel* p, const char* s1, int64_t L1, const char* s2, int64_t L2) {
    if (!p || L1 < 0 || L2 < 0 || L1 > p->max_L1 || L2 > p->max_L2 || (L1 && !s1) || (L2 && !s2))
        return fail(NW_ERR_ARG, "nw_panel_set_sequences: bad arguments");
    int64_t base = 0, rows = 0;
    int rc = nw_panel_partition(L2, p->nranks, p->rank, &base, &rows);
    if (!rc) rc = nw_panel_chain(L2, p->nranks, p->rank, &p->prev, &p->next, &p->pos);
    if (!rc) rc = nw_table_set_sequences(p->t, s1, L1, rows ? s2 + base : s2, rows);
    if (rc) return rc;
    p->t->row_base = base;
    p->t->L2_total = L2;
    p->L1 = L1;
    p->L2 = L2;
    p->row_base = base;
    p->rows = rows;
    p->have_seq = true;
    p->filled = false;
    return NW_OK;
}

int nw_panel_proxy_run(int64_t L1, int64_t xblk, int has_prev, int has_next, int launched,
                       const nw_panel_proxy_ops* ops) {
    if (!ops || L1 < 0 || xblk < 1 || (has_prev && !ops->recv) ||
        (has_next && (!ops->flag || !ops->send || !ops->poison)))
        return fail(NW_ERR_ARG, "nw_panel_proxy_run: bad arguments");
    const int64_t NB = L1 > 0 ? cdiv(cdiv(L1, kChunk), xblk) : 0;
    auto blk = [&](int64_t b, int64_t* off, int64_t* cnt) {
        *off = b * xblk * kChunk;
        *cnt = std::min<int64_t>(xblk * kChunk, L1 - *off);
    };
    // 1. every receive before anything is waited for
    for (int64_t b = 0; has_prev && b < NB; ++b) {
        int64_t off, cnt;
        blk(b, &off, &cnt);
        const int rc = ops->recv(ops->ctx, off, cnt);
        if (rc) return rc;
    }
    // 2. the row below, block by block
    int rc = NW_OK;
    bool broken = !launched;
    for (int64_t b = 0; has_next && b < NB; ++b) {
        int64_t off, cnt;
        blk(b, &off, &cnt);
        for (uint64_t spin = 0; !broken; ++spin) {
            const int f = ops->flag(ops->ctx, b, spin);
            if (f > 0) break;
            if (f < 0) broken = true;   // the kernel ended without this block
        }
        if (broken) {
            const int prc = ops->poison(ops->ctx, off, cnt);
            if (prc && !rc) rc = prc;
        }
        const int src = ops->send(ops->ctx, off, cnt);
        if (src) return src;
        if (rc) return rc;
    }
    return rc;
}

int nw_panel_fill(nw_panel* p, int32_t m, int32_t k, int32_t d, uint32_t out_mask) {
    if (!p) return fail(NW_ERR_ARG, "nw_panel_fill: NULL panel");
    if (p->transport == NW_PANEL_GROUP) return fail(NW_ERR_ARG, "nw_panel_fill: group panels use nw_panel_group_fill");
    if (!p->have_seq) return fail(NW_ERR_STATE, "nw_panel_fill: no sequences set");
    if (p->transport == NW_PANEL_IPC && p->nranks > 1 && !p->connected)
        return fail(NW_ERR_STATE, "nw_panel_fill: IPC panel not connected");
    if (p->transport == NW_PANEL_RCCL && p->nranks > 1 && !p->comm[0])
        return fail(NW_ERR_STATE, "nw_panel_fill: RCCL panel has no communicator");
    const double t0 = now_ms();
    NW_HIPCHK(hipSetDevice(p->device));
    const uint32_t prev_epoch = p->epoch;
    p->epoch = next_epoch(p->epoch);
    const uint32_t epoch = p->epoch;
    p->filled = false;
    p->have_global = false;
    p->last_d = d;
    configure(p, epoch, prev_epoch);
    nw_table* t = p->t;
    int rc = NW_OK;
    bool launched = false;
    if (p->rows > 0) {
        rc = nwi::fill_launch(t, m, k, d, out_mask);
        launched = rc == NW_OK;
    }
    if (rc == NW_OK) rc = post_credit(p, launched && t->xin);
    else (void)post_credit(p, false, true);
    const int64_t NC = cdiv(p->L1, kChunk);
    const int64_t NB = (p->rows > 0 && p->L1 > 0) ? cdiv(NC, p->xblk) : 0;
    int xrc = NW_OK;   // transport failure (reported after the local fill)
    if (p->transport == NW_PANEL_RCCL && NB > 0) {
        RcclProxy px{p, t, epoch};
        const nw_panel_proxy_ops ops{&px, RcclProxy::recv, RcclProxy::flag, RcclProxy::poison, RcclProxy::send};
        xrc = nw_panel_proxy_run(p->L1, p->xblk, p->prev >= 0, p->next >= 0, launched, &ops);
    }
    if (launched) {
        rc = nwi::fill_finish(t);
        if (rc != NW_OK) (void)post_credit(p, false, true);   // whatever the kernel got to
    }
    if (p->transport == NW_PANEL_IPC && rc != NW_OK && p->next >= 0 && p->rows > 0 && p->L1 > 0) {
        // we owe the panel below a row we could not produce
        const int prc = nwi::poison(p->peer_xin[(size_t)p->next], p->L1, epoch, p->s_send);
        if (!prc) (void)hipStreamSynchronize(p->s_send);
    }
    if (p->s_recv) {
        hipError_t e = hipStreamSynchronize(p->s_recv);
        if (e != hipSuccess && !xrc) xrc = fail(NW_ERR_HIP, std::string("recv stream: ") + hipGetErrorString(e));
    }
    {
        hipError_t e = hipStreamSynchronize(p->s_send);
        if (e != hipSuccess && !xrc) xrc = fail(NW_ERR_HIP, std::string("send stream: ") + hipGetErrorString(e));
    }
    if (rc == NW_OK) rc = xrc;
    p->last_rc = rc;
    p->filled = true;
    p->call_ms = (float)(now_ms() - t0);
    return rc;
}

int nw_panel_group_fill(nw_panel* const* ps, int n, int32_t m, int32_t k, int32_t d, uint32_t out_mask) {
    if (!ps || n < 1) return fail(NW_ERR_ARG, "nw_panel_group_fill: bad arguments");
    for (int r = 0; r < n; ++r) {
        const nw_panel* p = ps[r];
        if (!p || p->transport != NW_PANEL_GROUP || p->rank != r || p->nranks != n || p->group.size() != (size_t)n ||
            p->group[(size_t)r] != p)
            return fail(NW_ERR_ARG, "nw_panel_group_fill: panels must be one whole group in rank order");
        for (const nw_panel* q : p->group)
            if (!q) return fail(NW_ERR_STATE, "nw_panel_group_fill: a group member was destroyed");
        if (!p->have_seq) return fail(NW_ERR_STATE, "nw_panel_group_fill: no sequences set");
    }
    const double t0 = now_ms();
    const uint32_t prev_epoch = ps[0]->epoch;
    const uint32_t epoch = next_epoch(prev_epoch);
    for (int r = 0; r < n; ++r) {
        nw_panel* p = ps[r];
        p->epoch = epoch;
        p->filled = false;
        p->have_global = false;
        p->last_d = d;
        configure(p, epoch, prev_epoch);
    }
    // Launch top-down (a panel only ever waits on panels launched before it),
    // then complete top-down, poisoning the row a failed panel owes.
    std::vector<int> rcs((size_t)n, NW_OK);
    std::vector<char> launched((size_t)n, 0);
    bool stop = false;
    for (int r = 0; r < n; ++r) {
        nw_panel* p = ps[r];
        if (stop) {
            rcs[(size_t)r] = NW_ERR_PEER;
            (void)post_credit(p, false, true);
            continue;
        }
        if (p->rows > 0) {
            rcs[(size_t)r] = nwi::fill_launch(p->t, m, k, d, out_mask);
            launched[(size_t)r] = rcs[(size_t)r] == NW_OK;
            if (!launched[(size_t)r]) stop = true;
        }
        if (rcs[(size_t)r] == NW_OK) rcs[(size_t)r] = post_credit(p, launched[(size_t)r] && p->t->xin);
        else (void)post_credit(p, false, true);
    }
    for (int r = 0; r < n; ++r) {
        nw_panel* p = ps[r];
        if (launched[(size_t)r]) {
            rcs[(size_t)r] = nwi::fill_finish(p->t);
            if (rcs[(size_t)r] != NW_OK) (void)post_credit(p, false, true);
        }
        if (rcs[(size_t)r] != NW_OK && p->next >= 0 && launched[(size_t)p->next] && p->L1 > 0) {
            nw_panel* q = ps[p->next];
            (void)hipSetDevice(q->device);
            if (nwi::poison(q->xin, p->L1, epoch, q->s_send) == NW_OK) (void)hipStreamSynchronize(q->s_send);
        }
    }
    std::vector<int64_t> recs((size_t)n * NW_PANEL_REC);
    for (int r = 0; r < n; ++r) {
        ps[r]->last_rc = rcs[(size_t)r];
        ps[r]->filled = true;
        make_record(ps[r], &recs[(size_t)r * NW_PANEL_REC]);
    }
    nw_stats st{};
    const int rc = nw_panel_reduce(recs.data(), n, &st);
    const float ms = (float)(now_ms() - t0);
    for (int r = 0; r < n; ++r) {
        ps[r]->stats = st;
        ps[r]->have_global = rc == NW_OK;
        ps[r]->call_ms = ms;
    }
    return rc;   // nw_last_error() keeps the failing panel's detail
}

int nw_panel_record(nw_panel* p, int64_t rec[NW_PANEL_REC]) {
    if (!p || !rec) return fail(NW_ERR_ARG, "nw_panel_record: bad arguments");
    if (!p->filled) return fail(NW_ERR_STATE, "nw_panel_record: no fill");
    make_record(p, rec);
    return NW_OK;
}

int nw_panel_reduce(const int64_t* recs, int nranks, nw_stats* st) {
    if (!recs || nranks < 1 || !st) return fail(NW_ERR_ARG, "nw_panel_reduce: bad arguments");
    std::vector<int> rcs;
    nw_stats s{};
    s.corner = (int32_t)recs[5];
    int32_t gav = 0;
    uint32_t bc = 0;
    for (int r = 0; r < nranks; ++r) {
        const int64_t* x = recs + (size_t)r * NW_PANEL_REC;
        rcs.push_back((int)x[0]);
        if (x[1]) s.corner = (int32_t)x[2];
        gav = std::max(gav, (int32_t)x[3]);
        bc += (uint32_t)x[4];
    }
    s.greatest_abs_interior = gav;
    s.branch_count = bc;
    *st = s;
    return first_error(rcs);
}

int nw_panel_stats(nw_panel* p, nw_stats* st) {
    if (!p || !st) return fail(NW_ERR_ARG, "nw_panel_stats: bad arguments");
    if (!p->filled) return fail(NW_ERR_STATE, "nw_panel_stats: no fill");
    if (p->transport != NW_PANEL_GROUP && p->nranks == 1) {
        if (p->last_rc) return fail(p->last_rc, "nw_panel_stats: last fill failed");
        int64_t rec[NW_PANEL_REC];
        make_record(p, rec);
        return nw_panel_reduce(rec, 1, st);
    }
    if (!p->have_global)
        return fail(NW_ERR_STATE, p->transport == NW_PANEL_GROUP
                                      ? "nw_panel_stats: last group fill failed"
                                      : "nw_panel_stats: gather nw_panel_record()s and use nw_panel_reduce()");
    *st = p->stats;
    return NW_OK;
}

int nw_panel_hash_columns(nw_panel* p, uint64_t* hstate, uint64_t* dstate) {
    if (!p || !hstate || !dstate) return fail(NW_ERR_ARG, "nw_panel_hash_columns: bad arguments");
    if (!p->filled || p->last_rc != NW_OK) return fail(NW_ERR_STATE, "nw_panel_hash_columns: no completed fill");
    if (p->rows == 0) return NW_OK;   // no rows of its own
    // the first panel hashes global row 0 (the seed) too; the others start at their first own row
    return nw_table_hash_columns(p->t, p->row_base == 0 ? 0 : 1, hstate, dstate);
}

int nw_panel_credit_reached(uint32_t credit, uint32_t want) { return nwk::epoch_reached(credit, want) ? 1 : 0; }

int nw_panel_rows(const nw_panel* p, int64_t* row_base, int64_t* rows) {
    if (!p || !row_base || !rows) return fail(NW_ERR_ARG, "nw_panel_rows: bad arguments");
    if (!p->have_seq) return fail(NW_ERR_STATE, "nw_panel_rows: no sequences set");
    *row_base = p->row_base;
    *rows = p->rows;
    return NW_OK;
}

nw_table* nw_panel_table(nw_panel* p) { return p ? p->t : nullptr; }

int nw_panel_elapsed_ms(nw_panel* p, float* kernel_ms, float* call_ms) {
    if (!p) return fail(NW_ERR_ARG, "nw_panel_elapsed_ms: NULL panel");
    if (!p->filled) return fail(NW_ERR_STATE, "nw_panel_elapsed_ms: no fill");
    if (kernel_ms) *kernel_ms = p->t->filled ? p->t->kernel_ms : 0.f;
    if (call_ms) *call_ms = p->call_ms;
    return NW_OK;
}

}  // extern "C"
