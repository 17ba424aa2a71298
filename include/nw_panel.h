/* nw_panel.h -- multi-GPU row panels for the MI355X score-table fill.
 *
 * The reference fills one table in one process; its only parallelism is the
 * pthread column-cyclic schedule of `-p` (needleman-wunsch.c:444-475,
 * :557-574, :583-626), where thread t owns columns t+1, t+1+T, ... and waits
 * per cell for its left neighbour.  Across GPUs the table is split instead into
 * contiguous ROW panels: panel r holds global rows row_base+1 .. row_base+rows
 * (whole 128-row stripes; every panel but the last has a multiple of 128 rows,
 * so every feeding panel can run the two-rows-per-lane kernel)
 * for all columns.  This is the column-panel scheme
 * transposed to this fill's stripe orientation (waves sweep columns): the
 * exchange is the single boundary ROW, in blocks of columns, and a panel
 * starts as soon as the first block of the row above it is done.
 *
 * Each panel's kernel publishes its bottom row as tagged 8-byte granules
 * {epoch, H - d}; the panel below polls the tags, so no barrier or host
 * round trip sits between producer and consumer.  Two transports move the
 * granules (enum nw_panel_transport):
 *   - GROUP / IPC: the producer's kernel stores straight into the consumer's
 *     boundary buffer (same GPU, or a peer GPU over xGMI; across processes
 *     the buffer is mapped with hipIpcOpenMemHandle), no host involvement.
 *   - RCCL: a host proxy waits for the producer's per-block flag (pinned host
 *     memory) and issues ncclSend; the consumer posts its ncclRecvs up front.
 *     Two communicators, so a rank's send and receive links never share one.
 * A failed panel poisons the row it owes (tag = epoch | 2^31) so the panels
 * below stop with NW_ERR_PEER instead of waiting for the watchdog.
 *
 * Back-pressure (GROUP / IPC): ranks call nw_panel_fill with no barrier, so a
 * producer may start fill E+1 while the panel below still reads fill E's row.
 * The consumer's loader copies the row above into its own table (row0) as it
 * reads it, then posts E into a credit word behind its boundary buffer; the
 * producer's first boundary store of fill E+1 waits (in its kernel) until that
 * word reads E.  Every panel posts for every fill, so the chain never waits on
 * a panel with nothing to read.  RCCL needs no credit: a send completes only
 * into a posted receive, and receives are posted per fill.
 *
 * RCCL transport: EXPERIMENTAL.  It relies on RCCL's copy kernels writing
 * each aligned 8-byte {epoch, value} granule untorn (they move >= 16-byte
 * aligned vectors), which the consumer's tag poll assumes; it has not been
 * run on more than one GPU (RCCL refuses two ranks on one device).
 *
 * Stats of the whole table are bit-identical to a single-GPU fill: corner
 * from the last panel, max of greatest_abs_interior, sum of branch_count.  The local rows stay device-resident in the panel's
 * nw_table (nw_panel_table), local row j = global row row_base + j; its row
 * 0 is the last row of the panel above (scores exact, codes read as 0).
 */
#ifndef NW_PANEL_H
#define NW_PANEL_H

#include <stdint.h>

#include "nw_fill.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nw_panel nw_panel;

/* How a panel's bottom row reaches the panel below. */
enum nw_panel_transport {
        NW_PANEL_GROUP = 0,  /* one process, n panels: direct device stores        */
        NW_PANEL_IPC   = 1,  /* one process per GPU: direct stores into the peer's  */
                             /* boundary buffer, mapped with hipIpc (xGMI)          */
        NW_PANEL_RCCL  = 2   /* one process per GPU: host proxy + ncclSend/ncclRecv */
};

#define NW_PANEL_ID_BYTES  256  /* RCCL rendezvous: two ncclUniqueId           */
#define NW_PANEL_IPC_BYTES 64   /* hipIpcMemHandle_t of a boundary buffer      */
#define NW_PANEL_REC       8    /* int64 words of one rank's stats record      */

/* Row split of an L2-row table over nranks panels: whole 128-row stripes,
 * balanced to within one stripe.  Pure host logic (no device needed). */
int nw_panel_partition(int64_t L2, int nranks, int rank, int64_t *row_base, int64_t *rows);

/* Panels that exchange boundary rows (empty panels are skipped): the rank
 * above (*prev) and below (*next) `rank`, -1 when none, and its position in
 * that chain (-1 for an empty panel).  Pure host logic. */
int nw_panel_chain(int64_t L2, int nranks, int rank, int *prev, int *next, int *pos);

/* The RCCL transport's host proxy as pure host logic (no device needed), so
 * its sequencing is testable anywhere.  One fill's boundary row of L1
 * granules moves in blocks of xblk chunks (8 columns each; block b covers
 * granules [b*8*xblk, min(L1, (b+1)*8*xblk))).  The proxy
 *   1. posts every receive of the row above first (has_prev), so the panel
 *      above never blocks on this one;
 *   2. then (has_next), block by block in order, polls the producer kernel's
 *      flag for the block and sends it; once the kernel has ended without the
 *      block (flag() < 0, or launched == 0) it poisons that block and every
 *      later one (tag = epoch | 2^31, see above) and still sends them, so the
 *      panel below fails with NW_ERR_PEER instead of timing out.
 * It stops at the first failing recv / send callback and returns its code
 * (a poison failure is returned after that block is sent).  The callbacks:
 *   recv(ctx, off, cnt), send(ctx, off, cnt), poison(ctx, off, cnt):
 *        0 on success, an nw_err code otherwise;
 *   flag(ctx, b, spin): 1 = block b is ready, 0 = not yet (called again with
 *        spin + 1), -1 = the producer kernel ended without it.
 * The RCCL transport's callbacks are ncclRecv / ncclSend on the panel's two
 * communicators, the pinned per-block flag words and a poison kernel.  This
 * is the role of the reference's per-cell wait on the left neighbour
 * (needleman-wunsch.c:444-475), moved to one boundary row per panel. */
typedef struct {
        void *ctx;
        int (*recv)(void *ctx, int64_t off, int64_t cnt);
        int (*flag)(void *ctx, int64_t b, uint64_t spin);
        int (*poison)(void *ctx, int64_t off, int64_t cnt);
        int (*send)(void *ctx, int64_t off, int64_t cnt);
} nw_panel_proxy_ops;
int nw_panel_proxy_run(int64_t L1, int64_t xblk, int has_prev, int has_next, int launched,
                       const nw_panel_proxy_ops *ops);

/* RCCL only, rank 0: create the rendezvous id; the caller broadcasts it. */
int nw_panel_get_id(uint8_t id[NW_PANEL_ID_BYTES]);

/* One process per GPU (transport IPC or RCCL).  For RCCL this is collective
 * over the nranks processes and `id` is rank 0's nw_panel_get_id(); for IPC
 * `id` is ignored and the ranks then swap nw_panel_ipc_handle()s and call
 * nw_panel_ipc_connect().  max_L2 is the GLOBAL row capacity. */
int nw_panel_create(int transport, int device, int rank, int nranks, const uint8_t *id,
                    int64_t max_L1, int64_t max_L2, uint32_t out_mask, nw_panel **out);
int nw_panel_ipc_handle(nw_panel *p, uint8_t handle[NW_PANEL_IPC_BYTES]);
/* handles: every rank's handle, in rank order (nranks * NW_PANEL_IPC_BYTES). */
int nw_panel_ipc_connect(nw_panel *p, const uint8_t *handles);

/* In-process group of n panels on devices[0..n-1] (repeats allowed, e.g. n
 * panels on one GPU; distinct GPUs get peer access).  out[0..n-1]. */
int nw_panel_group_create(int n, const int *devices, int64_t max_L1, int64_t max_L2, uint32_t out_mask,
                          nw_panel **out);

void nw_panel_destroy(nw_panel *p);   /* group panels: destroy each one */

/* Full sequences (same on every rank); the panel uploads its own rows. */
int nw_panel_set_sequences(nw_panel *p, const char *s1, int64_t L1, const char *s2, int64_t L2);

/* IPC / RCCL: every rank calls it once per fill, same arguments.  Returns
 * this rank's status; a failure upstream surfaces as NW_ERR_PEER. */
int nw_panel_fill(nw_panel *p, int32_t m, int32_t k, int32_t d, uint32_t out_mask);

/* Back-pressure of the IPC / group transports.  A panel that receives a row
 * posts "read" into a credit word (the fill's epoch) and the panel above
 * waits for it before it overwrites that row in its next fill.  The credit
 * is posted on every path -- by the kernel once it has read the row, by the
 * host when the fill failed or never launched -- and the wait accepts the
 * awaited epoch or any later one, so a failed panel costs the panel above no
 * watchdog time-out on the next fill.  nw_panel_credit_reached is that
 * comparison (epochs run 1 .. 2^31-1 and wrap to 1): 1 when `credit` is at
 * or after `want`. */
int nw_panel_credit_reached(uint32_t credit, uint32_t want);

/* In-process group: fills all n panels of the group, in rank order. */
int nw_panel_group_fill(nw_panel *const *ps, int n, int32_t m, int32_t k, int32_t d, uint32_t out_mask);

/* Whole-table stats.  A group computes them itself (nw_panel_stats on any of
 * its panels).  Across processes the caller gathers every rank's record
 * (nw_panel_record, after the fill) and reduces them with nw_panel_reduce --
 * a few words of control traffic, left to the caller's own collective. */
int nw_panel_stats(nw_panel *p, nw_stats *st);
int nw_panel_record(nw_panel *p, int64_t rec[NW_PANEL_REC]);
int nw_panel_reduce(const int64_t *recs, int nranks, nw_stats *st);   /* pure; first error wins */

/* Whole-table parity hashes across panels: continue the per-column FNV
 * states (host, L1+1 each, in place; start at 0xcbf29ce484222325) over this
 * panel's own rows.  Called on every panel in rank order (any transport; the
 * states travel with the caller), nw_hash_fold() of the result is the
 * single-GPU nw_table_hash(). */
int nw_panel_hash_columns(nw_panel *p, uint64_t *hstate, uint64_t *dstate);

/* This panel's rows and its device-resident table (owned by the panel). */
int nw_panel_rows(const nw_panel *p, int64_t *row_base, int64_t *rows);
nw_table *nw_panel_table(nw_panel *p);

/* Milliseconds of the last fill: this panel's kernel (HIP events) and the
 * whole nw_panel_fill call on the host clock. */
int nw_panel_elapsed_ms(nw_panel *p, float *kernel_ms, float *call_ms);

#ifdef __cplusplus
}
#endif

#endif /* NW_PANEL_H */
