/*
 * nw_fill.h -- C ABI of the MI355X-native Needleman-Wunsch score-table fill.
 *
 * This is the drop-in seam for the reference's hot path:
 *
 *     void compute_table_scores(computation_t *C);   needleman-wunsch.c:583-626
 *
 * called once by the driver at needleman-wunsch.c:662, after the tables were
 * allocated (score-table.c:60-81, walk-table.c:58-79) and seeded
 * (computation.c:75-125).  Allocation, seeding and the fill all move to the
 * GPU behind these entry points; the host keeps the CLI, the reader
 * (read-sequences.c), the traceback (needleman-wunsch.c:209-331) and the
 * printer (print-table.c), fed from the outputs below.
 *
 * Conventions
 *   s1 = top string (reference C->top_string), L1 = strlen(s1): columns i.
 *   s2 = side string (C->side_string),         L2 = strlen(s2): rows j.
 *   Cells (i, j), 0 <= i <= L1, 0 <= j <= L2; "i-major" linear index
 *   c = i*(L2+1) + j, the reference's cells[col][row] order
 *   (score-table.c:71-78).
 *   m, k, d = match bonus, mismatch penalty, indel penalty (int operands,
 *   needleman-wunsch.c:783-785).  All arithmetic is int32, as in the
 *   reference; inputs whose scores could overflow int32 are rejected with
 *   NW_ERR_RANGE (the reference's behaviour there is undefined).
 *   Direction code of a cell: bit0 = diag, bit1 = up, bit2 = left, set for
 *   every candidate equal to the cell's score (needleman-wunsch.c:485-503);
 *   boundary cells: (0,0) = 0, (i,0) = left, (0,j) = up (computation.c:93-120).
 *
 * Errors: every entry point returns 0 (NW_OK) or a negative nw_err code and
 * never exit()s (the reference's check() -> exit(1), dbg.h:96-100, moves to
 * the caller).  nw_strerror() gives the message; nw_last_error() the detail
 * of the most recent failure on the calling thread.
 *
 * Threading: calls on one nw_table must not overlap; distinct tables may be
 * used from distinct threads.  Everything is synchronous unless stated.
 */
#ifndef NW_FILL_H
#define NW_FILL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nw_stats {
        int32_t  corner;                 /* H[L1][L2] (computation.c:279-280)     */
        int32_t  greatest_abs_interior;  /* max |H| over i,j >= 1; 0 if none      */
                                         /* (needleman-wunsch.c:538-541)          */
        uint32_t branch_count;           /* interior cells with >= 2 directions,  */
                                         /* wraps like walk-table.c:108-120       */
} nw_stats;

enum nw_out {
        NW_OUT_SCORES = 1u,  /* write the int32 score table                */
        NW_OUT_DIRS   = 2u,  /* write the packed direction codes           */
        NW_OUT_STATS  = 4u   /* compute greatest_abs_interior/branch_count */
};

enum nw_err {
        NW_OK            = 0,
        NW_ERR_ARG       = -1,  /* bad argument (NULL, negative length, ...)   */
        NW_ERR_NODEVICE  = -2,  /* no usable gfx950 device                     */
        NW_ERR_OOM       = -3,  /* device or host allocation failed            */
        NW_ERR_HIP       = -4,  /* a HIP runtime call failed                   */
        NW_ERR_RANGE     = -5,  /* int32 overflow possible for these inputs    */
        NW_ERR_TIMEOUT   = -6,  /* in-kernel hand-off watchdog fired           */
        NW_ERR_STATE     = -7,  /* call out of order (e.g. no sequences set)   */
        NW_ERR_PEER      = -8   /* a peer panel failed (nw_panel.h)            */
};

const char *nw_strerror(int rc);
const char *nw_last_error(void);

/* ---------------------------------------------------------------------------
 * One-shot fill into host buffers (the direct compute_table_scores analogue).
 *
 * H    : NULL or (L1+1)*(L2+1) int32, i-major (cells[i][j] at i*(L2+1)+j).
 * dirs : NULL or ceil((L1+1)*(L2+1)/2) bytes; cell c's code is the low nibble
 *        of dirs[c/2] when c is even, the high nibble when c is odd.
 * stats: NULL or filled; greatest_abs_interior / branch_count are computed
 *        only when out_mask has NW_OUT_STATS (else 0).
 * device: HIP device ordinal (-1: $NW_DEVICE or 0).
 */
int nw_fill(const char *s1, int64_t L1, const char *s2, int64_t L2,
            int32_t m, int32_t k, int32_t d, uint32_t out_mask, int device,
            int32_t *H, uint8_t *dirs, nw_stats *stats);

/* ---------------------------------------------------------------------------
 * Device-resident table (the 100k x 100k path: the 45 GB table stays in HBM).
 *
 * Device layout (for zero-copy consumers; everyone else uses the copy, hash
 * and walk entry points below, which decode it).  Which variant a fill left
 * in the table is reported by nw_table_layout(); the four fill kernels
 * (column scan, skewed stripes, two rows per lane, skewed 16-row groups --
 * chosen per shape, or by $NW_KERNEL) share the tiling and differ in how a
 * cell's row r = j - 1 and column q = i - 1 map into it:
 *   rr = pair ? 64*(2*(r/128) + r%2) + (r%128)/2 : r     (two rows per lane)
 *   t  = skew == 1 ? q + rr%64                           (stored by step)
 *      : skew == 2 ? q + (rr%64)/16                      (16-row groups one step apart)
 *      : q
 *   scores: stripe quad tiles.  Row 0 and column 0 (the seeds -i*d, -j*d) are
 *           not stored.  Interior cell (i, j) is element
 *             (rr/64)*P + ((t/4)*64 + rr%64)*4 + t%4,
 *           P = nw_table_score_pitch() = 512*NQ: a lane's 4 consecutive
 *           columns are 16 contiguous bytes, 8 columns of a stripe 2 KB.
 *   dirs  : 32-bit words, one per (64-row stripe g = rr/64, 8-column group,
 *           lane l = rr%64): word (g*(NQ+1) + t/8 + 1)*64 + l (row 0 of each
 *           stripe is padding) holds 8 codes of 3 bits, code of t%8 = s in bits
 *           [21-3s, 23-3s] (bits 24..31 are 0).
 *           NQ = 8-column groups per stripe of the layout (nw_layout.NQ).
 *   raw scores.  A fill with NW_OUT_SCORES and without NW_OUT_STATS that the
 *           two-rows-per-lane kernel ran (nw_layout.raw = 1; the 100k x 100k
 *           default) leaves the kernel's own shifted values in the tiles,
 *             G' = H + rw*d + (i - base)*d   (mod 2^32),
 *           rw = the row's offset inside its workgroup stripe, base = the
 *           first column of the cell's 4096-column group:
 *             g  = r/128;  big = SR*(SQ+1)
 *             s  = g < big ? g/(SQ+1) : SR + (g - big)/SQ
 *             rw = r - 128*(s*SQ + min(s, SR));  base = ((i-1)/4096)*4096
 *             H  = G' - (rw + i - base)*d
 *           with SQ, SR, d from nw_layout (the fill's stripe plan and indel
 *           penalty).  A fill with NW_OUT_SCORES that the 16-row-group kernel
 *           ran (nw_layout.raw = 2) does the same with 64-row stripes and no
 *           moving base: g = r/64, rw = r - 64*(s*SQ + min(s, SR)), base = 0,
 *           H = G' - (rw + i)*d.  Every entry point below returns H, never G'.
 */
typedef struct nw_table nw_table;

/* Allocate for sequences up to max_L1 x max_L2 with the outputs in out_mask. */
int nw_table_create(int device, int64_t max_L1, int64_t max_L2,
                    uint32_t out_mask, nw_table **out);
void nw_table_destroy(nw_table *t);

/* Upload (H2D) the two sequences; L1 <= max_L1, L2 <= max_L2. */
int nw_table_set_sequences(nw_table *t, const char *s1, int64_t L1,
                           const char *s2, int64_t L2);

/* Run the fill on the device-resident sequences.  Synchronous.
 * out_mask must be a subset of the mask given at creation; when it lacks
 * NW_OUT_SCORES the fill is score-only (only the last column H[L1][*] is
 * written).  */
int nw_table_fill(nw_table *t, int32_t m, int32_t k, int32_t d, uint32_t out_mask);

/* Results of the last fill. */
int nw_table_stats(nw_table *t, nw_stats *st);
/* Device time (ms) of the last fill kernel alone, and of the whole fill call
 * (memsets + seeding + fill), both measured with HIP events on the table's
 * stream. */
int nw_table_elapsed_ms(nw_table *t, float *fill_kernel_ms, float *fill_call_ms);
/* Column-chained FNV-1a-64 of the scores and of the direction codes
 * hH = FNV over the 8-byte LE FNV-1a-64 of each
 * column's int32 LE scores, i = 0..L1; hD likewise over one code byte per
 * cell.  Computed on the device. */
int nw_table_hash(nw_table *t, uint64_t *hH, uint64_t *hD);
/* The same hashes, split by rows: continue the per-column FNV-1a-64 states
 * hstate / dstate (host, L1+1 each, in place) over rows j0..L2 of this table.
 * A whole table: states = 0xcbf29ce484222325, j0 = 0.  Row panels
 * (nw_panel.h) chain them panel by panel (the first panel from j0 = 0, every
 * later one from its first own row, j0 = 1); nw_hash_fold() of the final
 * states is nw_table_hash()'s hH / hD of the whole table. */
int nw_table_hash_columns(nw_table *t, int64_t j0, uint64_t *hstate, uint64_t *dstate);
/* FNV-1a-64 over the 8-byte LE words state[0..n). */
uint64_t nw_hash_fold(const uint64_t *state, int64_t n);
/* Copy columns [i0, i1) of the score table to host, dense ((i1-i0)*(L2+1)). */
int nw_table_copy_scores(nw_table *t, int64_t i0, int64_t i1, int32_t *dst);
/* Copy the direction codes of columns [i0, i1) to host, one byte per cell. */
int nw_table_copy_codes(nw_table *t, int64_t i0, int64_t i1, uint8_t *dst);
/* Copy the last column H[L1][0..L2] (available in score-only mode too). */
int nw_table_copy_last_column(nw_table *t, int32_t *dst);
/* Slice copies are streamed: gather kernels fill two device staging buffers
 * while the DMA of the previous block runs.  A destination in pinned memory
 * (nw_host_alloc, or any hipHostMalloc'd / registered range) is written by
 * the DMA directly, at PCIe rate; a pageable one goes through two pinned
 * bounce buffers whose host copy overlaps the next DMA.  The reference holds
 * the whole table in host memory (score-table.c:60-81); here only the slice
 * a consumer asks for crosses PCIe.  nw_table_set_sequences likewise codes
 * the sequences into pinned staging and uploads from there (the reference
 * grows its input buffers in 4 KB steps, read-sequences.c:66-75). */
int nw_host_alloc(size_t bytes, void **p);
void nw_host_free(void *p);
/* Wall-clock ms and bytes of the last upload (nw_table_set_sequences, symbol
 * coding included) and of the last slice copy (nw_table_copy_scores /
 * nw_table_copy_codes / nw_table_copy_last_column).  Any pointer may be NULL. */
int nw_table_io_stats(nw_table *t, double *upload_ms, int64_t *upload_bytes, double *copy_ms,
                      int64_t *copy_bytes);
/* Geometry of the device layout (for zero-copy consumers): the layout
 * section above.  nw_table_layout fills *out for the last completed fill
 * (NW_ERR_STATE before one). */
typedef struct nw_layout {
        int64_t score_pitch;   /* P: int32 elements per 64-row stripe           */
        int64_t NQ;            /* 8-column groups per stripe                     */
        int32_t pair;          /* rows permuted (two-rows-per-lane kernel)       */
        int32_t skew;          /* stored by step: 1 skewed stripes, 2 16-row groups */
        int32_t raw;           /* score tiles hold G' (1 | 2), see "raw scores"   */
        int32_t SQ, SR;        /* raw: the fill's workgroup-stripe plan          */
        int32_t d;             /* raw: the fill's indel penalty                  */
        int32_t has_scores, has_dirs;
} nw_layout;
int64_t nw_table_score_pitch(const nw_table *t);
int nw_table_layout(const nw_table *t, nw_layout *out);
/* Device pointers of the score tiles and code words (NULL when not
 * allocated).  They stay valid until nw_table_destroy. */
int nw_table_device_buffers(const nw_table *t, const int32_t **scores, const uint32_t **dirs);
/* In-kernel timeline of the last fill, recorded only when $NW_TRACE is set:
 * 8 words per workgroup stripe s -- s_memrealtime (100 MHz) at [8s] dequeue,
 * [8s+1] first wave started, [8s+2] last wave finished; [8s+3] blockIdx |
 * hardware CU id << 32; s_memtime (shader clock) at [8s+4] first wave
 * started, [8s+5] last wave finished; [8s+6..7] reserved.  Copies min(n, total) words into dst (if non-NULL)
 * and returns the total word count (0 when no trace was recorded). */
int64_t nw_table_trace(nw_table *t, uint64_t *dst, int64_t n);
/* Waves per workgroup chosen for the last fill (tuning / reporting). */
int nw_table_waves(const nw_table *t);

/* ---------------------------------------------------------------------------
 * Walk services: results of the reference's traceback that do not need its
 * exponential enumeration, computed on the device from the direction codes of
 * the last fill (which must have had NW_OUT_DIRS; whole tables only, not row
 * panels).
 *
 * nw_table_count_alignments: the number of optimal alignments -- what the
 * reference's walk counts (construct_alignments, needleman-wunsch.c:356-388;
 * inc_solution_count at :250-255) and print_summary reports
 * (computation.c:271-281) -- as the reference's `unsigned` counter, i.e.
 * modulo 2^32.
 */
int nw_table_count_alignments(nw_table *t, uint32_t *count);

/* nw_table_first_path: the first alignment the reference prints -- its walk
 * tries diag, then left, then up (needleman-wunsch.c:296-322), so the first
 * arrival at (0,0) is that greedy path from the corner.  moves[0..*n) gets
 * the path in forward order ((0,0) to (L1,L2)): 1 = diag (s1[i] over s2[j]),
 * 2 = up (gap over s2[j]), 4 = left (s1[i] over a gap).  cap >= L1 + L2. */
int nw_table_first_path(nw_table *t, uint8_t *moves, int64_t cap, int64_t *n);

/* nw_table_enumerate_paths: every optimal alignment, in the order the
 * reference prints them, each computed independently on the device (the
 * reference's "parallel traceback" future work, README:195-200).  The
 * reference prints in the order of its depth-first walk, which tries diag,
 * then left, then up at every cell (needleman-wunsch.c:209-331).  With
 * C(i,j) = the number of code paths from (i,j) to (0,0) (a saturating
 * uint64 table on the device, cap 2^62), alignment k of that order is
 * unranked from the corner in O(L1 + L2): diag if k < C(diag cell), else
 * k -= C(diag cell) and try left, then up -- one thread per alignment.
 * Alignments first .. first+count-1: alignment first+p goes to
 * moves[p*stride ..] as its moves from (L1,L2) back to (0,0) -- the order the
 * reference fills its X / Y buffers -- 1 = diag, 2 = up, 4 = left, and
 * lens[p] = its length (0 past the last one).  stride >= L1 + L2.  *n (nullable)
 * = alignments written; *total (nullable) = alignments in all, saturated at
 * 2^62 (0 for two empty strings, whose walk prints nothing).  Device memory:
 * 8 bytes per cell for C, computed once per fill. */
int nw_table_enumerate_paths(nw_table *t, uint64_t first, uint64_t count, uint8_t *moves,
                             int64_t stride, int32_t *lens, uint64_t *n, uint64_t *total);

/* nw_first_path_banded: nw_table_first_path's result without the full
 * table, for pairs whose direction codes do not fit (or are not wanted) in
 * device memory: a score-only forward pass keeps one boundary row per band of
 * band_rows rows (a multiple of 64), then the bands are refilled with codes
 * bottom-up and walked greedily (needleman-wunsch.c:296-322), each only left
 * of where the walk entered it.  Device memory ~ band_rows * L1 / 2 bytes +
 * 8 * L1 per band; time ~ two fills.  Not in the reference (its traceback
 * needs every cell's walk state, walk-table.c:58-79).
 * device: as nw_fill; cap >= L1 + L2; moves as nw_table_first_path. */
int nw_first_path_banded(int device, const char *s1, int64_t L1, const char *s2, int64_t L2,
                         int32_t m, int32_t k, int32_t d, int64_t band_rows,
                         uint8_t *moves, int64_t cap, int64_t *n);
/* Device time (ms) of the last count / first-path kernel (HIP events). */
int nw_table_walk_elapsed_ms(nw_table *t, float *count_ms, float *path_ms);

/* ---------------------------------------------------------------------------
 * nw_fill_noalloc: the fill for callers that cannot allocate -- code under
 * HIP graph capture, tight serving loops, harnesses that forbid hipMalloc.
 * It has no counterpart in the reference (whose tables are calloc'd per run,
 * score-table.c:60-81); it is nw_table_fill() with every buffer either the
 * caller's or a fixed array inside the library.
 *
 * It calls no hipMalloc / hipFree / hipHostMalloc nor any other allocating
 * routine of the HIP runtime, on any path, and its success path does not
 * touch the host heap either (only an error return builds a message for
 * nw_last_error()).  It only enqueues work on `stream` (a hipStream_t, NULL
 * = the null stream): one set-up kernel, the fill kernel, one result kernel.
 * It does not wait for them; results are read from the caller's buffers
 * after the caller has synchronised with `stream`.
 *
 * The caller passes, all in DEVICE memory of `device`:
 *   s1_dev, s2_dev   the two sequences, L1 and L2 raw bytes (no padding)
 *   score_tiles_dev  NW_NOALLOC_SCORE_ELEMS(L1, L2) int32, or NULL without
 *                    NW_OUT_SCORES
 *   dir_words_dev    NW_NOALLOC_DIR_WORDS(L1, L2) uint32, or NULL without
 *                    NW_OUT_DIRS
 *   last_column_dev  NULL or L2 + 1 int32: H[L1][0..L2]
 *   result_dev       NULL or one nw_noalloc_result: status = 0 or the nw_err
 *                    the kernel hit (NW_ERR_TIMEOUT), and the stats
 *                    (greatest_abs_interior / branch_count only with
 *                    NW_OUT_STATS, else 0)
 * The tables come out in the device layout described above, always the
 * plain variant: pair = skew = raw = 0, P = 512 * ceil(L1/8).
 *
 * Everything else the fill needs (padded copies of the sequences, control
 * words, the score-only last-column staging, the hand-off rows between
 * workgroup stripes) is in one static device array of
 * NW_NOALLOC_SCRATCH_BYTES inside the library, which each GPU the library
 * runs on holds until the process ends; its size is what limits L1 and L2
 * to NW_NOALLOC_MAX_L1 / NW_NOALLOC_MAX_L2 -- beyond them the call returns
 * NW_ERR_ARG and enqueues nothing (use nw_table_fill).  All calls on one GPU
 * share that array: two calls whose work overlaps on one GPU (different
 * streams, or threads) race; calls on one stream, or otherwise ordered, are
 * fine, and each call clears what it needs at zero itself.
 * Returns 0 once the work is enqueued, or a negative nw_err (arguments,
 * NW_ERR_RANGE, a failed launch).
 */
#define NW_NOALLOC_MAX_L1 16384
#define NW_NOALLOC_MAX_L2 16384
#define NW_NOALLOC_SCRATCH_BYTES (9 * 1024 * 1024)
#define NW_NOALLOC_SCORE_ELEMS(L1, L2) \
        ((((int64_t)(L2) + 63) / 64 + 1) * (((int64_t)(L1) + 7) / 8 + 8) * 512)
#define NW_NOALLOC_DIR_WORDS(L1, L2) \
        ((((int64_t)(L2) + 63) / 64 + 1) * (((int64_t)(L1) + 7) / 8 + 9) * 64)
typedef struct nw_noalloc_result {
        int32_t  status;
        nw_stats stats;
} nw_noalloc_result;
int nw_fill_noalloc(int device, void *stream, const char *s1_dev, int64_t L1, const char *s2_dev,
                    int64_t L2, int32_t m, int32_t k, int32_t d, uint32_t out_mask,
                    int32_t *score_tiles_dev, uint32_t *dir_words_dev, int32_t *last_column_dev,
                    nw_noalloc_result *result_dev);

#ifdef __cplusplus
}
#endif
#endif /* NW_FILL_H */
