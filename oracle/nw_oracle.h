/*
 * nw_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the reference's DP fill, used as the parity
 * checker in tests/, by __graft_entry__.smoke() and as bench.py's
 * cpu_baseline ("port") leg.  The product (libnwfill.so, the CLI) never links
 * or calls it.  Pinned against the compiled reference (oracle/_ref) through
 * tests/golden/ref_kats.json.
 *
 * Conventions (shared with include/nw_fill.h):
 *   L1 = strlen(s1) (top string, columns i), L2 = strlen(s2) (side string,
 *   rows j); table cells (i, j), 0 <= i <= L1, 0 <= j <= L2, "i-major" order
 *   index i*(L2+1)+j -- the reference's cells[col][row] order
 *   (score-table.c:71-78).
 *   Direction code per cell: bit0 = diag, bit1 = up, bit2 = left
 *   (walk-table.h:44-54 flags).
 */
#ifndef NW_ORACLE_H
#define NW_ORACLE_H
#include <stdint.h>

typedef struct {
        int32_t  corner;                 /* H[L1][L2]                       */
        int32_t  greatest_abs_interior;  /* max |H| over i>=1, j>=1, else 0 */
        uint32_t branch_count;           /* interior cells with >=2 dirs    */
} nwo_stats;

/* splitmix64 DNA generator: seed 1 -> s1, seed 2 -> s2. */
void nwo_gen_dna(uint64_t seed, int64_t n, char *out);

/* FNV-1a-64 over a byte range, continuing from h. */
uint64_t nwo_fnv1a(uint64_t h, const void *p, int64_t n);
#define NWO_FNV_INIT 0xcbf29ce484222325ULL

/* Full fill: H (L1+1)*(L2+1) int32, D one code byte per cell (either may
 * be NULL).  Returns 0. */
int nwo_fill(const char *s1, int64_t L1, const char *s2, int64_t L2,
             int32_t m, int32_t k, int32_t d,
             int32_t *H, uint8_t *D, nwo_stats *st);

/* Row band (multi-GPU panel) given the row above it, top[0..L1]; H is
 * (L1+1)*(rows+1) with local row 0 = top, D codes (row 0: 0), stats over the
 * band's interior.  s2 = the band's side-string bytes. */
int nwo_fill_band(const char *s1, int64_t L1, const char *s2, int64_t rows, int64_t row_base,
                  const int32_t *top, int32_t m, int32_t k, int32_t d,
                  int32_t *H, uint8_t *D, nwo_stats *st);

/* Streaming fill in O(L2) memory: FNV-1a-64 of the score table (int32 LE)
 * and of the code bytes, in i-major order, plus the stats. */
int nwo_fill_hash(const char *s1, int64_t L1, const char *s2, int64_t L2,
                  int32_t m, int32_t k, int32_t d,
                  uint64_t *hH, uint64_t *hD, nwo_stats *st);

/* Streaming fill, column-chained hashes (the device-side parity hash of
 * include/nw_fill.h nw_table_hash): per column i, FNV-1a-64 of the int32 LE
 * scores H[i][0..L2] (resp. of the code bytes); hH2/hD2 = FNV-1a-64 over those
 * per-column hashes as 8-byte LE words, i = 0..L1. */
int nwo_fill_colchain(const char *s1, int64_t L1, const char *s2, int64_t L2,
                      int32_t m, int32_t k, int32_t d,
                      uint64_t *hH2, uint64_t *hD2, nwo_stats *st);

/* Score-only: returns H[L1][L2]; *hlast (nullable) = FNV of the last column
 * H[L1][0..L2]. */
int32_t nwo_score_only(const char *s1, int64_t L1, const char *s2, int64_t L2,
                       int32_t m, int32_t k, int32_t d, uint64_t *hlast);

/* Score-only on nthreads row bands (a band wavefront, O(L1 + L2) memory):
 * same results as nwo_score_only, for the sizes a single core cannot reach
 * (the 1M x 1M pin, tests/golden/make_big_scoreonly.py). */
int32_t nwo_score_only_mt(const char *s1, int64_t L1, const char *s2, int64_t L2,
                          int32_t m, int32_t k, int32_t d, int nthreads, uint64_t *hlast);

/* Blocked anti-diagonal multi-threaded full fill (CPU baseline, same output
 * as nwo_fill; D may be NULL, stats may be NULL). */
int nwo_fill_mt(const char *s1, int64_t L1, const char *s2, int64_t L2,
                int32_t m, int32_t k, int32_t d,
                int32_t *H, uint8_t *D, nwo_stats *st, int nthreads);

/* Walk services over a filled code table D (one byte per cell, i-major).
 * nwo_count_paths: the reference's optimal-alignment count (a uint32 that
 * wraps like its `unsigned` counter).  nwo_first_path: the first alignment the
 * reference prints, as moves in forward order (1 diag, 2 up, 4 left);
 * returns the move count (<= L1+L2) or -1. */
uint32_t nwo_count_paths(const uint8_t *D, int64_t L1, int64_t L2);
int64_t nwo_first_path(const uint8_t *D, int64_t L1, int64_t L2, uint8_t *moves);

#endif
