/*
 * nw_oracle.c -- TEST INFRASTRUCTURE ONLY (see nw_oracle.h).
 *
 * Clean-room restatement of the reference fill.  Each piece cites the
 * reference lines whose *behaviour* it restates:
 *
 *   seeding            computation.c:75-125  (H[0][0]=0 no dirs; H[i][0]=-i*d
 *                                             LEFT; H[0][j]=-j*d UP)
 *   cell recurrence    needleman-wunsch.c:418-510 (up/diag/left candidates,
 *                                             max3 :395-404, one flag per
 *                                             candidate equal to the max,
 *                                             branch if >1 flag :505-509)
 *   column loop + gav  needleman-wunsch.c:523-543 (|H| max over interior
 *                                             rows j>=1 of columns i>=1)
 *   column order       needleman-wunsch.c:557-574 (i = 1..L1 outer)
 *
 * Arithmetic is 32-bit two's complement with wrap-around (the reference's
 * `int` arithmetic is undefined on overflow; parity is only claimed where no
 * intermediate overflows; the GPU library rejects such inputs with
 * NW_ERR_RANGE).
 */
#include "nw_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t wmul(int64_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t iabs32(int32_t v) { return v < 0 ? (int32_t)(0u - (uint32_t)v) : v; }

void nwo_gen_dna(uint64_t seed, int64_t n, char *out)
{
        uint64_t st = seed;
        for (int64_t i = 0; i < n; i++) {
                st += 0x9E3779B97F4A7C15ULL;
                uint64_t z = st;
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
                z ^= z >> 31;
                out[i] = "ACGT"[z >> 62];
        }
}

uint64_t nwo_fnv1a(uint64_t h, const void *p, int64_t n)
{
        const uint8_t *b = (const uint8_t *)p;
        for (int64_t i = 0; i < n; i++) {
                h ^= b[i];
                h *= 0x100000001b3ULL;
        }
        return h;
}

/* One cell: needleman-wunsch.c:418-510.  Returns the score, writes the code. */
static inline int32_t cell(int32_t up_h, int32_t diag_h, int32_t left_h,
                           int match, int32_t m, int32_t k, int32_t d,
                           uint8_t *code)
{
        int32_t up = wsub(up_h, d);
        int32_t diag = match ? wadd(diag_h, m) : wsub(diag_h, k);
        int32_t left = wsub(left_h, d);
        int32_t h = up;                    /* max3(up, left, diag) :465 */
        if (h < left) h = left;
        if (h < diag) h = diag;
        *code = (uint8_t)((h == diag) | ((h == up) << 1) | ((h == left) << 2));
        return h;
}

static inline int popc3(uint8_t c) { return (c & 1) + ((c >> 1) & 1) + ((c >> 2) & 1); }

/* Fill column i (1..L1) from column i-1; prev/cur hold L2+1 rows. */
static inline void fill_column(const char *s1, const char *s2, int64_t L2,
                               int64_t i, int32_t m, int32_t k, int32_t d,
                               const int32_t *prev, int32_t *cur, uint8_t *codes,
                               int32_t *gav, uint32_t *bc)
{
        cur[0] = wmul(i, wsub(0, d));      /* computation.c:102-110 */
        if (codes) codes[0] = 4;           /* LEFT */
        const char a = s1[i - 1];
        int32_t g = *gav;
        uint32_t b = *bc;
        for (int64_t j = 1; j <= L2; j++) {
                uint8_t c;
                int32_t h = cell(cur[j - 1], prev[j - 1], prev[j], a == s2[j - 1], m, k, d, &c);
                cur[j] = h;
                if (codes) codes[j] = c;
                b += popc3(c) > 1;
                int32_t ah = iabs32(h);
                if (ah > g) g = ah;
        }
        *gav = g;
        *bc = b;
}

static void seed_column0(int64_t L2, int32_t d, int32_t *col, uint8_t *codes)
{
        col[0] = 0;                        /* computation.c:93-99 */
        if (codes) codes[0] = 0;
        for (int64_t j = 1; j <= L2; j++) {
                col[j] = wmul(j, wsub(0, d)); /* computation.c:112-120 */
                if (codes) codes[j] = 2;   /* UP */
        }
}

int nwo_fill(const char *s1, int64_t L1, const char *s2, int64_t L2,
             int32_t m, int32_t k, int32_t d,
             int32_t *H, uint8_t *D, nwo_stats *st)
{
        const int64_t N = L2 + 1;
        int32_t *tmp = NULL;
        if (!H) {
                tmp = malloc(sizeof(int32_t) * 2 * (size_t)N);
                if (!tmp) return -1;
        }
        int32_t gav = 0;
        uint32_t bc = 0;
        int32_t *c0 = H ? H : tmp;
        seed_column0(L2, d, c0, D);
        for (int64_t i = 1; i <= L1; i++) {
                const int32_t *prev = H ? H + (i - 1) * N : tmp + ((i - 1) & 1) * N;
                int32_t *cur = H ? H + i * N : tmp + (i & 1) * N;
                fill_column(s1, s2, L2, i, m, k, d, prev, cur, D ? D + i * N : NULL, &gav, &bc);
        }
        if (st) {
                st->corner = H ? H[L1 * N + L2] : tmp[(L1 & 1) * N + L2];
                st->greatest_abs_interior = gav;
                st->branch_count = bc;
        }
        free(tmp);
        return 0;
}

/* A band of rows (a multi-GPU row panel, include/nw_panel.h): global rows
 * row_base+1 .. row_base+rows, given the global row row_base above it as
 * top[0..L1].  The same recurrence (needleman-wunsch.c:418-510); column 0 is
 * the seed -j*d (computation.c:112-120) at global row j.  H is
 * (L1+1)*(rows+1) i-major with local row 0 = top; D (nullable) the codes of
 * local rows >= 1 (row 0: 0, it belongs to the band above).  Stats cover the
 * band's own interior cells.  s2 points at the band's first side-string byte. */
int nwo_fill_band(const char *s1, int64_t L1, const char *s2, int64_t rows, int64_t row_base,
                  const int32_t *top, int32_t m, int32_t k, int32_t d,
                  int32_t *H, uint8_t *D, nwo_stats *st)
{
        const int64_t N = rows + 1;
        int32_t gav = 0;
        uint32_t bc = 0;
        for (int64_t j = 0; j <= rows; j++) {
                H[j] = wmul(row_base + j, wsub(0, d));
                if (D) D[j] = j ? 2 : 0;
        }
        for (int64_t i = 1; i <= L1; i++) {
                int32_t *cur = H + i * N;
                const int32_t *prev = H + (i - 1) * N;
                cur[0] = top[i];
                if (D) D[i * N] = 0;
                const char a = s1[i - 1];
                for (int64_t j = 1; j <= rows; j++) {
                        uint8_t c;
                        int32_t h = cell(cur[j - 1], prev[j - 1], prev[j], a == s2[j - 1], m, k, d, &c);
                        cur[j] = h;
                        if (D) D[i * N + j] = c;
                        bc += popc3(c) > 1;
                        int32_t ah = iabs32(h);
                        if (ah > gav) gav = ah;
                }
        }
        if (st) {
                st->corner = H[L1 * N + rows];
                st->greatest_abs_interior = gav;
                st->branch_count = bc;
        }
        return 0;
}

int nwo_fill_hash(const char *s1, int64_t L1, const char *s2, int64_t L2,
                  int32_t m, int32_t k, int32_t d,
                  uint64_t *hH, uint64_t *hD, nwo_stats *st)
{
        const int64_t N = L2 + 1;
        int32_t *col = malloc(sizeof(int32_t) * 2 * (size_t)N);
        uint8_t *codes = malloc((size_t)N);
        if (!col || !codes) {
                free(col);
                free(codes);
                return -1;
        }
        uint64_t h1 = NWO_FNV_INIT, h2 = NWO_FNV_INIT;
        int32_t gav = 0;
        uint32_t bc = 0;
        seed_column0(L2, d, col, codes);
        h1 = nwo_fnv1a(h1, col, 4 * N);
        h2 = nwo_fnv1a(h2, codes, N);
        for (int64_t i = 1; i <= L1; i++) {
                const int32_t *prev = col + ((i - 1) & 1) * N;
                int32_t *cur = col + (i & 1) * N;
                fill_column(s1, s2, L2, i, m, k, d, prev, cur, codes, &gav, &bc);
                h1 = nwo_fnv1a(h1, cur, 4 * N);
                h2 = nwo_fnv1a(h2, codes, N);
        }
        if (hH) *hH = h1;
        if (hD) *hD = h2;
        if (st) {
                st->corner = col[(L1 & 1) * N + L2];
                st->greatest_abs_interior = gav;
                st->branch_count = bc;
        }
        free(col);
        free(codes);
        return 0;
}

int nwo_fill_colchain(const char *s1, int64_t L1, const char *s2, int64_t L2,
                      int32_t m, int32_t k, int32_t d,
                      uint64_t *hH2, uint64_t *hD2, nwo_stats *st)
{
        const int64_t N = L2 + 1;
        int32_t *col = malloc(sizeof(int32_t) * 2 * (size_t)N);
        uint8_t *codes = malloc((size_t)N);
        if (!col || !codes) {
                free(col);
                free(codes);
                return -1;
        }
        uint64_t h1 = NWO_FNV_INIT, h2 = NWO_FNV_INIT;
        int32_t gav = 0;
        uint32_t bc = 0;
        seed_column0(L2, d, col, codes);
        uint64_t c1 = nwo_fnv1a(NWO_FNV_INIT, col, 4 * N), c2 = nwo_fnv1a(NWO_FNV_INIT, codes, N);
        h1 = nwo_fnv1a(h1, &c1, 8);
        h2 = nwo_fnv1a(h2, &c2, 8);
        for (int64_t i = 1; i <= L1; i++) {
                const int32_t *prev = col + ((i - 1) & 1) * N;
                int32_t *cur = col + (i & 1) * N;
                fill_column(s1, s2, L2, i, m, k, d, prev, cur, codes, &gav, &bc);
                c1 = nwo_fnv1a(NWO_FNV_INIT, cur, 4 * N);
                c2 = nwo_fnv1a(NWO_FNV_INIT, codes, N);
                h1 = nwo_fnv1a(h1, &c1, 8);
                h2 = nwo_fnv1a(h2, &c2, 8);
        }
        if (hH2) *hH2 = h1;
        if (hD2) *hD2 = h2;
        if (st) {
                st->corner = col[(L1 & 1) * N + L2];
                st->greatest_abs_interior = gav;
                st->branch_count = bc;
        }
        free(col);
        free(codes);
        return 0;
}

int32_t nwo_score_only(const char *s1, int64_t L1, const char *s2, int64_t L2,
                       int32_t m, int32_t k, int32_t d, uint64_t *hlast)
{
        const int64_t N = L2 + 1;
        int32_t *col = malloc(sizeof(int32_t) * 2 * (size_t)N);
        if (!col) return 0;
        int32_t gav = 0;
        uint32_t bc = 0;
        seed_column0(L2, d, col, NULL);
        for (int64_t i = 1; i <= L1; i++)
                fill_column(s1, s2, L2, i, m, k, d, col + ((i - 1) & 1) * N,
                            col + (i & 1) * N, NULL, &gav, &bc);
        const int32_t *last = col + (L1 & 1) * N;
        if (hlast) *hlast = nwo_fnv1a(NWO_FNV_INIT, last, 4 * N);
        int32_t r = last[L2];
        free(col);
        return r;
}

/* ---- blocked anti-diagonal pthread fill (CPU baseline) ------------------ */

typedef struct {
        const char *s1, *s2;
        int64_t L1, L2;
        int32_t m, k, d;
        int32_t *H;
        uint8_t *D;
        int64_t bi, bj;           /* block size (columns, rows) */
        int64_t nbi, nbj;
        int nthreads;
        pthread_barrier_t bar;
} mt_ctx;

typedef struct {
        mt_ctx *c;
        int tid;
        int32_t gav;
        uint32_t bc;
} mt_arg;

static void *mt_worker(void *p)
{
        mt_arg *a = (mt_arg *)p;
        mt_ctx *c = a->c;
        const int64_t N = c->L2 + 1;
        for (int64_t t = 0; t < c->nbi + c->nbj - 1; t++) {
                int64_t lo = t - (c->nbj - 1) > 0 ? t - (c->nbj - 1) : 0;
                int64_t hi = t < c->nbi - 1 ? t : c->nbi - 1;
                for (int64_t b = lo + a->tid; b <= hi; b += c->nthreads) {
                        int64_t bi = b, bj = t - b;
                        int64_t i0 = 1 + bi * c->bi, i1 = i0 + c->bi;
                        int64_t j0 = 1 + bj * c->bj, j1 = j0 + c->bj;
                        if (i1 > c->L1 + 1) i1 = c->L1 + 1;
                        if (j1 > c->L2 + 1) j1 = c->L2 + 1;
                        for (int64_t i = i0; i < i1; i++) {
                                const int32_t *prev = c->H + (i - 1) * N;
                                int32_t *cur = c->H + i * N;
                                uint8_t *codes = c->D ? c->D + i * N : NULL;
                                const char ch = c->s1[i - 1];
                                for (int64_t j = j0; j < j1; j++) {
                                        uint8_t code;
                                        int32_t h = cell(cur[j - 1], prev[j - 1], prev[j],
                                                         ch == c->s2[j - 1], c->m, c->k, c->d, &code);
                                        cur[j] = h;
                                        if (codes) codes[j] = code;
                                        a->bc += popc3(code) > 1;
                                        int32_t ah = iabs32(h);
                                        if (ah > a->gav) a->gav = ah;
                                }
                        }
                }
                pthread_barrier_wait(&c->bar);
        }
        return NULL;
}

int nwo_fill_mt(const char *s1, int64_t L1, const char *s2, int64_t L2,
                int32_t m, int32_t k, int32_t d,
                int32_t *H, uint8_t *D, nwo_stats *st, int nthreads)
{
        if (nthreads < 1) nthreads = 1;
        const int64_t N = L2 + 1;
        seed_column0(L2, d, H, D);
        for (int64_t i = 1; i <= L1; i++) {
                H[i * N] = wmul(i, wsub(0, d));
                if (D) D[i * N] = 4;
        }
        mt_ctx c = {s1, s2, L1, L2, m, k, d, H, D, 512, 2048, 0, 0, nthreads, {{0}}};
        c.nbi = L1 > 0 ? (L1 + c.bi - 1) / c.bi : 0;
        c.nbj = L2 > 0 ? (L2 + c.bj - 1) / c.bj : 0;
        mt_arg *args = calloc((size_t)nthreads, sizeof(mt_arg));
        pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
        if (c.nbi > 0 && c.nbj > 0) {
                pthread_barrier_init(&c.bar, NULL, (unsigned)nthreads);
                for (int t = 0; t < nthreads; t++) {
                        args[t].c = &c;
                        args[t].tid = t;
                        pthread_create(&th[t], NULL, mt_worker, &args[t]);
                }
                for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
                pthread_barrier_destroy(&c.bar);
        }
        if (st) {
                st->corner = H[L1 * N + L2];
                st->greatest_abs_interior = 0;
                st->branch_count = 0;
                for (int t = 0; t < nthreads; t++) {
                        if (args[t].gav > st->greatest_abs_interior)
                                st->greatest_abs_interior = args[t].gav;
                        st->branch_count += args[t].bc;
                }
        }
        free(args);
        free(th);
        return 0;
}

/*
 * Walk services over a filled code table (one byte per cell, i-major).
 *
 * nwo_count_paths restates the number of alignments the reference's
 * depth-first walk reaches (construct_alignments_for_subtable,
 * needleman-wunsch.c:209-331, counting in inc_solution_count at :250-255 with
 * an `unsigned` counter, walk-table.c:108-147): every arrival at (0,0) is
 * one distinct path of code edges from the corner, so the count is the
 * path-count DP  P(0,0) = 1,  P(i,j) = [diag] P(i-1,j-1) + [left] P(i-1,j)
 * + [up] P(i,j-1), in uint32 arithmetic (it wraps exactly like the
 * reference's counter).
 */
uint32_t nwo_count_paths(const uint8_t *D, int64_t L1, int64_t L2)
{
        const int64_t N = L2 + 1;
        uint32_t *prev = malloc((size_t)N * sizeof *prev);
        uint32_t *cur = malloc((size_t)N * sizeof *cur);
        if (!prev || !cur) {
                free(prev);
                free(cur);
                return 0;
        }
        for (int64_t j = 0; j < N; j++) prev[j] = 1;   /* column 0: (0,0) then UP codes */
        for (int64_t i = 1; i <= L1; i++) {
                const uint8_t *c = D + i * N;
                cur[0] = prev[0];                      /* (i,0): LEFT code */
                for (int64_t j = 1; j < N; j++) {
                        uint32_t p = 0;
                        if (c[j] & 1) p += prev[j - 1];
                        if (c[j] & 4) p += prev[j];
                        if (c[j] & 2) p += cur[j - 1];
                        cur[j] = p;
                }
                uint32_t *t = prev;
                prev = cur;
                cur = t;
        }
        /* Two empty strings: the walk starts on (0,0), whose three directions
           init_computation marked done (computation.c:96-99), so its loop
           (needleman-wunsch.c:231-235) never runs and nothing is counted. */
        const uint32_t r = (L1 == 0 && L2 == 0) ? 0u : prev[L2];
        free(prev);
        free(cur);
        return r;
}

/*
 * The first alignment the reference's walk prints: from the corner it takes
 * the diagonal if flagged, else the left, else the up predecessor
 * (needleman-wunsch.c:296-322), and the first arrival at (0,0) prints.
 * moves[] receives the path in forward order ((0,0) -> (L1,L2)): 1 = diag,
 * 2 = up (gap in s1), 4 = left (gap in s2).  Returns the number of moves, or
 * -1 if a cell on the way has no code.
 */
int64_t nwo_first_path(const uint8_t *D, int64_t L1, int64_t L2, uint8_t *moves)
{
        const int64_t N = L2 + 1;
        int64_t i = L1, j = L2, n = 0;
        while (i > 0 || j > 0) {
                const uint8_t c = D[i * N + j];
                uint8_t mv;
                if (c & 1) {
                        mv = 1;
                        i--;
                        j--;
                } else if (c & 4) {
                        mv = 4;
                        i--;
                } else if (c & 2) {
                        mv = 2;
                        j--;
                } else {
                        return -1;
                }
                moves[n++] = mv;
        }
        for (int64_t a = 0, b = n - 1; a < b; a++, b--) {
                const uint8_t t = moves[a];
                moves[a] = moves[b];
                moves[b] = t;
        }
        return n;
}

/* ---- score-only band wavefront on T threads (pins the 1M x 1M fill) ---- */
/* Same recurrence as fill_column (needleman-wunsch.c:429-465) in O(L1 + L2)
 * memory: thread t owns rows of band t, walks the columns, takes the row
 * above from band t-1's published bottom row and publishes its own. */

typedef struct {
        const char *s1, *s2;
        int64_t L1, L2, nr;       /* rows per band */
        int32_t m, k, d;
        int32_t **bnd;            /* bnd[t][i] = H[i][last row of band t] */
        int64_t *prog;            /* columns of bnd[t] published */
        int32_t *lastcol;         /* H[L1][0..L2] */
        int nb;
} so_ctx;

typedef struct {
        so_ctx *c;
        int t;
} so_arg;

static void *so_worker(void *p)
{
        so_arg *a = (so_arg *)p;
        so_ctx *c = a->c;
        const int t = a->t;
        const int64_t r0 = 1 + (int64_t)t * c->nr;
        const int64_t r1 = (r0 + c->nr - 1 < c->L2) ? r0 + c->nr - 1 : c->L2;
        const int64_t nr = r1 - r0 + 1;
        const int32_t m = c->m, k = c->k, d = c->d;
        int32_t *prev = malloc(sizeof(int32_t) * (size_t)(nr + 1));
        int32_t *cur = malloc(sizeof(int32_t) * (size_t)(nr + 1));
        if (!prev || !cur) abort();
        for (int64_t x = 0; x <= nr; x++) prev[x] = (int32_t)(-(r0 - 1 + x) * (int64_t)d);   /* column 0 */
        c->bnd[t][0] = prev[nr];
        int64_t seen = 0;
        for (int64_t i = 1; i <= c->L1; i++) {
                int32_t top;
                if (t == 0) {
                        top = (int32_t)(-i * (int64_t)d);                   /* row 0 */
                } else {
                        while (seen < i) seen = __atomic_load_n(&c->prog[t - 1], __ATOMIC_ACQUIRE);
                        top = c->bnd[t - 1][i];
                }
                cur[0] = top;
                const char c1 = c->s1[i - 1];
                const char *s2 = c->s2 + (r0 - 1);
                for (int64_t x = 1; x <= nr; x++) {
                        const int32_t dg = prev[x - 1] + (c1 == s2[x - 1] ? m : -k);
                        const int32_t l = prev[x] - d, u = cur[x - 1] - d;
                        int32_t v = dg > l ? dg : l;
                        cur[x] = v > u ? v : u;
                }
                c->bnd[t][i] = cur[nr];
                if ((i & 63) == 0 || i == c->L1) __atomic_store_n(&c->prog[t], i, __ATOMIC_RELEASE);
                int32_t *tmp = prev;
                prev = cur;
                cur = tmp;
        }
        memcpy(c->lastcol + r0, prev + 1, sizeof(int32_t) * (size_t)nr);
        free(prev);
        free(cur);
        return NULL;
}

int32_t nwo_score_only_mt(const char *s1, int64_t L1, const char *s2, int64_t L2,
                          int32_t m, int32_t k, int32_t d, int nthreads, uint64_t *hlast)
{
        if (L1 == 0 || L2 == 0 || nthreads <= 1) return nwo_score_only(s1, L1, s2, L2, m, k, d, hlast);
        so_ctx c;
        c.s1 = s1;
        c.s2 = s2;
        c.L1 = L1;
        c.L2 = L2;
        c.m = m;
        c.k = k;
        c.d = d;
        c.nb = nthreads;
        c.nr = (L2 + nthreads - 1) / nthreads;
        while ((c.nb - 1) * c.nr >= L2) c.nb--;      /* no empty bands */
        c.bnd = malloc(sizeof(int32_t *) * (size_t)c.nb);
        c.prog = calloc((size_t)c.nb, sizeof(int64_t));
        c.lastcol = malloc(sizeof(int32_t) * (size_t)(L2 + 1));
        if (!c.bnd || !c.prog || !c.lastcol) abort();
        for (int t = 0; t < c.nb; t++) {
                c.bnd[t] = malloc(sizeof(int32_t) * (size_t)(L1 + 1));
                if (!c.bnd[t]) abort();
        }
        c.lastcol[0] = (int32_t)(-L1 * (int64_t)d);
        pthread_t *th = malloc(sizeof(pthread_t) * (size_t)c.nb);
        so_arg *args = malloc(sizeof(so_arg) * (size_t)c.nb);
        for (int t = 0; t < c.nb; t++) {
                args[t].c = &c;
                args[t].t = t;
                pthread_create(&th[t], NULL, so_worker, &args[t]);
        }
        for (int t = 0; t < c.nb; t++) pthread_join(th[t], NULL);
        if (hlast) *hlast = nwo_fnv1a(NWO_FNV_INIT, c.lastcol, 4 * (L2 + 1));
        const int32_t r = c.lastcol[L2];
        for (int t = 0; t < c.nb; t++) free(c.bnd[t]);
        free(c.bnd);
        free(c.prog);
        free(c.lastcol);
        free(th);
        free(args);
        return r;
}
