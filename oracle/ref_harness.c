/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Drives the *compiled reference* (objects built by oracle/Makefile from the
 * sources under /root/reference, outputs only into oracle/_ref/) through its
 * own library-style entry points, exactly as the reference driver does at
 * needleman-wunsch.c:658-662:
 *
 *     alloc_computation()            computation.c:51-58
 *     init_computation(C,...,T)      computation.c:145-191 (seeding :75-125)
 *     compute_table_scores(C)        needleman-wunsch.c:583-626  (the hot path)
 *
 * and then reads C->score_table / C->walk_table directly to emit the parity
 * statistics used to pin oracle/nw_oracle.c and the HIP path:
 *
 *   corner   = score_table->cells[M-1][N-1].score    (computation.c:279-280)
 *   gav      = score_table->greatest_abs_val         (needleman-wunsch.c:538-541,
 *              interior cells only, tflag=1)
 *   bc       = walk_table->branch_count              (walk-table.c:108-147)
 *   hH       = FNV-1a-64 over little-endian int32 scores, i-major (i=0..L1,
 *              j=0..L2 inner)
 *   hD       = FNV-1a-64 over one byte per cell, diag | up<<1 | left<<2,
 *              same order (walk-table.h:44-54 flags)
 *
 * Usage:
 *   ref_harness gen L1 L2 m k d [T] [dumpfile]   splitmix64 DNA, seeds 1 / 2
 *   ref_harness str S1 S2 m k d [T] [dumpfile]   literal strings ("" allowed)
 *
 * dumpfile (optional): int32 H[(L1+1)*(L2+1)] then uint8 D[(L1+1)*(L2+1)],
 * both i-major.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "computation.h"

extern int tflag;                      /* needleman-wunsch.h:54 */
void compute_table_scores(computation_t *C);   /* needleman-wunsch.c:583 */

static char *gen_dna(uint64_t seed, long n)
{
        char *s = malloc((size_t)n + 1);
        uint64_t st = seed;
        for (long i = 0; i < n; i++) {
                st += 0x9E3779B97F4A7C15ULL;
                uint64_t z = st;
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
                z ^= z >> 31;
                s[i] = "ACGT"[z >> 62];
        }
        s[n] = '\0';
        return s;
}

int main(int argc, char **argv)
{
        if (argc < 7) {
                fprintf(stderr, "usage: %s gen|str A B m k d [T] [dump]\n", argv[0]);
                return 2;
        }
        char *s1, *s2;
        if (strcmp(argv[1], "gen") == 0) {
                s1 = gen_dna(1, atol(argv[2]));
                s2 = gen_dna(2, atol(argv[3]));
        } else {
                s1 = strdup(argv[2]);
                s2 = strdup(argv[3]);
        }
        int m = atoi(argv[4]), k = atoi(argv[5]), d = atoi(argv[6]);
        int T = argc > 7 ? atoi(argv[7]) : 1;
        const char *dump = argc > 8 ? argv[8] : NULL;

        tflag = 1;
        struct timespec ti, t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &ti);
        computation_t *C = alloc_computation();
        /* allocation + seeding; with T > 1 also one mutex + condvar init per
         * cell (computation.c:80-89), the larger part of the -p path's cost */
        init_computation(C, s1, s2, m, k, d, (unsigned)T);
        clock_gettime(CLOCK_MONOTONIC, &t0);
        compute_table_scores(C);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        double init_s = (double)(t0.tv_sec - ti.tv_sec) + 1e-9 * (double)(t0.tv_nsec - ti.tv_nsec);
        double fill_s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        if (getenv("NW_REF_TIME_ONLY")) {   /* timing legs: skip the table hashes */
                printf("{\"L1\": %d, \"L2\": %d, \"corner\": %d, \"threads\": %d, \"init_s\": %.6f, "
                       "\"fill_s\": %.6f}\n", C->score_table->M - 1, C->score_table->N - 1,
                       C->score_table->cells[C->score_table->M - 1][C->score_table->N - 1].score, T, init_s,
                       fill_s);
                return 0;
        }

        score_table_t *S = C->score_table;
        walk_table_t *W = C->walk_table;
        uint64_t hH = 0xcbf29ce484222325ULL, hD = 0xcbf29ce484222325ULL;
        FILE *f = dump ? fopen(dump, "wb") : NULL;
        for (int i = 0; i < S->M; i++) {
                for (int j = 0; j < S->N; j++) {
                        uint32_t v = (uint32_t)S->cells[i][j].score;
                        for (int b = 0; b < 4; b++) {
                                hH ^= (v >> (8 * b)) & 0xff;
                                hH *= 0x100000001b3ULL;
                        }
                        walk_table_cell_t *w = &W->cells[i][j];
                        uint8_t c = (uint8_t)((w->diag ? 1 : 0) | (w->up ? 2 : 0) |
                                              (w->left ? 4 : 0));
                        hD ^= c;
                        hD *= 0x100000001b3ULL;
                }
        }
        if (f) {
                for (int i = 0; i < S->M; i++)
                        for (int j = 0; j < S->N; j++)
                                fwrite(&S->cells[i][j].score, 4, 1, f);
                for (int i = 0; i < S->M; i++)
                        for (int j = 0; j < S->N; j++) {
                                walk_table_cell_t *w = &W->cells[i][j];
                                uint8_t c = (uint8_t)((w->diag ? 1 : 0) | (w->up ? 2 : 0) |
                                                      (w->left ? 4 : 0));
                                fwrite(&c, 1, 1, f);
                        }
                fclose(f);
        }
        printf("{\"L1\": %d, \"L2\": %d, \"m\": %d, \"k\": %d, \"d\": %d, "
               "\"corner\": %d, \"gav\": %d, \"branch_count\": %u, "
               "\"hH\": \"%016llx\", \"hD\": \"%016llx\", \"threads\": %d, \"init_s\": %.6f, "
               "\"fill_s\": %.6f}\n",
               S->M - 1, S->N - 1, m, k, d,
               S->cells[S->M - 1][S->N - 1].score, S->greatest_abs_val,
               W->branch_count, (unsigned long long)hH, (unsigned long long)hD, T, init_s, fill_s);
        return 0;
}
