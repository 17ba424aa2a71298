/*
 * nw_host.h -- host side of the reference-compatible CLI.
 *
 * The reference keeps its whole program in one process: reader
 * (read-sequences.c), driver (needleman-wunsch.c:654-689), traceback
 * (needleman-wunsch.c:91-388), summary (computation.c:271-281), table printer
 * (print-table.c) and ANSI formatting (format.c/format.h).  Here those stay
 * on the host, fed by the GPU fill (include/nw_fill.h); they are restated in
 * C++ with the reference's exact output bytes.
 *
 * nwh_render() is a pure function of the filled tables, so the CPU test suite
 * can check it against the reference's golden output without a GPU.
 */
#ifndef NW_HOST_H
#define NW_HOST_H

#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nwh_flags {
        int cflag;   /* -c  ANSI colours              (format.h:113)          */
        int lflag;   /* -l  per-alignment counts      (needleman-wunsch.h:51) */
        int qflag;   /* -q  quiet                     (needleman-wunsch.h:52) */
        int sflag;   /* -s  summary to stderr         (needleman-wunsch.h:53) */
        int tflag;   /* -t  print the table           (needleman-wunsch.h:54) */
        int uflag;   /* -u  unicode arrows            (needleman-wunsch.h:55) */
} nwh_flags;

/* Does the run need the traceback (needleman-wunsch.c:667)? */
int nwh_needs_traceback(const nwh_flags *f);

/* Everything the reference prints after compute_table_scores()
 * (needleman-wunsch.c:664-685): alignments / counts to `out`, the summary to
 * `err`, the table to `out`.
 *   s1, s2 : the sequences (L1 = strlen(s1), L2 = strlen(s2))
 *   H      : (L1+1)*(L2+1) int32, i-major; needed only when f->tflag
 *   codes  : (L1+1)*(L2+1) direction codes (bit0 diag, bit1 up, bit2 left),
 *            i-major; needed when nwh_needs_traceback(f) or f->tflag
 *   corner : H[L1][L2];  gav : max |H| over interior cells (for -t)
 * Returns 0, or -1 if memory for the walk state could not be allocated. */
int nwh_render(const char *s1, const char *s2, const nwh_flags *f,
               const int32_t *H, const uint8_t *codes, int32_t corner,
               int32_t gav, FILE *out, FILE *err);

/* Source of the alignments for nwh_render_paths: sets *moves / *n to the next
 * alignment in print order -- its moves from (L1,L2) back to (0,0), 1 = diag,
 * 2 = up, 4 = left (nw_table_enumerate_paths) -- and returns 1; returns 0
 * after the last one, < 0 on failure. */
typedef int (*nwh_next_path)(void *ctx, const uint8_t **moves, int64_t *n);

/* nwh_render with the alignments supplied by `next` (the device enumeration)
 * instead of the host depth-first walk: prints them as the walk would
 * (needleman-wunsch.c:245-254), then the summary with `solutions`, then the
 * table, its optimal-path cells being those reachable from the corner along
 * the codes -- exactly the cells the reference's complete walk visits.
 * codes: needed for -t; H: for -t.  Returns 0, -1 on allocation failure, -2
 * when `next` fails. */
int nwh_render_paths(const char *s1, const char *s2, const nwh_flags *f,
                     const int32_t *H, const uint8_t *codes, int32_t corner,
                     int32_t gav, unsigned solutions, nwh_next_path next,
                     void *ctx, FILE *out, FILE *err);

/* The summary print_summary() writes under -s (computation.c:271-281):
 * "<n> optimal alignment[s]" and "Optimal score is <corner>". */
void nwh_print_summary(unsigned solutions, int32_t corner, FILE *err);

/* Same, into malloc'ed buffers (for tests); caller frees *out / *err. */
int nwh_render_to_buffers(const char *s1, const char *s2, const nwh_flags *f,
                          const int32_t *H, const uint8_t *codes,
                          int32_t corner, int32_t gav, char **out,
                          size_t *out_len, char **err, size_t *err_len);

void nwh_free(void *p);

/* Reader with read-sequences.c:43-122 semantics.  Returns 0 and two malloc'ed
 * NUL-terminated strings, or -1 after printing the reference's error message
 * (prog: error: ...) to stderr. */
int nwh_read_two_sequences(FILE *in, const char *prog, char **s1, char **s2);

#ifdef __cplusplus
}
#endif
#endif
