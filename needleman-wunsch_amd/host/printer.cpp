// printer.cpp -- output of the reference CLI after the fill: alignments and
// counts (needleman-wunsch.c:101-182), the stderr summary
// (computation.c:271-281), the score/arrow table (print-table.c:50-208) and
// the ANSI formats (format.c:47-97, format.h:42-102).  Byte-identical output
// is checked against the reference's goldens (tests/golden/cli_cases.json).
#include <cstdlib>
#include <cstring>

#include "nw_host_internal.h"

namespace nwh {

namespace {
const char* const kFmt[] = {
    "\x1b[1m",     // top string      (bold)
    "\x1b[1m",     // side string     (bold)
    "\x1b[32;1m",  // optimal path    (green, bold)
    "\x1b[36;1m",  // match arrow     (cyan, bold)
    "\x1b[31;1m",  // mismatch arrow  (red, bold)
    "\x1b[33;1m",  // gap arrow       (yellow, bold)
    "",            // match char
    "\x1b[31;1m",  // mismatch char   (= mismatch arrow)
    "",            // gap char
};
constexpr char kGap = '-';
}  // namespace

void set_fmt(const Render& r, Fmt f) {
    if (r.f.cflag) fputs(kFmt[f], r.out);
}

void reset_fmt(const Render& r) {
    if (r.f.cflag) fputs("\x1b[0m", r.out);
}

namespace {
void aligned_char(const Render& r, const char* a, const char* b, int64_t k) {
    if (a[k] == b[k]) set_fmt(r, MATCH_CHAR);
    else if (a[k] == kGap || b[k] == kGap) set_fmt(r, GAP_CHAR);
    else set_fmt(r, MISMATCH_CHAR);
    fputc(a[k], r.out);
    reset_fmt(r);
}
}  // namespace

void print_alignment(const Render& r, const char* X, const char* Y, int64_t n) {
    const bool strings = !r.f.qflag, counts = r.f.lflag != 0;
    int matches = 0, mismatches = 0, gaps = 0;
    for (int64_t k = n; k >= 0; --k) {   // stored back to front
        if (strings) aligned_char(r, X, Y, k);
        if (counts) {
            if (X[k] == Y[k]) ++matches;
            else if (X[k] == kGap || Y[k] == kGap) ++gaps;
            else ++mismatches;
        }
    }
    if (strings) {
        fputc('\n', r.out);
        for (int64_t k = n; k >= 0; --k) aligned_char(r, Y, X, k);
        fputc('\n', r.out);
    }
    if (counts)
        fprintf(r.out, "%d match%s, %d mismatch%s, %d indel%s\n", matches, matches == 1 ? "" : "es", mismatches,
                mismatches == 1 ? "" : "es", gaps, gaps == 1 ? "" : "s");
    fputc('\n', r.out);
}

namespace {

int width_for(int32_t x) {   // digits of |x| plus a sign column
    int w = 0;
    do {
        x /= 10;
        ++w;
    } while (x != 0);
    return w + 1;
}

enum Arrow { LEFT, UP, DIAG };

void arrow(const Render& r, Arrow a, bool opt, int width, int64_t col, int64_t row) {
    const bool u = r.f.uflag != 0;
    switch (a) {
        case LEFT:
            if (opt) set_fmt(r, GAP_ARROW);
            fprintf(r.out, "  %s ", u ? "←" : "<");
            break;
        case UP:
            if (opt) set_fmt(r, GAP_ARROW);
            fprintf(r.out, "%*s", u ? width + 2 : width, u ? "↑" : "^");
            break;
        case DIAG:
            if (opt) set_fmt(r, r.s1[col - 1] == r.s2[row - 1] ? MATCH_ARROW : MISMATCH_ARROW);
            fprintf(r.out, "  %s ", u ? "↖" : "\\");
            break;
    }
    if (opt) reset_fmt(r);
}

void print_table(const Render& r, const std::vector<uint16_t>& walk, int32_t gav) {
    const int64_t M = r.L1 + 1, N = r.L2 + 1;
    const int width = width_for(gav);
    auto opt = [&](int64_t col, int64_t row) { return !walk.empty() && (walk[(size_t)(col * N + row)] & WALK_OPT); };
    auto code = [&](int64_t col, int64_t row) { return r.codes[col * N + row]; };
    // header: top string (print-table.c:172-182; note: no reset afterwards)
    set_fmt(r, TOP_STRING);
    fprintf(r.out, "*    %*s", width, "-");
    for (int64_t i = 0; i < M - 1; ++i) fprintf(r.out, "    %*s%c", width - 1, "", r.s1[i]);
    fputc('\n', r.out);
    for (int64_t row = 0; row < N; ++row) {
        // arrows row: diagonal and up arrows of each cell
        fputc(' ', r.out);
        for (int64_t col = 0; col < M; ++col) {
            const bool o = opt(col, row);
            if (code(col, row) & 1) arrow(r, DIAG, o, width, col, row);
            else fputs("    ", r.out);
            if (code(col, row) & 2) arrow(r, UP, o, width, col, row);
            else fprintf(r.out, "%*s", width, "");
        }
        fputc('\n', r.out);
        // score row: side-string letter, left arrows and scores
        set_fmt(r, SIDE_STRING);
        fputc(row == 0 ? '-' : r.s2[row - 1], r.out);
        reset_fmt(r);
        for (int64_t col = 0; col < M; ++col) {
            const bool o = opt(col, row);
            if (code(col, row) & 4) arrow(r, LEFT, o, width, col, row);
            else fputs("    ", r.out);
            if (o) set_fmt(r, OPT_PATH);
            fprintf(r.out, "%+*d", width, r.H[col * N + row]);
            if (o) reset_fmt(r);
        }
        fputc('\n', r.out);
    }
}

}  // namespace
}  // namespace nwh

extern "C" {

int nwh_needs_traceback(const nwh_flags* f) {
    return f->qflag != 1 || f->lflag == 1 || f->sflag == 1 || f->tflag == 1;   // needleman-wunsch.c:667
}

int nwh_render(const char* s1, const char* s2, const nwh_flags* f, const int32_t* H, const uint8_t* codes,
               int32_t corner, int32_t gav, FILE* out, FILE* err) {
    nwh::Render r{s1, s2, (int64_t)strlen(s1), (int64_t)strlen(s2), *f, H, codes, out, err};
    std::vector<uint16_t> walk;
    unsigned solutions = 0;
    if (nwh_needs_traceback(f)) {
        try {
            if (!nwh::walk_alignments(r, walk, solutions)) return -1;
        } catch (const std::bad_alloc&) {
            return -1;
        }
    }
    if (f->sflag) nwh_print_summary(solutions, corner, err);
    if (f->tflag) {   // needleman-wunsch.c:677-685
        if (f->qflag != 1 || f->sflag == 1 || f->lflag == 1) fputc('\n', out);
        nwh::print_table(r, walk, gav);
    }
    return 0;
}

int nwh_render_paths(const char* s1, const char* s2, const nwh_flags* f, const int32_t* H, const uint8_t* codes,
                     int32_t corner, int32_t gav, unsigned solutions, nwh_next_path next, void* ctx, FILE* out,
                     FILE* err) {
    nwh::Render r{s1, s2, (int64_t)strlen(s1), (int64_t)strlen(s2), *f, H, codes, out, err};
    const int64_t M = r.L1 + 1, N = r.L2 + 1;
    try {
        if (nwh_needs_traceback(f) && (!f->qflag || f->lflag)) {
            std::vector<char> X((size_t)(M + N)), Y((size_t)(M + N));
            for (;;) {
                const uint8_t* mv = nullptr;
                int64_t n = 0;
                const int got = next(ctx, &mv, &n);
                if (got < 0) return -2;
                if (got == 0) break;
                int64_t i = r.L1, j = r.L2;
                for (int64_t q = 0; q < n; ++q) {   // X / Y back to front, as the walk fills them
                    if (mv[q] == 1) {
                        X[(size_t)q] = s1[--i];
                        Y[(size_t)q] = s2[--j];
                    } else if (mv[q] == 4) {
                        X[(size_t)q] = s1[--i];
                        Y[(size_t)q] = '-';
                    } else {
                        X[(size_t)q] = '-';
                        Y[(size_t)q] = s2[--j];
                    }
                }
                nwh::print_alignment(r, X.data(), Y.data(), n - 1);
            }
        }
        if (f->sflag) nwh_print_summary(solutions, corner, err);
        if (f->tflag) {   // needleman-wunsch.c:677-685
            // The complete walk visits every cell reachable from the corner
            // along the codes (each such cell has a path on to (0,0)); two
            // empty strings: the walk never runs.
            std::vector<uint16_t> walk((size_t)(M * N), 0);
            if (r.L1 > 0 || r.L2 > 0) walk[(size_t)(M * N - 1)] = nwh::WALK_OPT;
            for (int64_t i = r.L1; i >= 0; --i)
                for (int64_t j = r.L2; j >= 0; --j) {
                    const size_t c = (size_t)(i * N + j);
                    if (!(walk[c] & nwh::WALK_OPT)) continue;
                    const uint8_t code = (uint8_t)(codes[c] & 7);
                    if ((code & 1) && i > 0 && j > 0) walk[c - (size_t)N - 1] |= nwh::WALK_OPT;
                    if ((code & 4) && i > 0) walk[c - (size_t)N] |= nwh::WALK_OPT;
                    if ((code & 2) && j > 0) walk[c - 1] |= nwh::WALK_OPT;
                }
            if (f->qflag != 1 || f->sflag == 1 || f->lflag == 1) fputc('\n', out);
            nwh::print_table(r, walk, gav);
        }
    } catch (const std::bad_alloc&) {
        return -1;
    }
    return 0;
}

void nwh_print_summary(unsigned solutions, int32_t corner, FILE* err) {   // computation.c:271-281
    fprintf(err, "%d optimal alignment%s\n", (int)solutions, solutions > 1 ? "s" : "");
    fprintf(err, "Optimal score is %-d\n", corner);
}

int nwh_render_to_buffers(const char* s1, const char* s2, const nwh_flags* f, const int32_t* H,
                          const uint8_t* codes, int32_t corner, int32_t gav, char** out, size_t* out_len,
                          char** err, size_t* err_len) {
    FILE* o = open_memstream(out, out_len);
    FILE* e = open_memstream(err, err_len);
    if (!o || !e) return -1;
    const int rc = nwh_render(s1, s2, f, H, codes, corner, gav, o, e);
    fclose(o);
    fclose(e);
    return rc;
}

void nwh_free(void* p) { free(p); }

}  // extern "C"
