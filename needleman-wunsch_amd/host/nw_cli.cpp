// nw_cli.cpp -- `needleman-wunsch`, the reference CLI over the GPU fill.
//
// Same options, operands, messages and exit codes as the reference driver
// (needleman-wunsch.c:65-89 usage, :698-795 main, dbg.c:7-15 program name,
// dbg.h:67-100 error format).  Between reading the sequences and printing,
// compute_table_scores() (needleman-wunsch.c:583) is replaced by a
// device-resident nw_table fill (include/nw_fill.h) on the GPU, and the
// traceback's enumeration by nw_table_enumerate_paths (one device thread per
// alignment, in the reference's order).  -p N is accepted and validated exactly as
// in the reference (it must be > 1) but the fill always runs on the GPU:
// there is no CPU path.  Failure to run the GPU fill is an error (exit 1).
#include <getopt.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "nw_fill.h"
#include "nw_host.h"

namespace {

const char* g_prog = "needleman-wunsch";

void log_err_errno(const char* msg) {
    fprintf(stderr, "%s: error: %s: %s\n", g_prog, msg, errno == 0 ? "\b\b \b" : strerror(errno));
}

[[noreturn]] void usage() {
    fputs("usage: needleman-wunsch [-c][-h][-l][-q][-s][-t][-u]\n"
          "                        [-p num-threads] [-f sequence-file] m k d\n"
          "Align two sequences with the Needleman-Wunsch algorithm\n"
          "operands:\n"
          "   m   match bonus\n"
          "   k   mismatch penalty\n"
          "   d   indel (gap) penalty\n"
          "options:\n"
          "  -c   color the output with ANSI escape sequences\n"
          "  -f sequence-file\n"
          "       read the input strings from 'sequence-file' instead of standard input\n"
          "  -h   print this usage message\n"
          "  -l   list match, mismatch, and indel counts for each alignment pair\n"
          "  -p num-threads\n"
          "       parallelize the computation with 'num-threads' threads (must be >1)\n"
          "  -q   be quiet and don't print the aligned strings\n"
          "  -s   summarize the algorithm's run\n"
          "  -t   print the scores table; only useful for shorter input strings\n"
          "  -u   use unicode arrows when printing the scores table\n",
          stderr);
    exit(1);
}

// Alignments in print order, fetched from the device in batches
// (nw_table_enumerate_paths) for nwh_render_paths.
struct PathBatches {
    nw_table* t = nullptr;
    int64_t stride = 1;
    uint64_t next = 0;          // first alignment of the next batch
    uint64_t have = 0, pos = 0; // alignments in the buffers / handed out
    std::vector<uint8_t> moves;
    std::vector<int32_t> lens;
    int rc = NW_OK;
};

int next_path(void* ctx, const uint8_t** mv, int64_t* n) {
    auto* b = static_cast<PathBatches*>(ctx);
    if (b->pos == b->have) {
        const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(1u << 16, ((uint64_t)256 << 20) / (uint64_t)b->stride));
        if (b->lens.size() < want) {
            b->moves.resize((size_t)(want * (uint64_t)b->stride));
            b->lens.resize((size_t)want);
        }
        uint64_t got = 0;
        b->rc = nw_table_enumerate_paths(b->t, b->next, want, b->moves.data(), b->stride, b->lens.data(), &got,
                                         nullptr);
        if (b->rc != NW_OK) return -1;
        b->have = got;
        b->pos = 0;
        b->next += got;
        if (got == 0) return 0;
    }
    *mv = b->moves.data() + b->pos * (uint64_t)b->stride;
    *n = b->lens[(size_t)b->pos];
    ++b->pos;
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argv[0][0] == '.' && argv[0][1] == '/') g_prog = argv[0] + 2;
    else g_prog = argv[0];
    errno = 0;

    nwh_flags f{};
    const char* infile = nullptr;
    int c;
    char msg[256];
    while ((c = getopt(argc, argv, "cf:hlp:qstu")) != -1) {
        switch (c) {
            case 'c': f.cflag = 1; break;
            case 'f': infile = optarg; break;
            case 'h': usage();
            case 'l': f.lflag = 1; break;
            case 'p': {
                const int nthreads = atoi(optarg);
                if (!(nthreads > 1)) {
                    snprintf(msg, sizeof msg, "num-threads == %d; num-threads must be greater than 1", nthreads);
                    log_err_errno(msg);
                    exit(1);
                }
                break;
            }
            case 'q': f.qflag = 1; break;
            case 's': f.sflag = 1; break;
            case 't': f.tflag = 1; break;
            case 'u': f.uflag = 1; break;
            default: usage();
        }
    }
    const int nops = argc - optind;
    if (nops != 3) {
        snprintf(msg, sizeof msg, "expected %d operands but received%s %d", 3,
                 (nops > 3 || nops == 0) ? "" : " only", nops);
        log_err_errno(msg);
        usage();
    }
    FILE* in = stdin;
    if (infile) {
        in = fopen(infile, "r");
        if (!in) {
            snprintf(msg, sizeof msg, "failed to open %s", infile);
            log_err_errno(msg);
            exit(1);
        }
    }
    char *s1 = nullptr, *s2 = nullptr;
    if (nwh_read_two_sequences(in, g_prog, &s1, &s2) != 0) exit(1);
    const int m = atoi(argv[optind + 0]);
    const int k = atoi(argv[optind + 1]);
    const int d = atoi(argv[optind + 2]);

    // ---- the fill (GPU) -----------------------------------------------------
    // The table stays on the device.  What the reference derives from it on
    // the host comes from the device too: the alignment count for -s
    // (nw_table_count_alignments), the alignments themselves, in print order,
    // for plain / -l output (nw_table_enumerate_paths: each one unranked on
    // its own, the parallel traceback of README:195-200); only -t copies the
    // scores and codes to the host for the table printer.
    const int64_t L1 = (int64_t)strlen(s1), L2 = (int64_t)strlen(s2);
    const bool listing = nwh_needs_traceback(&f) && (!f.qflag || f.lflag);
    const uint32_t mask = (listing || f.sflag || f.tflag ? (uint32_t)NW_OUT_DIRS : 0u) |
                          (f.tflag ? (uint32_t)(NW_OUT_SCORES | NW_OUT_STATS) : 0u);
    nw_table* t = nullptr;
    nw_stats st{};
    uint32_t count = 0;
    std::vector<int32_t> H;
    std::vector<uint8_t> codes;
    int rc = nw_table_create(-1, L1, L2, mask, &t);
    if (rc == NW_OK) rc = nw_table_set_sequences(t, s1, L1, s2, L2);
    if (rc == NW_OK) rc = nw_table_fill(t, m, k, d, mask);
    if (rc == NW_OK) rc = nw_table_stats(t, &st);
    if (rc == NW_OK && f.sflag) rc = nw_table_count_alignments(t, &count);
    if (rc == NW_OK && f.tflag) {
        const int64_t ncell = (L1 + 1) * (L2 + 1);
        H.resize((size_t)ncell);
        codes.resize((size_t)ncell);
        rc = nw_table_copy_scores(t, 0, L1 + 1, H.data());
        if (rc == NW_OK) rc = nw_table_copy_codes(t, 0, L1 + 1, codes.data());
    }
    if (rc != NW_OK) {
        fprintf(stderr, "%s: error: GPU fill failed: %s: %s\n", g_prog, nw_strerror(rc), nw_last_error());
        exit(1);
    }
    PathBatches pb;
    pb.t = t;
    pb.stride = std::max<int64_t>(L1 + L2, 1);
    if (listing) {
        // The device enumeration keeps 8 bytes per cell.  When that does not
        // fit, walk the codes on the host as the reference does
        // (needleman-wunsch.c:209-331) -- slower, same output.
        uint64_t total = 0;
        const int prc = nw_table_enumerate_paths(t, 0, 0, nullptr, pb.stride, nullptr, nullptr, &total);
        if (prc == NW_ERR_OOM) {
            if (codes.empty()) {
                codes.resize((size_t)((L1 + 1) * (L2 + 1)));
                rc = nw_table_copy_codes(t, 0, L1 + 1, codes.data());
                if (rc != NW_OK) {
                    fprintf(stderr, "%s: error: GPU fill failed: %s: %s\n", g_prog, nw_strerror(rc), nw_last_error());
                    exit(1);
                }
            }
            if (nwh_render(s1, s2, &f, f.tflag ? H.data() : nullptr, codes.data(), st.corner,
                           st.greatest_abs_interior, stdout, stderr) != 0) {
                errno = ENOMEM;
                log_err_errno("malloc failed");
                exit(1);
            }
            nw_table_destroy(t);
            free(s1);
            free(s2);
            if (in != stdin) fclose(in);
            return 0;
        }
    }
    const int r = nwh_render_paths(s1, s2, &f, f.tflag ? H.data() : nullptr, f.tflag ? codes.data() : nullptr,
                                   st.corner, st.greatest_abs_interior, count, next_path, &pb, stdout, stderr);
    if (r == -2) {
        fprintf(stderr, "%s: error: GPU traceback failed: %s: %s\n", g_prog, nw_strerror(pb.rc), nw_last_error());
        exit(1);
    }
    if (r != 0) {
        errno = ENOMEM;
        log_err_errno("malloc failed");
        exit(1);
    }
    nw_table_destroy(t);
    free(s1);
    free(s2);
    if (in != stdin) fclose(in);
    return 0;
}
