// traceback.cpp -- enumerate every optimal alignment from the direction codes.
//
// Behaviour of construct_alignments() (needleman-wunsch.c:356-388) and its
// iterative walk (needleman-wunsch.c:209-331): a depth-first walk from the
// bottom-right cell that tries the diagonal, then the left, then the up
// predecessor of each cell, prints an alignment (through print_alignment) every
// time it reaches (0, 0), and marks visited cells for the table printer.  The
// reference keeps 32 bytes of walk state per cell (walk-table.h:44-54); here a
// cell is 16 bits derived from the 4-bit direction code of the GPU fill.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nw_host_internal.h"

namespace nwh {

namespace {
constexpr uint16_t F_DIAG = 1, F_UP = 2, F_LEFT = 4;            // direction flags
constexpr uint16_t D_DIAG = 8, D_UP = 16, D_LEFT = 32;          // "done" marks
constexpr uint16_t SRC_SHIFT = 6, SRC_MASK = 3 << SRC_SHIFT;    // src_direction
constexpr uint16_t SRC_UP = 1, SRC_LEFT = 2, SRC_DIAG = 3;
constexpr uint16_t OPT = 1 << 8;                                // in_optimal_path
constexpr uint16_t ALL_DONE = D_DIAG | D_UP | D_LEFT;

inline uint16_t fresh(uint16_t flags) {
    // done == !flag for every direction (computation.c:96-120,
    // needleman-wunsch.c:486-503): a cell's walk starts untried.
    return (uint16_t)(flags | ((flags & F_DIAG) ? 0 : D_DIAG) | ((flags & F_UP) ? 0 : D_UP) |
                      ((flags & F_LEFT) ? 0 : D_LEFT));
}
}  // namespace

bool walk_alignments(const Render& r, std::vector<uint16_t>& cell, unsigned& solutions) {
    const int64_t M = r.L1 + 1, N = r.L2 + 1;
    cell.assign((size_t)(M * N), 0);
    for (int64_t c = 0; c < M * N; ++c) cell[c] = fresh(r.codes[c] & 7);
    const int64_t cap = M + N + 1;
    std::vector<char> X((size_t)cap), Y((size_t)cap);
    auto at = [&](int64_t i, int64_t j) -> uint16_t& { return cell[(size_t)(i * N + j)]; };

    const int64_t si = M - 1, sj = N - 1;
    int64_t i = si, j = sj, n = 0;
    solutions = 0;
    while (!(i == si && j == sj && (at(i, j) & ALL_DONE) == ALL_DONE)) {
        uint16_t& w = at(i, j);
        if (r.f.tflag) w |= OPT;
        if (i == 0 && j == 0) {
            if (!r.f.qflag || r.f.lflag) print_alignment(r, X.data(), Y.data(), n - 1);
            ++solutions;
        }
        if ((w & ALL_DONE) == ALL_DONE) {
            // every predecessor tried: re-arm this cell and step back
            const uint16_t src = (w & SRC_MASK) >> SRC_SHIFT;
            w = (uint16_t)((w & ~(ALL_DONE | SRC_MASK)) | (fresh(w & 7) & ALL_DONE) | (w & SRC_MASK));
            if (src == SRC_UP) {
                j += 1;
                at(i, j) |= D_UP;
            } else if (src == SRC_LEFT) {
                i += 1;
                at(i, j) |= D_LEFT;
            } else if (src == SRC_DIAG) {
                i += 1;
                j += 1;
                at(i, j) |= D_DIAG;
            } else {
                return false;   // unreachable() in the reference
            }
            n -= 1;
        } else {
            uint16_t src;
            if ((w & F_DIAG) && !(w & D_DIAG)) {
                X[n] = r.s1[i - 1];
                Y[n] = r.s2[j - 1];
                i -= 1;
                j -= 1;
                src = SRC_DIAG;
            } else if ((w & F_LEFT) && !(w & D_LEFT)) {
                X[n] = r.s1[i - 1];
                Y[n] = '-';
                i -= 1;
                src = SRC_LEFT;
            } else {
                X[n] = '-';
                Y[n] = r.s2[j - 1];
                j -= 1;
                src = SRC_UP;
            }
            uint16_t& nx = at(i, j);
            nx = (uint16_t)((nx & ~SRC_MASK) | (src << SRC_SHIFT));
            n += 1;
        }
    }
    return true;
}

}  // namespace nwh
