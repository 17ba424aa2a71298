// nw_host_internal.h -- shared between the host render units.
#ifndef NW_HOST_INTERNAL_H
#define NW_HOST_INTERNAL_H

#include <cstdint>
#include <cstdio>
#include <vector>

#include "nw_host.h"

namespace nwh {

struct Render {
    const char* s1;
    const char* s2;
    int64_t L1, L2;
    nwh_flags f;
    const int32_t* H;
    const uint8_t* codes;
    FILE* out;
    FILE* err;
};

// ANSI formats of format.h:42-102 (set only when -c).
enum Fmt { TOP_STRING, SIDE_STRING, OPT_PATH, MATCH_ARROW, MISMATCH_ARROW, GAP_ARROW, MATCH_CHAR, MISMATCH_CHAR,
           GAP_CHAR };
void set_fmt(const Render& r, Fmt f);
void reset_fmt(const Render& r);

// Print one alignment (X, Y hold it reversed, last index n).
void print_alignment(const Render& r, const char* X, const char* Y, int64_t n);

// The depth-first enumeration; fills the per-cell walk state (OPT bit = 1<<8
// marks cells on an optimal path) and counts the alignments.
bool walk_alignments(const Render& r, std::vector<uint16_t>& cell, unsigned& solutions);

constexpr uint16_t WALK_OPT = 1 << 8;

}  // namespace nwh

#endif
