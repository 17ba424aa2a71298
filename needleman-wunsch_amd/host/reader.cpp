// reader.cpp -- two whitespace-separated sequences from a stream, with the
// behaviour of read-sequences.c:43-122: a token ends at the first isspace()
// byte or EOF; EOF before the second token starts is an error; anything after
// the second token is ignored; a leading whitespace byte makes s1 empty.
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>

#include "nw_host.h"

namespace {

// The reference's log_err (dbg.h:67-71, NDEBUG form): errno 0 prints a
// backspace sequence that erases the trailing ": ".
void log_err(const char* prog, const char* msg) {
    fprintf(stderr, "%s: error: %s: %s\n", prog, msg, errno == 0 ? "\b\b \b" : strerror(errno));
}

// read-sequences.c:43-81.  Returns false after printing the error.  The
// caller holds the stream lock, so bytes come from getc_unlocked (fgetc takes
// the lock per byte, ~10x slower on megabase inputs), and the token grows
// geometrically (std::string) instead of in the reference's 4 KB realloc
// steps (read-sequences.c:66-75).
bool read_token(FILE* in, bool eof_ok, const char* prog, std::string& tok) {
    int c;
    while ((c = getc_unlocked(in)) != EOF && !isspace(c)) tok.push_back((char)c);
    if (ferror(in)) {
        log_err(prog, "fgetc failed");
        return false;
    }
    if (!eof_ok && feof(in)) {
        log_err(prog, "got EOF too early when reading input strings");
        return false;
    }
    return true;
}

char* dup_cstr(const std::string& s) {
    // The reference's strings are C strings: an embedded NUL ends them
    // (strlen, computation.c:158,160).
    const size_t n = strlen(s.c_str());
    char* p = static_cast<char*>(malloc(n + 1));
    if (p) {
        memcpy(p, s.c_str(), n);
        p[n] = '\0';
    }
    return p;
}

}  // namespace

namespace {

int read_two(FILE* in, const char* prog, char** s1, char** s2) {
    std::string a, b;
    if (!read_token(in, false, prog, a)) return -1;
    int c = ' ';
    while (isspace(c)) c = getc_unlocked(in);   // read-sequences.c:90-98
    if (ferror(in)) {
        log_err(prog, "fgetc failed");
        return -1;
    }
    if (feof(in)) {
        log_err(prog, "got EOF too early when reading input strings");
        return -1;
    }
    if (ungetc(c, in) == EOF) {
        log_err(prog, "ungetc failed");
        return -1;
    }
    if (!read_token(in, true, prog, b)) return -1;
    *s1 = dup_cstr(a);
    *s2 = dup_cstr(b);
    if (!*s1 || !*s2) {
        log_err(prog, "malloc failed");
        return -1;
    }
    return 0;
}

}  // namespace

extern "C" int nwh_read_two_sequences(FILE* in, const char* prog, char** s1, char** s2) {
    flockfile(in);
    const int rc = read_two(in, prog, s1, s2);
    funlockfile(in);
    return rc;
}
