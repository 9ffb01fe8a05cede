// anyseq_io.cpp — host-side alignment-output adapters.
//
// construct_* (import.h:14-27) return the reference's SPARSE layout: both strings
// first blank-filled over [0, n+m), then each traceback step written at i+j+1
// (traceback.impala:14-80), so a diagonal step leaves a blank pair behind it and
// '_' marks a gap.  These turn it into the dense pairwise alignment (what
// print_alignment, alignment_io.cpp:13-38, would print after dropping blanks) and
// into an extended CIGAR (=, X, I, D; query = read, subject = reference: a '_' in
// alQuery consumes a subject base -> D, a '_' in alSubject -> I).
// Host code only: no GPU is touched.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/anyseq.h"

extern "C" {

int64_t anyseq_alignment_dense(const char* alQuery, const char* alSubject, int64_t len, char* outQuery,
                               char* outSubject) {
    if (!alQuery || !alSubject || len < 0) return -1;
    int64_t k = 0;
    for (int64_t i = 0; i < len; ++i) {
        if (alQuery[i] == ' ' && alSubject[i] == ' ') continue;
        if (outQuery) outQuery[k] = alQuery[i];
        if (outSubject) outSubject[k] = alSubject[i];
        ++k;
    }
    return k;
}

int64_t anyseq_alignment_cigar(const char* alQuery, const char* alSubject, int64_t len, char* out, int64_t cap) {
    if (!alQuery || !alSubject || len < 0) return -1;
    int64_t n = 0;   // characters of the full CIGAR (excluding the NUL)
    char op = 0;
    int64_t run = 0;
    char buf[32];
    auto flush = [&]() {
        if (!run) return;
        const int w = snprintf(buf, sizeof buf, "%lld%c", (long long)run, op);
        for (int t = 0; t < w; ++t, ++n)
            if (out && n < cap - 1) out[n] = buf[t];
    };
    for (int64_t i = 0; i < len; ++i) {
        const char a = alQuery[i], b = alSubject[i];
        if (a == ' ' && b == ' ') continue;
        const char o = a == '_' ? 'D' : (b == '_' ? 'I' : (a == b ? '=' : 'X'));
        if (o != op) {
            flush();
            op = o;
            run = 0;
        }
        ++run;
    }
    flush();
    if (out && cap > 0) out[n < cap ? n : cap - 1] = '\0';
    return n;
}

}  // extern "C"
