// Test harness (oracle/_ref only): prints the first record main.cpp would align
// from a file, read by the REFERENCE's own sequence_io.cpp (compiled from
// /root/reference/src by `make -C oracle ref`).  Mirrors main.cpp:182-189:
// make_sequence_reader(path); if has_next(): data = next().data.  Output: one
// JSON-ish line "ok <hex header> <hex data>" or "err <what()>".
#include <cstdio>
#include <exception>
#include <string>

#include "sequence_io.h"

static void hex(const std::string& s) {
    for (unsigned char c : s) std::printf("%02x", c);
}

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        try {
            auto r = anyseq::make_sequence_reader(argv[i]);
            if (r->has_next()) {
                auto seq = r->next();
                std::printf("ok ");
                hex(seq.header);
                std::printf(" ");
                hex(seq.data);
                std::printf(" .\n");
            } else {
                std::printf("none\n");
            }
        } catch (std::exception& e) {
            std::printf("err %s\n", e.what());
        }
    }
    return 0;
}
