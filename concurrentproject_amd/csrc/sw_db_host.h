// sw_db_host.h -- the host side of the FASTA databases:
// the database structure and its parsers, plain C++ with no HIP, so that they
// build both into libswmi355.so and into the sanitizer test binary
// (make -C concurrentproject_amd/csrc asan; tests/test_sanitize.py).
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

struct sw_db {
    std::vector<unsigned char> res;     // residues of every record, back to back
    std::vector<int64_t> off;           // record i: res[off[i], off[i] + len[i])
    std::vector<int> len;
    std::vector<std::string> header;    // the '>' line without '>' and line end
    std::vector<int> order;             // record indices, longest first
    int dna = -1;                       // every residue in {A,C,G,T}: 1 / 0, -1 not scanned yet (sw_db.hip)
    struct Dev {
        unsigned char* arena = nullptr; // residues, then two query slots of qcap bytes
        size_t qcap = 0;
        int* scores = nullptr;          // two score buffers of the record count (sw_db_search_db alternates)
        int* hscores = nullptr;         // pinned host copies of both
        void* stream = nullptr;         // sw_db_search_db's hipStream_t (queries pipelined on it; sw_db.hip)
        void* done[2] = {nullptr, nullptr};   // its hipEvent_t per score buffer
    };
    std::map<int, Dev> dev;             // per device ordinal (sw_db.hip)
    std::mutex mu;                      // one search at a time per database
};

namespace swmi {
// sets the calling thread's sw_last_error() text (sw_engine.hip)
void report_error(const char* msg);

sw_db* parse_fasta(const char* text, size_t nbytes);
sw_db* parse_binary(const std::vector<char>& b);
bool read_file(const char* path, std::vector<char>& buf);
}  // namespace swmi
