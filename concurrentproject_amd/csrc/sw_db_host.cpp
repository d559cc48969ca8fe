// sw_db_host.cpp -- FASTA / database-file parsing and the host-only sw_db_* entry
// points (include/algoGPU.h).  No HIP here: the same file is compiled into
// libswmi355.so and, with -fsanitize=address,undefined, into the sanitizer test
// binary that feeds it malformed files (tests/test_sanitize.py).  The searches,
// which need the device, are in sw_db.hip.
//
// The reference reaches databases only through the external CUDASW++4 tool
// (timing.sh:3-8: `makedb SwissProt.fasta benchdb/sp`, then
// `align --query q.fa --db benchdb/sp`; Makefile_CUDASW4.mak:44-56), which is
// not vendored; this is the same workflow over this engine.
#include "sw_db_host.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>

#include "../../include/algoGPU.h"

namespace swmi {
namespace {

constexpr char kMagic[8] = {'S', 'W', 'M', 'I', 'D', 'B', '0', '1'};

void finish(sw_db* db) {
    db->order.resize(db->len.size());
    std::iota(db->order.begin(), db->order.end(), 0);
    std::stable_sort(db->order.begin(), db->order.end(), [db](int a, int b) { return db->len[a] > db->len[b]; });
}

bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

}  // namespace

// FASTA: a record starts at a line beginning with '>' (its header is the rest of
// the line); the following lines up to the next header are its residues, with
// whitespace dropped.  Lines beginning with ';' are comments.  Text before the
// first header that is not blank is an error.
sw_db* parse_fasta(const char* text, size_t nbytes) {
    sw_db* db = new sw_db();
    size_t i = 0;
    bool in_record = false;
    while (i < nbytes) {
        size_t e = i;
        while (e < nbytes && text[e] != '\n') ++e;
        const char* line = text + i;
        size_t ll = e - i;
        if (ll > 0 && line[0] == '>') {
            size_t hl = ll - 1;
            while (hl > 0 && (line[hl] == '\r')) --hl;
            db->header.emplace_back(line + 1, hl);
            db->off.push_back((int64_t)db->res.size());
            db->len.push_back(0);
            in_record = true;
        } else if (ll > 0 && line[0] == ';') {
            // comment line
        } else {
            size_t before = db->res.size();
            for (size_t k = 0; k < ll; ++k) {
                const unsigned char c = (unsigned char)line[k];
                if (!is_space(c)) db->res.push_back(c);
            }
            const size_t added = db->res.size() - before;
            if (added > 0) {
                if (!in_record) {
                    delete db;
                    report_error("FASTA: sequence data before the first '>' header");
                    return nullptr;
                }
                const long long nl = (long long)db->len.back() + (long long)added;
                if (nl > 0x7fffffffLL) {
                    delete db;
                    report_error("FASTA: a record is longer than 2^31 - 1 residues");
                    return nullptr;
                }
                db->len.back() = (int)nl;
            }
        }
        i = e + 1;
    }
    if (db->len.size() > 0x7fffffffULL) {
        delete db;
        report_error("FASTA: more than 2^31 - 1 records");
        return nullptr;
    }
    finish(db);
    return db;
}

bool read_file(const char* path, std::vector<char>& buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    char tmp[1 << 16];
    size_t r;
    while ((r = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    const bool ok = !std::ferror(f);
    std::fclose(f);
    return ok;
}

// binary database: magic, u64 count, u64 residues, u64 header bytes, then per
// record {i64 off, i32 len, i32 header length}, the headers, the residues
sw_db* parse_binary(const std::vector<char>& b) {
    auto fail = [](sw_db* db) -> sw_db* {
        delete db;
        report_error("database file is truncated or inconsistent");
        return nullptr;
    };
    sw_db* db = new sw_db();
    size_t p = 8;
    auto get = [&](void* dst, size_t n) {
        if (p > b.size() || n > b.size() - p) return false;
        std::memcpy(dst, b.data() + p, n);
        p += n;
        return true;
    };
    uint64_t count = 0, nres = 0, hbytes = 0;
    if (!get(&count, 8) || !get(&nres, 8) || !get(&hbytes, 8) || count > 0x7fffffffULL) return fail(db);
    if (count * 16 > b.size()) return fail(db);
    std::vector<int> hl((size_t)count);
    db->off.resize((size_t)count);
    db->len.resize((size_t)count);
    uint64_t hsum = 0;
    for (uint64_t k = 0; k < count; ++k) {
        if (!get(&db->off[k], 8) || !get(&db->len[k], 4) || !get(&hl[k], 4)) return fail(db);
        // off + len compared without a sum that could wrap (off, len >= 0 here)
        if (db->off[k] < 0 || db->len[k] < 0 || hl[k] < 0 || (uint64_t)db->off[k] > nres ||
            (uint64_t)db->len[k] > nres - (uint64_t)db->off[k])
            return fail(db);
        hsum += (uint64_t)hl[k];
    }
    // sizes compared without sums that could wrap: the headers and then exactly
    // nres residue bytes must fill the rest of the file
    if (hsum != hbytes || p > b.size() || hbytes > b.size() - p || nres != b.size() - p - hbytes) return fail(db);
    db->header.resize((size_t)count);
    for (uint64_t k = 0; k < count; ++k) {
        if ((size_t)hl[k] > b.size() - p) return fail(db);
        db->header[k].assign(b.data() + p, (size_t)hl[k]);
        p += (size_t)hl[k];
    }
    if (b.size() - p != nres) return fail(db);
    db->res.assign(b.begin() + (ptrdiff_t)p, b.end());
    finish(db);
    return db;
}

}  // namespace swmi

using namespace swmi;

extern "C" {

sw_db* sw_db_from_fasta(const char* text, long long nbytes) {
    if (nbytes < 0 || (nbytes > 0 && !text)) {
        report_error("sw_db_from_fasta: invalid arguments");
        return nullptr;
    }
    return parse_fasta(text, (size_t)nbytes);
}

sw_db* sw_db_open(const char* path) {
    std::vector<char> buf;
    if (!path || !read_file(path, buf)) {
        report_error("sw_db_open: cannot read the file");
        return nullptr;
    }
    if (buf.size() >= 8 && std::memcmp(buf.data(), kMagic, 8) == 0) return parse_binary(buf);
    return parse_fasta(buf.data(), buf.size());
}

int sw_db_save(const sw_db* db, const char* path) {
    if (!db || !path) {
        report_error("sw_db_save: invalid arguments");
        return -1;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        report_error("sw_db_save: cannot create the file");
        return -1;
    }
    const uint64_t count = db->len.size(), nres = db->res.size();
    uint64_t hbytes = 0;
    for (const auto& h : db->header) hbytes += h.size();
    bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(&count, 8, 1, f) == 1 &&
              std::fwrite(&nres, 8, 1, f) == 1 && std::fwrite(&hbytes, 8, 1, f) == 1;
    for (uint64_t k = 0; ok && k < count; ++k) {
        const int hl = (int)db->header[k].size();
        ok = std::fwrite(&db->off[k], 8, 1, f) == 1 && std::fwrite(&db->len[k], 4, 1, f) == 1 &&
             std::fwrite(&hl, 4, 1, f) == 1;
    }
    for (uint64_t k = 0; ok && k < count; ++k)
        ok = db->header[k].empty() || std::fwrite(db->header[k].data(), 1, db->header[k].size(), f) == db->header[k].size();
    if (ok && nres) ok = std::fwrite(db->res.data(), 1, nres, f) == nres;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) report_error("sw_db_save: write failed");
    return ok ? 0 : -1;
}

int sw_db_count(const sw_db* db) { return db ? (int)db->len.size() : -1; }

long long sw_db_residues(const sw_db* db) { return db ? (long long)db->res.size() : -1; }

int sw_db_record(const sw_db* db, int i, const unsigned char** seq, int* len, const char** header) {
    if (!db || i < 0 || i >= (int)db->len.size()) {
        report_error("sw_db_record: no such record");
        return -1;
    }
    if (seq) *seq = db->res.data() + db->off[i];
    if (len) *len = db->len[i];
    if (header) *header = db->header[i].c_str();
    return 0;
}

}  // extern "C"
