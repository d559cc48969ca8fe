// sw_db.hip -- FASTA databases and query x database scoring.
//
// The reference reaches databases only through the external CUDASW++4 tool
// (timing.sh:3-8: `makedb SwissProt.fasta benchdb/sp`, then
// `align --query q.fa --db benchdb/sp`; Makefile_CUDASW4.mak:44-56), which is
// not vendored.  This module gives the same workflow over this engine: the
// FASTA parse and the binary database file (host only, sw_db_host.cpp), and
// searches that score one query against every record with ONE batch launch
// (sw_score_batch_device) over residues kept resident in HBM.  Scoring is the reference's (byte equality + affine
// gaps, main.cpp:28-66), so every score equals SmithWatermanScore of the pair.
//
// Layout: all records' residues back to back in one arena (host, and once per
// device), the query in a tail slot of the device arena behind them.  Records
// are launched longest first (the work-claiming kernels take pairs in order, so
// the long tail starts early); scores come back in record order.
#include "sw_internal.h"
#include "sw_db_host.h"
#include "../../include/algoGPU.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

namespace swmi {
namespace {

#define DBCHK(expr)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            char m_[256];                                                                    \
            std::snprintf(m_, sizeof m_, "%s failed: %s", #expr, hipGetErrorString(e_));     \
            report_error(m_);                                                                \
            return -1;                                                                       \
        }                                                                                    \
    } while (0)

// the database's device arena on the current device, with two query slots of at least qlen
// bytes behind the residues and two score buffers (sw_db_search_db alternates them).  A new
// arena is built in locals and committed to the Dev entry only when every step succeeded (a
// failed copy must not leave an arena that looks ready).
int device_arena(sw_db* db, int qlen, sw_db::Dev** out) {
    int d = 0;
    DBCHK(hipGetDevice(&d));
    sw_db::Dev& v = db->dev[d];
    if (!v.arena || v.qcap < (size_t)qlen) {
        if (v.arena) DBCHK(hipFree(v.arena));
        if (v.scores) DBCHK(hipFree(v.scores));
        v.arena = nullptr;
        v.scores = nullptr;
        v.qcap = 0;
        const size_t qcap = (std::max<size_t>((size_t)qlen + (size_t)qlen / 4, 4096) + 15) / 16 * 16;
        unsigned char* arena = nullptr;
        int* scores = nullptr;
        hipError_t e = hipMalloc((void**)&arena, db->res.size() + 2 * qcap);
        if (e == hipSuccess) e = hipMalloc((void**)&scores, 2 * std::max<size_t>(db->len.size(), 1) * sizeof(int));
        if (e == hipSuccess && !db->res.empty())
            e = hipMemcpy(arena, db->res.data(), db->res.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (arena) (void)hipFree(arena);
            if (scores) (void)hipFree(scores);
            char m[256];
            std::snprintf(m, sizeof m, "database device arena: %s", hipGetErrorString(e));
            report_error(m);
            return -1;
        }
        v.arena = arena;
        v.scores = scores;
        v.qcap = qcap;
    }
    *out = &v;
    return 0;
}

bool all_dna(const unsigned char* p, size_t n) {
    unsigned bad = 0;
    for (size_t i = 0; i < n; ++i) bad |= !(p[i] == 'A' || p[i] == 'C' || p[i] == 'G' || p[i] == 'T');
    return bad == 0;
}

// the engine's int32 score range, checked here so an error names the record
int check_range(const sw_db* db, int qlen) {
    int match = 1;
    sw_get_params(&match, nullptr, nullptr, nullptr);
    for (size_t r = 0; r < db->len.size(); ++r) {
        if ((long long)std::min(qlen, db->len[r]) * std::max(match, 1) >= (1LL << 28)) {
            char m[160];
            std::snprintf(m, sizeof m, "record %d: score range exceeds the int32 engine (min length * MATCH >= 2^28)", (int)r);
            report_error(m);
            return -1;
        }
    }
    return 0;
}

// the alphabet the engine would scan for on the device (its alphabet_kernel), known on the host:
// the records' once per database, the query's per search
int search_flags(sw_db* db, const unsigned char* query, int qlen) {
    if (db->dna < 0) db->dna = all_dna(db->res.data(), db->res.size()) ? 1 : 0;
    return db->dna == 1 && all_dna(query, (size_t)qlen) ? SW_FLAG_DNA : SW_FLAG_BYTES;
}

// Launch one query's search on `stream` (null: synchronous) into score buffer / query slot `slot`;
// records are launched longest first (b_off / blen in db->order)
int launch_query(sw_db* db, sw_db::Dev* v, const unsigned char* query, int qlen, int slot, hipStream_t stream,
                 const std::vector<int64_t>& b_off, const std::vector<int>& blen) {
    const int nrec = (int)db->len.size();
    const int64_t qoff = (int64_t)db->res.size() + (int64_t)slot * (int64_t)v->qcap;
    if (qlen > 0) {
        if (stream) DBCHK(hipMemcpyAsync(v->arena + qoff, query, (size_t)qlen, hipMemcpyHostToDevice, stream));
        else DBCHK(hipMemcpy(v->arena + qoff, query, (size_t)qlen, hipMemcpyHostToDevice));
    }
    std::vector<int64_t> a_off((size_t)nrec, qoff);
    std::vector<int> alen((size_t)nrec, qlen);
    return sw_score_batch_device(v->arena, a_off.data(), alen.data(), b_off.data(), blen.data(), nrec,
                                 v->scores + (size_t)slot * (size_t)nrec, search_flags(db, query, qlen), stream);
}

void record_order(const sw_db* db, std::vector<int64_t>& b_off, std::vector<int>& blen) {
    const size_t nrec = db->len.size();
    b_off.resize(nrec);
    blen.resize(nrec);
    for (size_t k = 0; k < nrec; ++k) {   // slot k scores record order[k]
        const int r = db->order[k];
        b_off[k] = db->off[r];
        blen[k] = db->len[r];
    }
}

// qslot: room to reserve for the query (>= qlen)
int search(sw_db* db, const unsigned char* query, int qlen, int* scores_out, int qslot) {
    const int nrec = (int)db->len.size();
    if (nrec == 0) return 0;
    if (check_range(db, qlen)) return -1;
    sw_db::Dev* v = nullptr;
    if (device_arena(db, std::max(qlen, qslot), &v)) return -1;
    std::vector<int64_t> b_off;
    std::vector<int> blen;
    record_order(db, b_off, blen);
    if (launch_query(db, v, query, qlen, 0, nullptr, b_off, blen)) return -1;
    std::vector<int> got((size_t)nrec);
    DBCHK(hipMemcpy(got.data(), v->scores, (size_t)nrec * sizeof(int), hipMemcpyDeviceToHost));
    for (int k = 0; k < nrec; ++k) scores_out[db->order[k]] = got[k];
    return 0;
}

// Every query of `queries` against the database, pipelined on the database's own stream: query q
// is planned and launched into slot q % 2 (its query slot, score buffer and pinned host copy) while
// query q - 1 runs; slot q % 2's scores (query q - 2) are collected first.  The host's per-search
// planning (~1.5 ms for 65536 records) then overlaps the kernels instead of adding to them.
int search_many(sw_db* db, const sw_db* queries, int* scores_out) {
    const int nrec = (int)db->len.size(), nq = (int)queries->len.size();
    if (nrec == 0 || nq == 0) return 0;
    int longest = 0;
    for (int l : queries->len) longest = std::max(longest, l);
    if (check_range(db, longest)) return -1;
    sw_db::Dev* v = nullptr;
    if (device_arena(db, longest, &v)) return -1;
    if (!v->stream) {
        hipStream_t st = nullptr;
        DBCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        v->stream = st;
    }
    for (int k = 0; k < 2; ++k)
        if (!v->done[k]) {
            hipEvent_t ev = nullptr;
            DBCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            v->done[k] = ev;
        }
    if (!v->hscores) DBCHK(hipHostMalloc((void**)&v->hscores, 2 * (size_t)nrec * sizeof(int), hipHostMallocDefault));
    hipStream_t st = (hipStream_t)v->stream;
    std::vector<int64_t> b_off;
    std::vector<int> blen;
    record_order(db, b_off, blen);
    const auto collect = [&](int q) -> int {   // query q's scores, from its slot's pinned copy
        const int slot = q & 1;
        DBCHK(hipEventSynchronize((hipEvent_t)v->done[slot]));
        const int* got = v->hscores + (size_t)slot * (size_t)nrec;
        int* out = scores_out + (size_t)q * (size_t)nrec;
        for (int k = 0; k < nrec; ++k) out[db->order[k]] = got[k];
        return 0;
    };
    for (int q = 0; q < nq; ++q) {
        const int slot = q & 1;
        if (q >= 2 && collect(q - 2)) return -1;
        if (launch_query(db, v, queries->res.data() + queries->off[q], queries->len[q], slot, st, b_off, blen)) return -1;
        DBCHK(hipMemcpyAsync(v->hscores + (size_t)slot * (size_t)nrec, v->scores + (size_t)slot * (size_t)nrec,
                             (size_t)nrec * sizeof(int), hipMemcpyDeviceToHost, st));
        DBCHK(hipEventRecord((hipEvent_t)v->done[slot], st));
    }
    for (int q = std::max(0, nq - 2); q < nq; ++q)
        if (collect(q)) return -1;
    return sw_stream_status(st);   // a kernel's hand-off timeout surfaces here
}

}  // namespace
}  // namespace swmi

using namespace swmi;

extern "C" {

int sw_db_search(sw_db* db, const unsigned char* query, int qlen, int* scores_out) {
    if (!db || qlen < 0 || (qlen > 0 && !query) || (!db->len.empty() && !scores_out)) {
        report_error("sw_db_search: invalid arguments");
        return -1;
    }
    std::lock_guard<std::mutex> g(db->mu);
    return search(db, query, qlen, scores_out, qlen);
}

int sw_db_search_db(sw_db* db, const sw_db* queries, int* scores_out) {
    if (!db || !queries || (!db->len.empty() && !queries->len.empty() && !scores_out)) {
        report_error("sw_db_search_db: invalid arguments");
        return -1;
    }
    std::lock_guard<std::mutex> g(db->mu);
    return search_many(db, queries, scores_out);
}

void sw_db_close(sw_db* db) {
    if (!db) return;
    int cur = 0;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    for (auto& kv : db->dev) {
        if (hipSetDevice(kv.first) != hipSuccess) continue;
        if (kv.second.stream) (void)hipStreamSynchronize((hipStream_t)kv.second.stream);
        if (kv.second.arena) (void)hipFree(kv.second.arena);
        if (kv.second.scores) (void)hipFree(kv.second.scores);
        if (kv.second.hscores) (void)hipHostFree(kv.second.hscores);
        for (void* ev : kv.second.done)
            if (ev) (void)hipEventDestroy((hipEvent_t)ev);
        if (kv.second.stream) (void)hipStreamDestroy((hipStream_t)kv.second.stream);
    }
    if (have && !db->dev.empty()) (void)hipSetDevice(cur);
    delete db;
}

}  // extern "C"
