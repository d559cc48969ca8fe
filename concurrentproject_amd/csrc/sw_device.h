// sw_device.h -- device helpers shared by the gfx950 kernels (sw_kernels.hip,
// sw_flow2.hip): DPP moves, pair descriptors, buffer resources, and the tagged
// granule hand-off between workgroups.  Not part of the public C-ABI.
#pragma once
#include "sw_internal.h"

#include <type_traits>

namespace swmi {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int DPP_WAVE_ROL1 = 0x134;
constexpr int DPP_WAVE_SHR1 = 0x138;
constexpr int DPP_WAVE_SHL1 = 0x130;
constexpr unsigned RSRC_FLAGS = 0x00020000u;   // raw buffer, gfx950 (cdna_hip_programming.md T8)
constexpr int AUX_SC1 = 16;                    // cache policy: sc1 (L1 bypass / write-through)
constexpr unsigned OOR = 0xFFFFFFF0u;          // out-of-range buffer offset: load returns 0, store dropped

constexpr int SENT_DNA = 0x0C0C0C04;   // perm selector: byte 0 -> S0 byte 0 (= 0) => biased score 0 (-128)
constexpr int SENT_BYTE = 0x100;       // never equal to a column byte
constexpr int DEAD_COL_BYTE = 0x200;   // dead (past-the-end) column value, byte mode
constexpr int DEAD = 1 << 29;          // t offset that keeps dead columns out of the max

// The same for a spin loop that keeps its own start time: n counts the polls (one counter per
// strip pass, shared by its loops).
__device__ __forceinline__ bool spin_expired(int& n, long long t0, long long ticks) {
    return ((++n & 63) == 0) && ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks);
}

// Deadline of a spin loop.  The clock (s_memrealtime) is an SMEM round trip far slower than
// the LDS or L2 poll it guards, so it is read only every 64th poll (r05; measured neutral on
// C2, C5 and the column slab).
struct SpinDeadline {
    long long t0;
    long long ticks;
    int n;
    __device__ SpinDeadline(long long start, long long timeout) : t0(start), ticks(timeout), n(0) {}
    __device__ __forceinline__ bool expired() {
        return ((++n & 63) == 0) && ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks);
    }
};

__device__ __forceinline__ int dpp_shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
__device__ __forceinline__ int dpp_rol1(int src) {   // every lane has a source: no 'old', no copy
    return __builtin_amdgcn_mov_dpp(src, DPP_WAVE_ROL1, 0xF, 0xF, true);
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
// v_max3_i32 the compiler cannot split: when it knows two operands are >= 0 it
// emits v_max_i32 + v_max_u32 instead.  A plain VOP3 (hardware interlocked);
// every consumer of the result is compiler-visible, so DPP wait states after it
// are still inserted by the compiler.
__device__ __forceinline__ int vmax3(int a, int b, int c) {
    int d;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// 'A','C','G','T' -> 0,1,2,3  (only used when the host verified the alphabet)
__device__ __forceinline__ int dna_code(unsigned c) { return (int)(((c >> 1) ^ (c >> 2)) & 3u); }

__device__ __forceinline__ PairDesc load_pair(const KParams& kp, int idx) {
    // every field made provably wave-uniform: buffer descriptors built from them
    // must live in SGPRs (no waterfall loops, cdna_hip_programming.md T20)
    const PairDesc raw = kp.pairs[idx];
    PairDesc pd;
    pd.col_off = uniform64(raw.col_off);
    pd.row_off = uniform64(raw.row_off);
    pd.bnd_off = uniform64(raw.bnd_off);
    pd.n = __builtin_amdgcn_readfirstlane(raw.n);
    pd.m = __builtin_amdgcn_readfirstlane(raw.m);
    pd.strips = __builtin_amdgcn_readfirstlane(raw.strips);
    pd.out_idx = __builtin_amdgcn_readfirstlane(raw.out_idx);
    return pd;
}

// last pair whose item_base <= item (uniform binary search)
__device__ __forceinline__ int find_pair(const KParams& kp, int item) {
    int lo = 0, hi = kp.npairs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (kp.item_base[mid] <= item) lo = mid; else hi = mid - 1;
    }
    return __builtin_amdgcn_readfirstlane(lo);
}

// ---- strip / group edges ----------------------------------------------------
// An edge carries one column's (H - G_INIT, E - G_EXT) per row from a producer
// strip to its consumer as tagged 16-B granules.  Row r of the edge lives at
// stream position pos0 + r, in slot (pos0 + r) & mask of the edge's buffer, and
// its checksum covers the position (granule_chk), so a slot still holding an
// older position -- or an older launch's epoch -- never passes the check:
//   * linear edges (one m-row buffer per boundary, write-once): pos0 = 0, mask = ~0;
//   * ring edges (flow2 ring mode, sw_flow2.hip): a boundary's rows stream through a
//     power-of-two ring shared by every round of one block, pos0 = round * m;
//   * slab edges (another GPU's kernel writes them over xGMI): linear, and every
//     load and store of them is system scope (sc0 sc1, AUX_SYS) -- the LLVM AMDGPU
//     memory model's encoding of a relaxed system-scope atomic on gfx942/gfx950,
//     which keeps the access coherent with a peer agent's stores to this memory
//     (fine-grained allocation, sw_slab_alloc).  In-GPU edges stay device scope (sc1).
// The cache policy is a template argument (AUX_SC1 or AUX_SYS), fixed per
// instantiation of a kernel's hand-off loop: a runtime choice would put each load
// and store behind a branch, and the compiler's vmcnt counting across such joins
// falls back to full drains, which costs the prefetch distance (measured: C2
// 4.9 -> 6.9 ms).
struct Edge {
    __amdgpu_buffer_rsrc_t rsrc;
    unsigned pos0;    // stream position of row 0
    unsigned mask;    // slot = (pos0 + row) & mask
    unsigned epoch;   // tag of this launch's granules
};
constexpr int AUX_SYS = 17;   // cache policy sc0|sc1: system scope

__device__ __forceinline__ unsigned edge_off(const Edge& e, int row) { return ((e.pos0 + (unsigned)row) & e.mask) * 16u; }

// the granule of row `row` (store with offset OOR where `st` is false: dropped)
template <int AUX = AUX_SC1>
__device__ __forceinline__ void edge_publish(const Edge& e, int row, bool st, int hg, int eh) {
    u32x4 g;
    g.x = e.epoch;
    g.y = (unsigned)hg;
    g.z = (unsigned)eh;
    g.w = granule_chk(e.epoch, hg, eh, (int)(e.pos0 + (unsigned)row));
    __builtin_amdgcn_raw_buffer_store_b128(g, e.rsrc, st ? edge_off(e, row) : OOR, 0, AUX);
}

// Rows up to 2^27 - 1 (the host rejects longer ones): m * 16 fits the 32-bit record count.
__device__ __forceinline__ Edge linear_edge(Granule* base, int m, unsigned epoch) {
    return Edge{__builtin_amdgcn_make_buffer_rsrc(base, 0, (int)((unsigned)m * 16u), RSRC_FLAGS), 0u, ~0u, epoch};
}

// strip / pairwg kernels: the buffer of strip boundary `boundary` of a pair
__device__ __forceinline__ Edge strip_edge(const KParams& kp, const PairDesc& pd, int boundary) {
    Granule* base = kp.bnd + pd.bnd_off + (uint64_t)(boundary < 0 ? 0 : boundary) * (uint64_t)pd.m;
    return linear_edge(base, pd.m, kp.epoch);
}

// Grouped modes: the edge of group boundary b (between groups b and b+1).
// b = -1 is the slab inflow and b = ngroups-1 the slab outflow of a multi-GPU
// column slab (KParams::slab_in / slab_out, the ranks' common epoch); without a
// slab those roles never reach a granule load or store.  In ring mode
// (kp.ring_rows > 0, one pair, block j runs groups j, j + G, j + 2G, ... for a
// grid of G blocks) boundary b = k*G + j goes through ring j when j < G - 1
// (both groups run in round k) and through the wrap ring otherwise (the
// consumer, block 0, runs it in round k + 1).
__device__ __forceinline__ Edge group_edge(const KParams& kp, const PairDesc& pd, int b, int ngroups) {
    if (b < 0 && kp.slab_in != nullptr) return linear_edge(kp.slab_in, pd.m, kp.slab_epoch);
    if (b >= ngroups - 1 && kp.slab_out != nullptr) return linear_edge(kp.slab_out, pd.m, kp.slab_epoch);
    const int bb = b < 0 ? 0 : b;
    if (kp.ring_rows > 0) {
        const int G = (int)gridDim.x;
        const int j = bb % G, k = bb / G;
        const bool wrap = j == G - 1;
        const int rows = wrap ? kp.wrap_rows : kp.ring_rows;
        Granule* base = kp.bnd + (uint64_t)j * (uint64_t)kp.ring_rows;
        return Edge{__builtin_amdgcn_make_buffer_rsrc(base, 0, rows * 16, RSRC_FLAGS), (unsigned)k * (unsigned)pd.m,
                    (unsigned)rows - 1u, kp.epoch};
    }
    return linear_edge(kp.bnd + pd.bnd_off + (uint64_t)bb * (uint64_t)pd.m, pd.m, kp.epoch);
}

__device__ __forceinline__ bool granule_ok(const u32x4& g, const Edge& e, int row) {
    // bitwise, not short-circuit: no exec-mask branch per lane
    return (g.x == e.epoch) & (g.w == granule_chk(e.epoch, (int)g.y, (int)g.z, (int)(e.pos0 + (unsigned)row)));
}

template <int C, int AUX = AUX_SC1>
__device__ __forceinline__ u32x4 fetch_granules(const Edge& e, int k0, int lane, int m) {
    const int row = k0 + lane;
    const bool live = lane < C && row >= 0 && row < m;
    return __builtin_amdgcn_raw_buffer_load_b128(e.rsrc, live ? edge_off(e, row) : OOR, 0, AUX);
}

// Slow path of await_granules: re-poll until every granule of the chunk is
// published or the deadline passes.  Out of line on purpose: inlined, its
// reload loop leaves outstanding loads in the registers of the join point and
// the compiler then waits for ALL loads (vmcnt(0)) in the fast path, which
// defeats the one-chunk prefetch.
struct AwaitRes {
    u32x4 g;
    int failed;
};
// (The edge goes in as its parts, not as an Edge: a struct argument of a call
// made the compiler keep the caller's buffer resource in VGPRs across the call
// and wrap every granule load of the chunk loop in a waterfall loop.)
template <int AUX>
__device__ __noinline__ AwaitRes await_slow(__amdgpu_buffer_rsrc_t rsrc, unsigned pos0, unsigned mask,
                                            unsigned epoch, u32x4 g, const int row, const bool need,
                                            const long long timeout_ticks, Ctrl* ctrl, const int strip,
                                            const int lane) {
    const Edge e{rsrc, pos0, mask, epoch};
    SpinDeadline dl((long long)__builtin_amdgcn_s_memrealtime(), timeout_ticks);
    bool ok = !need || granule_ok(g, e, row);
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (!ok) g = __builtin_amdgcn_raw_buffer_load_b128(e.rsrc, edge_off(e, row), 0, AUX);
        ok = !need || granule_ok(g, e, row);
        if (__all(ok)) return AwaitRes{g, 0};
        if (dl.expired()) {
            if (lane == 0) {
                atomicOr(&ctrl->error, ERR_TIMEOUT);
                atomicMax(&ctrl->err_item, (unsigned)strip);
            }
            return AwaitRes{g, 1};
        }
    }
}

// Wait until the granules of rows [k0, k0+C) of edge e are all published (bounded spin).
template <int C, int AUX = AUX_SC1>
__device__ __forceinline__ void await_granules(const KParams& kp, const Edge& e, u32x4& g, int k0, int lane, int m,
                                               int strip, bool& failed) {
    if (failed) return;
    const int row = k0 + lane;
    const bool need = lane < C && row >= 0 && row < m;
    const bool ok = (!need) | granule_ok(g, e, row);
    if (__all(ok)) return;
    const AwaitRes r = await_slow<AUX>(e.rsrc, e.pos0, e.mask, e.epoch, g, row, need, kp.timeout_ticks, kp.ctrl,
                                       strip, lane);
    g = r.g;
    failed = r.failed != 0;
}

__device__ __forceinline__ int lds_load(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void compiler_fence() { __asm__ __volatile__("" ::: "memory"); }

// where a wave's strip inflow comes from / its outflow goes (flow kernels)
// (FLOW_PEER: a slab edge, granules to / from another GPU, system scope)
// (FLOW_WRAP: flow2 pair per workgroup, wave 3 -> wave 0 of the next round through an
// LDS buffer holding a whole round's rows, without back-pressure)
enum : int { FLOW_NONE = 0, FLOW_GRANULE = 1, FLOW_LDS = 2, FLOW_PEER = 3, FLOW_WRAP = 4 };
// the cache policy of a granule hand-off kind
__host__ __device__ constexpr int flow_aux(int kind) { return kind == FLOW_PEER ? AUX_SYS : AUX_SC1; }
__host__ __device__ constexpr bool flow_granule(int kind) { return kind == FLOW_GRANULE || kind == FLOW_PEER; }

// A strip's (inflow, outflow) kinds as compile-time constants: calls f(IN{}, OUT{}),
// so every hand-off loop is instantiated per role with unconditional memory ops.
// SET = KINDS_GRANULE (a kernel that never runs a slab): the 9 combinations without
// FLOW_PEER.  The 16-combination body (KINDS_PEER) measured 8 % slower on C2 even
// though the peer roles never ran there (code layout), so slab launches get their own
// kernel.  KINDS_LDS: NONE, LDS and WRAP (the pair-per-workgroup kernel).
enum : int { KINDS_GRANULE = 0, KINDS_PEER = 1, KINDS_LDS = 2 };
template <int SET, class F>
__device__ __forceinline__ void dispatch_kinds(int in_kind, int out_kind, F&& f) {
    constexpr bool PEER = SET == KINDS_PEER, GRAN = SET != KINDS_LDS;
    using K0 = std::integral_constant<int, FLOW_NONE>;
    using K1 = std::integral_constant<int, FLOW_GRANULE>;
    using K2 = std::integral_constant<int, FLOW_LDS>;
    using K3 = std::integral_constant<int, FLOW_PEER>;
    using K4 = std::integral_constant<int, FLOW_WRAP>;
    auto outs = [&](auto in_c) __attribute__((always_inline)) {
        if (out_kind == FLOW_LDS) f(in_c, K2{});
        else if (!GRAN && out_kind == FLOW_WRAP) f(in_c, std::conditional_t<GRAN, K0, K4>{});
        else if (GRAN && out_kind == FLOW_GRANULE) f(in_c, std::conditional_t<GRAN, K1, K0>{});
        else if (PEER && out_kind == FLOW_PEER) f(in_c, std::conditional_t<PEER, K3, K1>{});
        else f(in_c, K0{});
    };
    if (in_kind == FLOW_LDS) outs(K2{});
    else if (!GRAN && in_kind == FLOW_WRAP) outs(std::conditional_t<GRAN, K0, K4>{});
    else if (GRAN && in_kind == FLOW_GRANULE) outs(std::conditional_t<GRAN, K1, K0>{});
    else if (PEER && in_kind == FLOW_PEER) outs(std::conditional_t<PEER, K3, K1>{});
    else outs(K0{});
}

#ifndef SW_SPIN_SLEEP
#define SW_SPIN_SLEEP 1      // s_sleep units (64 cycles) between LDS progress polls
#endif

}  // namespace
}  // namespace swmi
