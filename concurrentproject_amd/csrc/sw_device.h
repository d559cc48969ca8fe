// sw_device.h -- device helpers shared by the gfx950 kernels (sw_kernels.hip,
// sw_flow2.hip): DPP moves, pair descriptors, buffer resources, and the tagged
// granule hand-off between workgroups.  Not part of the public C-ABI.
#pragma once
#include "sw_internal.h"

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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t bnd_rsrc(const KParams& kp, const PairDesc& pd, int boundary) {
    Granule* base = kp.bnd + pd.bnd_off + (uint64_t)(boundary < 0 ? 0 : boundary) * (uint64_t)pd.m;
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, pd.m * 16, RSRC_FLAGS);
}

// Grouped modes: granule buffer of group boundary b (between groups b and b+1).
// b = -1 is the slab inflow and b = ngroups-1 the slab outflow of a multi-GPU
// column slab (KParams::slab_in / slab_out); without a slab those roles never
// reach a granule load or store, and the resource points at the arena.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t group_rsrc(const KParams& kp, const PairDesc& pd, int b,
                                                             int ngroups) {
    Granule* base = kp.bnd + pd.bnd_off + (uint64_t)(b < 0 ? 0 : b) * (uint64_t)pd.m;
    if (b < 0 && kp.slab_in != nullptr) base = kp.slab_in;
    if (b >= ngroups - 1 && kp.slab_out != nullptr) base = kp.slab_out;
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, pd.m * 16, RSRC_FLAGS);
}
// epoch of the granules crossing group boundary b (slab edges carry the ranks' common epoch)
__device__ __forceinline__ unsigned group_epoch(const KParams& kp, int b, int ngroups) {
    if (b < 0 && kp.slab_in != nullptr) return kp.slab_epoch;
    if (b >= ngroups - 1 && kp.slab_out != nullptr) return kp.slab_epoch;
    return kp.epoch;
}

__device__ __forceinline__ bool granule_ok(const u32x4& g, unsigned epoch, int row) {
    // bitwise, not short-circuit: no exec-mask branch per lane
    return (g.x == epoch) & (g.w == granule_chk(epoch, (int)g.y, (int)g.z, row));
}

template <int C>
__device__ __forceinline__ u32x4 fetch_granules(const __amdgpu_buffer_rsrc_t in_rsrc, int k0, int lane, int m) {
    const int row = k0 + lane;
    const bool live = lane < C && row >= 0 && row < m;
    return __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, live ? (unsigned)row * 16u : OOR, 0, AUX_SC1);
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
__device__ __noinline__ AwaitRes await_slow(__amdgpu_buffer_rsrc_t in_rsrc, u32x4 g, const int row, const bool need,
                                            const unsigned epoch, const long long timeout_ticks, Ctrl* ctrl,
                                            const int strip, const int lane) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool ok = !need || granule_ok(g, epoch, row);
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (!ok) g = __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, (unsigned)row * 16u, 0, AUX_SC1);
        ok = !need || granule_ok(g, epoch, row);
        if (__all(ok)) return AwaitRes{g, 0};
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
            if (lane == 0) {
                atomicOr(&ctrl->error, ERR_TIMEOUT);
                atomicMax(&ctrl->err_item, (unsigned)strip);
            }
            return AwaitRes{g, 1};
        }
    }
}

// Wait until the granules of rows [k0, k0+C) are all published with `epoch` (bounded spin).
template <int C>
__device__ __forceinline__ void await_granules(const KParams& kp, const __amdgpu_buffer_rsrc_t in_rsrc, u32x4& g,
                                               int k0, int lane, int m, int strip, bool& failed, unsigned epoch) {
    if (failed) return;
    const int row = k0 + lane;
    const bool need = lane < C && row >= 0 && row < m;
    const bool ok = (!need) | granule_ok(g, epoch, row);
    if (__all(ok)) return;
    const AwaitRes r = await_slow(in_rsrc, g, row, need, epoch, kp.timeout_ticks, kp.ctrl, strip, lane);
    g = r.g;
    failed = r.failed != 0;
}

__device__ __forceinline__ int lds_load(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void compiler_fence() { __asm__ __volatile__("" ::: "memory"); }

// where a wave's strip inflow comes from / its outflow goes (flow kernels)
enum : int { FLOW_NONE = 0, FLOW_GRANULE = 1, FLOW_LDS = 2 };

#ifndef SW_SPIN_SLEEP
#define SW_SPIN_SLEEP 1      // s_sleep units (64 cycles) between LDS progress polls
#endif

}  // namespace
}  // namespace swmi
