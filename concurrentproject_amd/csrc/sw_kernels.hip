// sw_kernels.hip -- hand-written gfx950 (CDNA4) kernels for the affine-gap
// Smith-Waterman score.  Replaces the per-anti-diagonal kernels of the
// reference (simpleGPU.cu:76-107 DPMatrices, cudaLazy.cu:21-56 sw_kernel_diag,
// cudaSmithM.cu:87-126 kernel_compute_diagonal, SmithDiagonalGPU.cu:40-67) with
// ONE persistent launch that never materialises H/E/F in HBM.
//
// Recurrence (main.cpp:54-66; q = column sequence, d = row sequence):
//   E[i][j] = max(E[i][j-1] - G_EXT, H[i][j-1] - G_INIT)
//   F[i][j] = max(F[i-1][j] - G_EXT, H[i-1][j] - G_INIT)
//   H[i][j] = max(0, H[i-1][j-1] + s(q[j-1], d[i-1]), E[i][j], F[i][j])
//   score   = max H
// computed in an exactly equivalent "clamped" form (Arithmetic):
//   * E and F are kept as max(E,0), max(F,0): H never sees a negative E/F
//     because of the 0 floor, and clamping commutes with the recurrence when
//     G_EXT >= 0, so every H is bit-identical;
//   * the running maximum is taken over t = H[i-1][j-1] + s only: every H that
//     comes from E or F is <= some earlier H (penalties >= 0), so max H ==
//     max(0, max t).
//
// Work decomposition (Kernels):
//   * a WAVE owns a strip of 64*W consecutive columns; lane l holds columns
//     [l*W, l*W+W) of the strip in registers;
//   * the wave sweeps the strip's rows as an anti-diagonal wavefront: at step k
//     every (lane, position) computes the cell of anti-diagonal k, so the W
//     cells of a lane are independent (ILP) and the left neighbour of position
//     0 is the previous step's position W-1 of lane l-1: ONE wave_shr:1 DPP
//     move per flowing quantity (H-G_INIT, E-G_EXT, row code) per step;
//   * the strip's left column enters at lane 0 and its right column leaves at
//     lane 63 through one I/O register per quantity that is rotated by
//     wave_rol:1 every step (lane 0 consumes the next inflow, lane 63 collects
//     the outflow), so C rows of hand-off cost one load and one store per lane;
//   * three grid organisations share that strip pass:
//       sw_strip_kernel  -- independent waves claim (pair, strip) items in
//                           order; strips hand off through tagged granules;
//       sw_chain_kernel  -- a single long pair: a workgroup's 4 waves run 4
//                           consecutive strips in lock step (barrier per
//                           chunk) with LDS-ring hand-offs, granules only
//                           between workgroups;
//       sw_pairwg_kernel -- batches: a workgroup's 4 waves interleave one
//                           pair's strips (wave w: strips w, w+4, ...), so
//                           every granule hand-off has a whole strip pass of
//                           slack and all 4 chains are co-resident.
//   * strip boundaries cross CUs as tagged 16-byte granules (write-through sc1
//     stores, sc1 polls; no fences); work is claimed strictly in order or
//     assigned so that every producer is resident: no co-residency assumption
//     beyond the workgroup, no deadlock, any grid size.
#include <type_traits>

#include "sw_device.h"

namespace swmi {

namespace {


// ---------------------------------------------------------------------------
// Per-lane state of one strip pass (W columns per lane).
// ---------------------------------------------------------------------------
#define SW_PRAGMA_(x) _Pragma(#x)
#define SW_PRAGMA(x) SW_PRAGMA_(x)
#ifndef SW_STRIP_UNROLL
#define SW_STRIP_UNROLL 2   // step pairs per rolled iteration of the int32 strip chunk
#endif

template <int W, bool DNA>
struct Strip {
    int prof[W], tb[W];                     // column profile / bias (fixed for the strip)
    int hgA[W], hgB[W], eh[W], r[W], fh[W]; // DP state, see step()
    int L0, M, IOH, IOE, IOR;

    __device__ __forceinline__ void setup(const KParams& kp, const PairDesc& pd, int strip, int lane) {
        constexpr int SW = 64 * W;
        const int go = kp.gap_init, ge = kp.gap_ext;
        const unsigned char* colseq = kp.seq + pd.col_off;
#pragma unroll
        for (int p = 0; p < W; ++p) {
            const int c = strip * SW + lane * W + p;
            if (c < pd.n) {
                const unsigned ch = colseq[c];
                if constexpr (DNA) {
                    const int code = dna_code(ch);
                    prof[p] = (int)(code == 0 ? kp.prof[0] : code == 1 ? kp.prof[1] : code == 2 ? kp.prof[2] : kp.prof[3]);
                    tb[p] = go - 128;
                } else {
                    prof[p] = (int)ch;
                    tb[p] = go;
                }
            } else {
                prof[p] = DNA ? 0 : DEAD_COL_BYTE;
                tb[p] = -DEAD;
            }
        }
        const int sent = DNA ? SENT_DNA : SENT_BYTE;
#pragma unroll
        for (int p = 0; p < W; ++p) {   // everything starts at the border (H = E = F = 0)
            hgA[p] = -go; hgB[p] = -go; eh[p] = -ge; fh[p] = -ge; r[p] = sent;
        }
        L0 = -go; M = 0; IOH = -go; IOE = -ge; IOR = sent;
    }

    // One anti-diagonal step for the W positions of the lane.
    //   hgCur : on entry H-G_INIT two steps ago (diagonal source); on exit this step's
    //   hgPrev: H-G_INIT of the previous step (left source for p>0, up source for F)
    //   eh, r : E-G_EXT and row code of the previous step, updated in place
    //   fh    : F-G_EXT of the previous step (own column), updated in place
    // Positions run from W-1 down to 0 so the in-place arrays still hold the
    // previous step's p-1 when p reads it.  The I/O registers are rotated first so
    // the inflow DPPs can take them as their (dying) 'old' operand: no copies.
    __device__ __forceinline__ void step(int (&hgCur)[W], const int (&hgPrev)[W], const bool l63, const int go,
                                         const int ge, const int ma, const int mi) {
        const int ioh = dpp_rol1(IOH), ioe = dpp_rol1(IOE), ior = dpp_rol1(IOR);
        const int hgL0 = dpp_shr1(IOH, hgPrev[W - 1]);
        const int ehL0 = dpp_shr1(IOE, eh[W - 1]);
        const int rL0 = dpp_shr1(IOR, r[W - 1]);
#pragma unroll
        for (int p = W - 1; p >= 0; --p) {
            const int q = p > 0 ? p - 1 : 0;
            const int hgL = p > 0 ? hgPrev[q] : hgL0;
            const int ehL = p > 0 ? eh[q] : ehL0;
            const int rL = p > 0 ? r[q] : rL0;
            const int hgD = p > 0 ? hgCur[q] : L0;
            int s;
            if constexpr (DNA) {
                s = (int)__builtin_amdgcn_perm(0u, (unsigned)prof[p], (unsigned)rL);   // biased byte
            } else {
                s = (rL == prof[p]) ? ma : mi;
            }
            const int t = hgD + s + tb[p];               // H[i-1][j-1] + s(q_j, d_i)   (v_add3_u32)
            const int E = max3i(ehL, hgL, 0);            // clamped E
            const int F = max3i(fh[p], hgPrev[p], 0);    // clamped F
            const int H = vmax3(t, E, F);
            M = max(M, t);
            hgCur[p] = H - go;
            eh[p] = E - ge;
            fh[p] = F - ge;
            r[p] = rL;
        }
        L0 = hgL0;
        IOH = l63 ? hgCur[W - 1] : ioh;   // lane 63 <- this step's right-edge output
        IOE = l63 ? eh[W - 1] : ioe;
        IOR = ior;
    }

    template <int C>
    __device__ __forceinline__ void run(const bool l63, const int go, const int ge, const int ma, const int mi) {
        SW_PRAGMA(unroll SW_STRIP_UNROLL)
        for (int s = 0; s < C; s += 2) {
            step(hgA, hgB, l63, go, ge, ma, mi);
            step(hgB, hgA, l63, go, ge, ma, mi);
        }
    }

    // inflow of the next C rows into lanes [0, C)
    __device__ __forceinline__ void feed(int lane, int C, int hg_in, int eh_in, int code) {
        if (lane < C) { IOH = hg_in; IOE = eh_in; IOR = code; }
    }

    __device__ __forceinline__ void commit_max(const KParams& kp, const PairDesc& pd, int lane) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) M = max(M, __shfl_xor(M, off));
        if (lane == 0 && M > 0) atomicMax(&kp.scores[pd.out_idx], M);
    }
};

// Row bytes of rows [k0, k0+C) for lanes [0, C), issued one chunk ahead and
// converted only when the chunk starts (code_of): converting right after the
// load would make the compiler wait for it (vmcnt(0)) and serialise a memory
// round trip into every chunk.  Out-of-range lanes load from OOR (returns 0).
__device__ __forceinline__ unsigned fetch_raw(const __amdgpu_buffer_rsrc_t row_rsrc, int k0, int lane, int C, int m) {
    const int row = k0 + lane;
    const bool live = lane < C && row >= 0 && row < m;
    return __builtin_amdgcn_raw_buffer_load_b8(row_rsrc, live ? (unsigned)row : OOR, 0, 0);
}

template <bool DNA>
__device__ __forceinline__ int code_of(unsigned raw, int k0, int lane, int C, int m) {
    const int row = k0 + lane;
    const bool live = lane < C && row >= 0 && row < m;
    if constexpr (DNA) return live ? (dna_code(raw) | 0x0C0C0C00) : SENT_DNA;
    else return live ? (int)raw : SENT_BYTE;
}


// Publish the right-edge outflow collected in lanes [64-C, 64) of a chunk that
// started at step k0: rows k0 - (64W-1) .. k0 + C - 1 - (64W-1).
template <int W, int C, int AUX = AUX_SC1>
__device__ __forceinline__ void publish_granules(const Edge& out, int k0, int lane, int m, int IOH, int IOE) {
    const int row_out = k0 + (lane - (64 - C)) - (64 * W - 1);
    const bool st = lane >= 64 - C && row_out >= 0 && row_out < m;
    edge_publish<AUX>(out, row_out, st, IOH, IOE);
}

// One full strip pass with granule inflow (strip > 0) and outflow (strip < strips-1).
template <int W, int C, bool DNA>
__device__ void strip_pass(const KParams& kp, const PairDesc& pd, const int strip, const int lane) {
    constexpr int SW = 64 * W;
    static_assert(C % 4 == 0 && C <= 64 && (C & (C - 1)) == 0, "chunk");
    const int m = pd.m;
    const int go = kp.gap_init, ge = kp.gap_ext, ma = kp.match, mi = kp.mismatch;
    const bool l63 = lane == 63;
    Strip<W, DNA> S;
    S.setup(kp, pd, strip, lane);

    const bool has_in = strip > 0;
    const bool has_out = strip < pd.strips - 1;
    const Edge in_e = strip_edge(kp, pd, strip - 1);
    const Edge out_e = strip_edge(kp, pd, strip);
    const __amdgpu_buffer_rsrc_t row_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + pd.row_off), 0, m, RSRC_FLAGS);

    const int nchunks = (m + SW - 1 + C - 1) / C;
    bool failed = false;
    unsigned raw_nxt = fetch_raw(row_rsrc, 0, lane, C, m);
    u32x4 g_nxt = has_in ? fetch_granules<C>(in_e, 0, lane, m) : u32x4{0u, 0u, 0u, 0u};
    for (int c = 0; c < nchunks; ++c) {
        const int k0 = c * C;
        const unsigned raw = raw_nxt;
        u32x4 g = g_nxt;
        // next chunk's rows in flight while this chunk computes
        raw_nxt = fetch_raw(row_rsrc, k0 + C, lane, C, m);
        if (has_in) await_granules<C>(kp, in_e, g, k0, lane, m, strip, failed);
        if (has_in) g_nxt = fetch_granules<C>(in_e, k0 + C, lane, m);
        const int code = code_of<DNA>(raw, k0, lane, C, m);
        const bool real = has_in && k0 + lane < m;
        S.feed(lane, C, real ? (int)g.y : -go, real ? (int)g.z : -ge, code);
        S.template run<C>(l63, go, ge, ma, mi);
        if (has_out) publish_granules<W, C>(out_e, k0, lane, m, S.IOH, S.IOE);
    }
    S.commit_max(kp, pd, lane);
}

// ---------------------------------------------------------------------------
// Kernel 1: independent waves claim (pair, strip) items strictly in order.
// ---------------------------------------------------------------------------
template <int W, int C, bool DNA>
__global__ void __launch_bounds__(256) sw_strip_kernel(KParams kp) {
    const int lane = threadIdx.x & 63;
    for (;;) {
        unsigned item = 0;
        if (lane == 0) item = atomicAdd(&kp.ctrl->next_item, 1u);
        item = __builtin_amdgcn_readfirstlane(item);
        if ((int)item >= kp.total_items) return;
        const int pi = find_pair(kp, (int)item);
        const PairDesc pd = load_pair(kp, pi);
        const int strip = __builtin_amdgcn_readfirstlane((int)item - kp.item_base[pi]);
        strip_pass<W, C, DNA>(kp, pd, strip, lane);
    }
}

// ---------------------------------------------------------------------------
// Kernel 2 (batches): workgroup b scores pairs b, b+gridDim, ...; its wave w
// runs strips w, w+4, w+8, ... of each pair.  A consumer wave starts its strip
// one strip pass after its previous one, so every hand-off but the first of a
// pair has a full pass of slack.  The four chains of a pair live in one
// workgroup, hence are co-resident: no deadlock for any grid size.
// ---------------------------------------------------------------------------
template <int W, int C, bool DNA>
__global__ void __launch_bounds__(256) sw_pairwg_kernel(KParams kp) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int pi = blockIdx.x; pi < kp.npairs; pi += gridDim.x) {
        const PairDesc pd = load_pair(kp, pi);
        for (int strip = wave; strip < pd.strips; strip += 4) strip_pass<W, C, DNA>(kp, pd, strip, lane);
    }
}

// ---------------------------------------------------------------------------
// Kernel 3 (one long pair): a workgroup claims a group of 4 consecutive
// strips; wave w runs strip 4g+w.  The four waves advance in lock step, one
// barrier per chunk of C rows; wave w+1 runs D = 64W/C + 1 chunks behind wave
// w and takes its inflow from an LDS ring that wave w filled before the
// previous barrier (no memory round trip).  Only the group's first and last
// strips exchange tagged granules with the neighbouring groups.
// ---------------------------------------------------------------------------
template <int W, int C, bool DNA>
__global__ void __launch_bounds__(256) sw_chain_kernel(KParams kp) {
    constexpr int SW = 64 * W;
    constexpr int D = SW / C + 1;          // chunk lag between consecutive waves
    constexpr int R = 4 * C;               // LDS ring rows per link (> 2C+1 live rows)
    __shared__ int2 ring[3][R];
    __shared__ int s_item;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool l63 = lane == 63;
    const int go = kp.gap_init, ge = kp.gap_ext, ma = kp.match, mi = kp.mismatch;
    for (;;) {
        if (threadIdx.x == 0) s_item = (int)atomicAdd(&kp.ctrl->next_item, 1u);
        __syncthreads();
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        __syncthreads();
        if (item >= kp.total_items) return;
        const int pi = find_pair(kp, item);
        const PairDesc pd = load_pair(kp, pi);
        const int m = pd.m;
        const int group = item - kp.item_base[pi];
        const int strip = 4 * group + wave;
        const bool real = strip < pd.strips;
        Strip<W, DNA> S;
        S.setup(kp, pd, strip, lane);   // past-the-end strips are all dead columns
        const int ngroups = (pd.strips + 3) / 4;
        const bool last = strip == pd.strips - 1;
        // the pair's first strip takes a slab inflow, its last strip feeds a slab outflow
        const bool gin = real && wave == 0 && (strip > 0 || kp.slab_in != nullptr);
        const bool gout = real && ((wave == 3 && !last) || (last && kp.slab_out != nullptr));
        const bool lin = real && wave > 0;
        const bool lout = real && wave < 3 && strip + 1 < pd.strips;
        // granule buffers exist only between groups: boundary g joins group g and g+1
        const Edge in_e = group_edge(kp, pd, group - 1, ngroups);
        const Edge out_e = group_edge(kp, pd, group, ngroups);
        const __amdgpu_buffer_rsrc_t row_rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + pd.row_off), 0, m, RSRC_FLAGS);
        const int nloc = (m + SW - 1 + C - 1) / C;
        const int nT = nloc + 3 * D;
        bool failed = false;
        int c = -wave * D;   // this wave's local chunk
        // Row bytes and (wave 0) granules are prefetched TWO chunks ahead into two
        // buffers that the 2x-unrolled loop refills in place (no register
        // rotation, hence no wait at the back-edge).  A one-chunk lead is shorter
        // than the sc1 store->load round trip: a consumer that has caught up
        // would miss and re-poll on every chunk; with two, one initial miss sets
        // a lag after which every prefetch hits.  The loop is instantiated per
        // granule role so that its global loads/stores are unconditional (rows
        // outside the chunk's range are predicated by the OOR offset) and the
        // compiler can count vmcnt exactly instead of draining at every join.
        // gin_c / gout_c: 0 (no granule edge) or the edge's cache policy (AUX_SC1, or
        // AUX_SYS for a slab edge to / from another GPU)
        auto chunk_loop = [&](auto gin_c, auto gout_c) __attribute__((always_inline)) {
            constexpr int GIN_AUX = decltype(gin_c)::value, GOUT_AUX = decltype(gout_c)::value;
            constexpr bool GIN = GIN_AUX != 0, GOUT = GOUT_AUX != 0;
            unsigned r0 = fetch_raw(row_rsrc, c * C, lane, C, m), r1 = fetch_raw(row_rsrc, c * C + C, lane, C, m);
            u32x4 g0 = u32x4{0u, 0u, 0u, 0u}, g1 = g0;
            if constexpr (GIN) {
                g0 = fetch_granules<C, GIN_AUX>(in_e, c * C, lane, m);
                g1 = fetch_granules<C, GIN_AUX>(in_e, c * C + C, lane, m);
            }
            auto chunk = [&](const int cc, u32x4& gbuf, unsigned& rbuf) __attribute__((always_inline)) {
                const int k0 = cc * C;
                const bool active = cc >= 0 && cc < nloc;
                // consume the buffers before refilling them, so each refill can
                // land in the registers the loop carries (no back-edge copies)
                if constexpr (GIN) await_granules<C, GIN_AUX>(kp, in_e, gbuf, k0, lane, m, strip, failed);
                const int code = code_of<DNA>(rbuf, k0, lane, C, m);
                int hg_in = -go, eh_in = -ge;
                const int row = k0 + lane;
                if (active && row >= 0 && row < m && lane < C) {
                    if constexpr (GIN) {
                        hg_in = (int)gbuf.y; eh_in = (int)gbuf.z;
                    } else if (lin) {
                        const int2 v = ring[wave - 1][row & (R - 1)];
                        hg_in = v.x; eh_in = v.y;
                    }
                }
                rbuf = fetch_raw(row_rsrc, k0 + 2 * C, lane, C, m);
                if constexpr (GIN) gbuf = fetch_granules<C, GIN_AUX>(in_e, k0 + 2 * C, lane, m);
                S.feed(lane, C, hg_in, eh_in, code);
                S.template run<C>(l63, go, ge, ma, mi);
                if constexpr (GOUT) {
                    publish_granules<W, C, GOUT_AUX>(out_e, k0, lane, m, S.IOH, S.IOE);
                } else if (active && lout) {
                    const int row_out = k0 + (lane - (64 - C)) - (SW - 1);
                    if (lane >= 64 - C && row_out >= 0 && row_out < m) ring[wave][row_out & (R - 1)] = make_int2(S.IOH, S.IOE);
                }
                __syncthreads();
            };
            int T = 0;
            for (; T + 1 < nT; T += 2, c += 2) {
                chunk(c, g0, r0);
                chunk(c + 1, g1, r1);
            }
            if (T < nT) chunk(c, g0, r0);
        };
        using N_ = std::integral_constant<int, 0>;
        using D_ = std::integral_constant<int, AUX_SC1>;
        using P_ = std::integral_constant<int, AUX_SYS>;
        const bool gin_peer = gin && strip == 0, gout_peer = gout && last && kp.slab_out != nullptr;
        if (gin && gout) {   // a one-strip group between two group or slab edges
            if (gin_peer && gout_peer) chunk_loop(P_{}, P_{});
            else if (gin_peer) chunk_loop(P_{}, D_{});
            else if (gout_peer) chunk_loop(D_{}, P_{});
            else chunk_loop(D_{}, D_{});
        } else if (gin) {
            if (gin_peer) chunk_loop(P_{}, N_{});
            else chunk_loop(D_{}, N_{});
        } else if (gout) {
            if (gout_peer) chunk_loop(N_{}, P_{});
            else chunk_loop(N_{}, D_{});
        } else {
            chunk_loop(N_{}, N_{});
        }
        if (real) S.commit_max(kp, pd, lane);
    }
}

// ---------------------------------------------------------------------------
// Kernel 3b (one long DNA pair, rows staged in LDS, barrier-free): the same
// groups of 4 consecutive strips as sw_chain_kernel, but the waves free-run
// and every hand-off inside the workgroup is a progress word in LDS.
//
//   * the group's row sequence is converted to 2-bit codes (4 = past the end)
//     and staged in LDS once per item, while the group still waits for its
//     left neighbour; no wave touches the row bytes in HBM afterwards;
//   * wave w publishes its right-edge rows into ring w, then advances prod[w]
//     (rows published); wave w+1 reads prod[w] and the chunk's ring rows in
//     one LDS round trip (re-polling both until the word covers the chunk),
//     then advances cons[w+1] (rows consumed): wave w never overwrites a ring
//     slot still unread (back-pressure; R >= 2C, so the two waits cannot
//     deadlock).  DS instructions of one wave execute in issue order, so rows
//     written before the word are visible to a reader that saw the word; a
//     compiler barrier keeps the compiler from reordering them;
//   * the rings start at the border values (H = E = 0), and every slot a
//     consumer may read past the last row holds either that or a real cell of
//     the same column, so no per-row range checks are needed (dead rows only
//     ever see values <= the true maximum);
//   * lanes that have nothing to publish write to per-lane sink slots, so the
//     feed / publish code has no exec-mask branches.
// Lag between strips: 64W + C rows plus one LDS round trip (the lock-step
// chain pays a barrier per chunk and the slowest wave's chunk every chunk).
// ---------------------------------------------------------------------------

#ifndef SW_GPREF
#define SW_GPREF 1           // granule prefetch distance of the flow kernel, in chunks (1 measured best)
#endif


// Phase stamps for tools/trace_flow.py: built with -DSW_PHASE_STAMPS
// (make stamps) to time each chunk's prologue / steps / epilogue in cycles.
#ifdef SW_PHASE_STAMPS
__device__ __forceinline__ unsigned long long sw_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define SW_STAMP() sw_stamp()
#else
#define SW_STAMP() 0ull
#endif


template <int W, int C>
__global__ void __launch_bounds__(256) sw_flow_kernel(KParams kp) {
    constexpr int SW = 64 * W;
    constexpr int R = flow_ring_rows(W, C);
    static_assert(3 * R * 8 + 4 * 64 * 8 + (4 + 4 + 256 + 1) * 4 <= flow_static_lds(W, C), "flow static LDS");
    extern __shared__ unsigned char rc[];        // staged row codes (dynamic LDS)
    __shared__ int2 ring[3][R];
    __shared__ int2 sink2[4][64];
    __shared__ int prod[4], cons[4], sink[4][64];
    __shared__ int s_item;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const bool l63 = lane == 63;
    const bool lo_lane = lane < C;              // lanes fed at a chunk start
    const bool hi_lane = lane >= 64 - C;        // lanes holding a chunk's outflow
    const int go = kp.gap_init, ge = kp.gap_ext, ma = kp.match, mi = kp.mismatch;
    for (;;) {
        if (tid == 0) s_item = (int)atomicAdd(&kp.ctrl->next_item, 1u);
        __syncthreads();   // every wave is done with the previous item
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= kp.total_items) return;
        const int pi = find_pair(kp, item);
        const PairDesc pd = load_pair(kp, pi);
        const int m = pd.m;
        const int group = item - kp.item_base[pi];
        // stage: progress words, border-valued rings, row codes
        if (tid < 4) { prod[tid] = 0; cons[tid] = 0; }
        for (int i = tid; i < 3 * R; i += 256) ring[i / R][i % R] = make_int2(-go, -ge);
        {
            const __amdgpu_buffer_rsrc_t row_rsrc =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + pd.row_off), 0, m, RSRC_FLAGS);
            const int nst = flow_stage_rows(m, W, C);
            for (int i = tid * 4; i < nst; i += 1024) {
                unsigned w = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const unsigned ch = __builtin_amdgcn_raw_buffer_load_b8(row_rsrc, (unsigned)(i + j), 0, 0);
                    w |= (i + j < m ? (unsigned)dna_code(ch) : 4u) << (8 * j);
                }
                *reinterpret_cast<unsigned*>(rc + i) = w;
            }
        }
        __syncthreads();
        const int strip = 4 * group + wave;
        if (strip >= pd.strips) continue;
        Strip<W, true> S;
        S.setup(kp, pd, strip, lane);
        const int ngroups = (pd.strips + 3) / 4;
        const int in_kind = wave > 0 ? FLOW_LDS : strip > 0 ? FLOW_GRANULE : kp.slab_in != nullptr ? FLOW_PEER : FLOW_NONE;
        const int out_kind = strip + 1 >= pd.strips ? (kp.slab_out != nullptr ? FLOW_PEER : FLOW_NONE)
                             : wave < 3           ? FLOW_LDS
                                                  : FLOW_GRANULE;
        const Edge in_e = group_edge(kp, pd, group - 1, ngroups);
        const Edge out_e = group_edge(kp, pd, group, ngroups);
        const int nloc = (m + SW - 1 + C - 1) / C;
        bool failed = false;
        const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
        [[maybe_unused]] int spin_n = 0;   // polls (spin_expired)
        long long t_first = t_start;
        int spins = 0;
        unsigned long long cyc_pro = 0, cyc_run = 0, cyc_epi = 0;
        long long tl[5] = {0, 0, 0, 0, 0};   // SW_TIMELINE: wall clock at chunks 1, 2, 3, 50, 1000
        // per-lane LDS addresses of the progress words (lane 0) or the sinks
        int* const prod_out = lane == 0 ? &prod[wave] : &sink[wave][lane];
        int* const cons_out = lane == 0 ? &cons[wave] : &sink[wave][lane];
        auto flow_loop = [&](auto in_c, auto out_c) __attribute__((always_inline)) {
            constexpr int IN = decltype(in_c)::value, OUT = decltype(out_c)::value;
            constexpr int AIN = flow_aux(IN), AOUT = flow_aux(OUT);
            u32x4 g0 = u32x4{0u, 0u, 0u, 0u}, g1 = g0;
            if constexpr (flow_granule(IN)) {
                g0 = fetch_granules<C, AIN>(in_e, 0, lane, m);
                if constexpr (SW_GPREF == 2) g1 = fetch_granules<C, AIN>(in_e, C, lane, m);
            }
            unsigned code_nxt = rc[lane];
            int cons_seen = 0;   // OUT == FLOW_LDS: last value read of the consumer's word
            auto chunk = [&](const int c, u32x4& gbuf) __attribute__((always_inline)) {
                const int k0 = c * C;
                const int row = k0 + lane;
                const unsigned long long ts0 = SW_STAMP();
#ifdef SW_TIMELINE
                if (c == 1 || c == 2 || c == 3 || c == 50 || c == 1000) {
                    const long long now = (long long)__builtin_amdgcn_s_memrealtime();
                    if (c == 1) tl[0] = now;
                    else if (c == 2) tl[1] = now;
                    else if (c == 3) tl[2] = now;
                    else if (c == 50) tl[3] = now;
                    else tl[4] = now;
                }
#endif
                int hg_in = -go, eh_in = -ge;
                if constexpr (flow_granule(IN)) {
                    await_granules<C, AIN>(kp, in_e, gbuf, k0, lane, m, strip, failed);
                    const bool live = row < m;
                    hg_in = live ? (int)gbuf.y : -go;
                    eh_in = live ? (int)gbuf.z : -ge;
#ifdef SW_TIMELINE
                    if (c == 0) t_first = (long long)__builtin_amdgcn_s_memrealtime();
#endif
                    gbuf = fetch_granules<C, AIN>(in_e, k0 + SW_GPREF * C, lane, m);
                } else if constexpr (IN == FLOW_LDS) {
                    const int need = min(k0 + C, m);
                    // the progress word and the rows behind it in one round trip;
                    // re-read both until the word covers the chunk
                    int avail = lds_load(&prod[wave - 1]);
                    compiler_fence();
                    int2 v = ring[wave - 1][row & (R - 1)];
                    if (__builtin_amdgcn_readfirstlane(avail) < need) {
                        do {
                            __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                            ++spins;
                            avail = lds_load(&prod[wave - 1]);
                            compiler_fence();
                            v = ring[wave - 1][row & (R - 1)];
                            if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                failed = true;   // reported after the strip: no global op in the loop
                                break;
                            }
                        } while (__builtin_amdgcn_readfirstlane(avail) < need);
#ifdef SW_TIMELINE
                        if (c == 0) t_first = (long long)__builtin_amdgcn_s_memrealtime();
#endif
                    }
                    hg_in = v.x;
                    eh_in = v.y;
                    compiler_fence();
                    *cons_out = need;   // executes after the ring read (in-order DS)
                }
                const int code = (int)code_nxt | 0x0C0C0C00;
                if (lo_lane) { S.IOH = hg_in; S.IOE = eh_in; S.IOR = code; }
                compiler_fence();   // keep the next prefetch behind the ring-data wait
                code_nxt = rc[k0 + C + lane];
                const unsigned long long ts1 = SW_STAMP();
                S.template run<C>(l63, go, ge, ma, mi);
                const unsigned long long ts2 = SW_STAMP();
                if constexpr (flow_granule(OUT)) {
                    publish_granules<W, C, AOUT>(out_e, k0, lane, m, S.IOH, S.IOE);
                } else if constexpr (OUT == FLOW_LDS) {
                    const int hi = k0 + C - SW;   // last row this chunk completes
                    if (hi >= 0) {
                        // ring slots of rows <= hi must have been read: rows < hi + 1 - R consumed
                        const int floor_rows = hi + 1 - R;
                        // the consumer's word is re-read only when the cached value no
                        // longer covers the floor (every ~(R - lag) / C chunks)
                        if (cons_seen < floor_rows) {
                            cons_seen = __builtin_amdgcn_readfirstlane(lds_load(&cons[wave + 1]));
                            while (cons_seen < floor_rows) {
                                __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                cons_seen = __builtin_amdgcn_readfirstlane(lds_load(&cons[wave + 1]));
                                if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                    failed = true;
                                    break;
                                }
                            }
                        }
                        // rows below 0 land in slots of rows not yet written, rows past
                        // the end in slots already consumed: no range check needed
                        const int row_out = k0 + (lane - (64 - C)) - (SW - 1);
                        int2* dst = hi_lane ? &ring[wave][row_out & (R - 1)] : &sink2[wave][lane];
                        *dst = make_int2(S.IOH, S.IOE);
                        compiler_fence();
                        *prod_out = min(hi + 1, m);
                    }
                }
                cyc_pro += ts1 - ts0;
                cyc_run += ts2 - ts1;
                cyc_epi += SW_STAMP() - ts2;
            };
            int c = 0;
            for (; c + 1 < nloc; c += 2) {
                chunk(c, g0);
                chunk(c + 1, SW_GPREF == 2 ? g1 : g0);
            }
            if (c < nloc) chunk(c, g0);
        };
        dispatch_kinds<KINDS_PEER>(in_kind, out_kind, flow_loop);
        if (kp.trace != nullptr && lane == 0) {
            unsigned long long* t = kp.trace + 16ull * (unsigned)strip;
            t[0] = (unsigned long long)t_start;
            t[1] = (unsigned long long)t_first;
            t[2] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
            t[3] = (unsigned long long)spins;
            t[4] = cyc_pro;
            t[5] = cyc_run;
            t[6] = cyc_epi;
            t[7] = (unsigned long long)nloc;
            for (int q = 0; q < 5; ++q) t[8 + q] = (unsigned long long)tl[q];
        }
        if (failed && lane == 0) {   // an LDS wait gave up (granule waits report themselves too)
            atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
            atomicMax(&kp.ctrl->err_item, (unsigned)strip);
        }
        S.commit_max(kp, pd, lane);
    }
}

// ---------------------------------------------------------------------------
// Packed-u16 "duo" path (DNA batches whose scores fit 16 bits): every lane
// value holds the same cell of two pairs, pair 0 in the low and pair 1 in the
// high half, so each v_pk_* instruction updates two cells.  Saturating
// (clamped) arithmetic throughout, exact for the same reasons as the int32
// path (Arithmetic), with
//   A  = H + MATCH            exact (the host guarantees MATCH*min(n,m)+MATCH <= 65535)
//   Hg = max(H - G_INIT, 0),  Eh = max(E - G_EXT, 0),  Fh = max(F - G_EXT, 0)
//   t  = max(A_diag - pen, 0) with pen = MATCH - s(q, d) from one v_perm_b32
//        over both pairs' 4-byte column profiles (selector 13 -> 0xFF: dead
//        columns and sentinel rows get penalty 255, which keeps them <= the
//        true maximum without a separate mask).
// ---------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as16(unsigned v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ unsigned as32(u16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ u16x2 vmax2(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 vsubs2(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ u16x2 splat2(int v) { return u16x2{(unsigned short)v, (unsigned short)v}; }
// a + b of both halves as ONE 32-bit add (VOP2 v_add_u32: about half the issue cost of
// v_pk_add_u16 on gfx950, tools/ubench_bank.hip) -- exact when no low-half sum reaches
// 2^16, which duo_fits guarantees for A = H + MATCH <= MATCH*min(n,m) + MATCH <= 65535
__device__ __forceinline__ u16x2 add2(u16x2 a, u16x2 b) { return as16(as32(a) + as32(b)); }

// v_pk_maximum3_f16 as an UNSIGNED 16-bit max3 (gfx950): for halves in [0, 0x7BFF]
// -- sign clear, no Inf/NaN encodings, f16 denormals preserved (the HIP default
// mode) -- the IEEE maximum of the f16 values is the integer maximum of the bit
// patterns (checked exhaustively on the GPU: tools/check_pkmax3.hip).  One VOP3P
// instead of two v_pk_max_u16; the host enables it only when every score, E, F
// and t fits below 0x7C00 (duo_f16_fits).
__device__ __forceinline__ u16x2 vmax3h(u16x2 a, u16x2 b, u16x2 c) {
    unsigned d;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(as32(a)), "v"(as32(b)), "v"(as32(c)));
    return as16(d);
}

constexpr unsigned SENT_DUO = 0x0C0D0C0Du;   // selector 13 in both halves -> penalty 0xFF

// RAW: batches of any byte values (main.cpp:28-33 compares raw bytes; sw_engine.hip duo_fits)
// on the same step, the penalty taken from the bytes instead of a 2-bit code and a profile.
// A row word holds byte << 8 in each half (0x00FF for rows below 0 or past m), a column word
// byte << 8 (0x007F past n), and pen = min(row ^ col, MATCH - MISMATCH) per half (one XOR and
// one v_pk_min_u16 where the DNA step has one v_perm_b32):
//   equal bytes            0
//   different bytes        row ^ col >= 256            -> MATCH - MISMATCH
//   sentinel row, any col  low byte 0xFF ^ (0 or 0x7F)  -> MATCH - MISMATCH
//   live row, dead col     low byte 0x7F = 127          -> MATCH - MISMATCH
// with MATCH - MISMATCH <= 127 (host).  Sentinel and dead cells thus score as mismatches; with
// MISMATCH < 0 (host) each such t = H_diag + MISMATCH < H_diag, and every such H is below the
// cells it derives from, so they stay below the true maximum as the DNA path's penalty 255 keeps
// them (and the rows above row 0 keep H = 0: t = sat(MATCH - pen) = 0).
constexpr unsigned SENT_RAW = 0x00FF00FFu;
__device__ __forceinline__ u16x2 vmin2(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ unsigned col_raw(const unsigned char* c, int col, int n) {
    return col < n ? (unsigned)c[col] << 8 : 0x7Fu;
}

__device__ __forceinline__ DuoDesc load_duo(const KParams& kp, int idx) {
    const DuoDesc raw = kp.duos[idx];
    DuoDesc d;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        d.col_off[h] = uniform64(raw.col_off[h]);
        d.row_off[h] = uniform64(raw.row_off[h]);
        d.n[h] = __builtin_amdgcn_readfirstlane(raw.n[h]);
        d.m[h] = __builtin_amdgcn_readfirstlane(raw.m[h]);
        d.out_idx[h] = __builtin_amdgcn_readfirstlane(raw.out_idx[h]);
    }
    d.bnd_off = uniform64(raw.bnd_off);
    d.n_pad = __builtin_amdgcn_readfirstlane(raw.n_pad);
    d.m_pad = __builtin_amdgcn_readfirstlane(raw.m_pad);
    d.strips = __builtin_amdgcn_readfirstlane(raw.strips);
    return d;
}

// LIN (G_INIT == G_EXT, the reference's defaults): E+ = sat(H_left - G) and
// F+ = sat(H_up - G) exactly (sw_flow2.hip, LIN), so a position keeps A and hg
// only: 5.5 VALU per position and 5 per step instead of 9.5 and 7.
// The chunk's steps unrolled whole by default: the rolled loop's back edge made the
// compiler copy 8 row-code / A registers per iteration and keep the chunk's loop
// overhead (C3, W = 8: 7.26 -> 7.06 ms; W = 4: 8.11 -> 7.74 ms at 8 of 16 iterations,
// profiles/r03_ab/duo_unroll.txt).
#ifndef SW_DUO_UNROLL
#define SW_DUO_UNROLL 64
#endif

// the column words of a duo strip's W positions: DNA penalty profiles (pA: pair 0, pB: pair 1)
// or, RAW, the two pairs' column bytes in one word (pA; pB unused)
template <int W, bool RAW>
__device__ __forceinline__ void duo_columns(const KParams& kp, const DuoDesc& d, int strip, int lane, unsigned (&pA)[W],
                                            unsigned (&pB)[W]) {
    constexpr int SW = 64 * W;
    const unsigned char* c0 = kp.seq + d.col_off[0];
    const unsigned char* c1 = kp.seq + d.col_off[1];
#pragma unroll
    for (int p = 0; p < W; ++p) {
        const int c = strip * SW + lane * W + p;
        if constexpr (RAW) {
            pA[p] = col_raw(c0, c, d.n[0]) | (col_raw(c1, c, d.n[1]) << 16);
            pB[p] = 0u;
        } else {
            unsigned w0 = 0xFFFFFFFFu, w1 = 0xFFFFFFFFu;   // dead column: penalty 255 for every row code
            if (c < d.n[0]) {
                const int q = dna_code(c0[c]);
                w0 = q == 0 ? kp.pen[0] : q == 1 ? kp.pen[1] : q == 2 ? kp.pen[2] : kp.pen[3];
            }
            if (c < d.n[1]) {
                const int q = dna_code(c1[c]);
                w1 = q == 0 ? kp.pen[0] : q == 1 ? kp.pen[1] : q == 2 ? kp.pen[2] : kp.pen[3];
            }
            pA[p] = w0;
            pB[p] = w1;
        }
    }
}

// the penalty MATCH - s of one position for both pairs (RAW: see SENT_RAW)
template <bool RAW>
__device__ __forceinline__ u16x2 duo_pen(unsigned pA, unsigned pB, unsigned rL, u16x2 P2) {
    if constexpr (RAW) return vmin2(as16(rL ^ pA), P2);
    else return as16(__builtin_amdgcn_perm(pB, pA, rL));
}

template <int W, bool M3, bool LIN = false, bool RAW = false>
struct StripDuo {
    static constexpr unsigned SENT = RAW ? SENT_RAW : SENT_DUO;
    unsigned pA[W], pB[W];                   // column penalty words: pair 0 (perm src1), pair 1 (perm src0)
    u16x2 aA[W], aB[W];                      // A = H + MATCH, ping-pong (diagonal source)
    u16x2 hg[W], eh[W], fh[W];               // saturated H-G_INIT, E-G_EXT, F-G_EXT
    unsigned r[W];                           // row-code perm selectors (RAW: row bytes)
    u16x2 L0, M, P2;                         // P2: MATCH - MISMATCH in both halves (RAW)
    unsigned IOA, IOE, IOR;

    __device__ __forceinline__ void setup(const KParams& kp, const DuoDesc& d, int strip, int lane) {
        duo_columns<W, RAW>(kp, d, strip, lane, pA, pB);
        const u16x2 ma2 = splat2(kp.match);
        P2 = splat2(kp.match - kp.mismatch);
#pragma unroll
        for (int p = 0; p < W; ++p) {   // border: H = E = F = 0
            aA[p] = ma2; aB[p] = ma2; hg[p] = splat2(0); eh[p] = splat2(0); fh[p] = splat2(0); r[p] = SENT;
        }
        L0 = ma2; M = splat2(0); IOA = as32(ma2); IOE = 0u; IOR = SENT;
    }

    // One anti-diagonal step; S = the step's index mod W.  Position p's row code lives
    // in r[(p - S) mod W]: the slot of position p at step S is the slot of position
    // p-1 at step S-1, so the codes advance one position per step with no register
    // move, and the code entering position 0 (lane l-1's position W-1, or the inflow
    // at lane 0) is written in place by the DPP that fetches it.
    template <int S>
    __device__ __forceinline__ void step_lin(u16x2 (&aCur)[W], const u16x2 (&aPrev)[W], const u16x2 go2,
                                             const u16x2 ma2, const u16x2 gom2) {
        const u16x2 aL0 = as16((unsigned)dpp_shr1((int)IOA, (int)as32(aPrev[W - 1])));
        constexpr int s0 = (W - S % W) % W;
        const unsigned ior = IOR;
        IOR = (unsigned)__builtin_amdgcn_mov_dpp((int)ior, DPP_WAVE_SHL1, 0xF, 0xF, true);
        r[s0] = (unsigned)dpp_shr1((int)ior, (int)r[s0]);
        const u16x2 hgL0 = vsubs2(aL0, gom2);
        u16x2 tOdd = splat2(0);
#pragma unroll
        for (int p = W - 1; p >= 0; --p) {
            const int q = p > 0 ? p - 1 : 0;
            const u16x2 hgL = p > 0 ? hg[q] : hgL0;   // E+ = sat(H_left - G)
            const unsigned rL = r[(p + W - S % W) % W];
            const u16x2 aD = p > 0 ? aCur[q] : L0;
            const u16x2 pen = duo_pen<RAW>(pA[p], pB[p], rL, P2);
            const u16x2 t = vsubs2(aD, pen);
            u16x2 H;
            if constexpr (M3) {
                H = vmax3h(t, hgL, hg[p]);             // hg[p] (last step) = F+ = sat(H_up - G)
                if constexpr (W == 1) M = vmax2(M, t);
                else if (p & 1) tOdd = t;
                else M = vmax3h(M, tOdd, t);
            } else {
                H = vmax2(vmax2(t, hgL), hg[p]);
                M = vmax2(M, t);
            }
            aCur[p] = add2(H, ma2);
            hg[p] = vsubs2(H, go2);
        }
        L0 = aL0;
        IOA = (unsigned)__builtin_amdgcn_update_dpp((int)as32(aCur[W - 1]), (int)IOA, DPP_WAVE_SHL1, 0xF, 0xF, false);
    }

    template <int S>
    __device__ __forceinline__ void step(u16x2 (&aCur)[W], const u16x2 (&aPrev)[W], const u16x2 go2,
                                         const u16x2 ge2, const u16x2 ma2, const u16x2 gom2) {
        if constexpr (LIN) {
            step_lin<S>(aCur, aPrev, go2, ma2, gom2);
            return;
        }
        const u16x2 aL0 = as16((unsigned)dpp_shr1((int)IOA, (int)as32(aPrev[W - 1])));
        const u16x2 ehL0 = as16((unsigned)dpp_shr1((int)IOE, (int)as32(eh[W - 1])));
        constexpr int s0 = (W - S % W) % W;     // slot of position 0 (= last step's position W-1)
        const unsigned ior = IOR;   // rotated first: the slot DPP then takes the old IOR (no copy)
        IOR = (unsigned)__builtin_amdgcn_mov_dpp((int)ior, DPP_WAVE_SHL1, 0xF, 0xF, true);
        r[s0] = (unsigned)dpp_shr1((int)ior, (int)r[s0]);
        const u16x2 hgL0 = vsubs2(aL0, gom2);   // H - G_INIT of the left neighbour, from its A
        u16x2 tOdd = splat2(0);                 // M3: t of position p+1, folded with p's into M
#pragma unroll
        for (int p = W - 1; p >= 0; --p) {
            const int q = p > 0 ? p - 1 : 0;
            const u16x2 hgL = p > 0 ? hg[q] : hgL0;
            const u16x2 ehL = p > 0 ? eh[q] : ehL0;
            const unsigned rL = r[(p + W - S % W) % W];
            const u16x2 aD = p > 0 ? aCur[q] : L0;
            const u16x2 pen = duo_pen<RAW>(pA[p], pB[p], rL, P2);
            const u16x2 t = vsubs2(aD, pen);                 // max(H_diag + s, 0)
            const u16x2 E = vmax2(ehL, hgL);
            const u16x2 F = vmax2(fh[p], hg[p]);
            u16x2 H;
            if constexpr (M3) {
                H = vmax3h(t, E, F);
                if constexpr (W == 1) M = vmax2(M, t);
                else if (p & 1) tOdd = t;                    // positions (2k+1, 2k): one max3 into M
                else M = vmax3h(M, tOdd, t);
            } else {
                H = vmax2(vmax2(t, E), F);
                M = vmax2(M, t);
            }
            aCur[p] = add2(H, ma2);
            hg[p] = vsubs2(H, go2);
            eh[p] = vsubs2(E, ge2);
            fh[p] = vsubs2(F, ge2);
        }
        L0 = aL0;
        // the I/O registers move down one lane (wave_shl:1); lane 63, which has no
        // source, keeps the 'old' operand: this step's right-edge outflow (no select)
        IOA = (unsigned)__builtin_amdgcn_update_dpp((int)as32(aCur[W - 1]), (int)IOA, DPP_WAVE_SHL1, 0xF, 0xF, false);
        IOE = (unsigned)__builtin_amdgcn_update_dpp((int)as32(eh[W - 1]), (int)IOE, DPP_WAVE_SHL1, 0xF, 0xF, false);
    }

    // steps K, K+1, ... of an unrolled group of U = max(W, 2): slot rotation by S = K mod W,
    // A ping-pong by K mod 2
    template <int K, int U>
    __device__ __forceinline__ void steps(const u16x2 go2, const u16x2 ge2, const u16x2 ma2, const u16x2 gom2) {
        if constexpr (K < U) {
            if constexpr (K % 2 == 0) step<K % W>(aA, aB, go2, ge2, ma2, gom2);
            else step<K % W>(aB, aA, go2, ge2, ma2, gom2);
            steps<K + 1, U>(go2, ge2, ma2, gom2);
        }
    }

    template <int C>
    __device__ __forceinline__ void run(const u16x2 go2, const u16x2 ge2, const u16x2 ma2, const u16x2 gom2) {
        constexpr int U = W < 2 ? 2 : W;
        static_assert(C % U == 0, "a chunk is a whole number of slot rotations");
        SW_PRAGMA(unroll SW_DUO_UNROLL)
        for (int s = 0; s < C; s += U) steps<0, U>(go2, ge2, ma2, gom2);
    }

    __device__ __forceinline__ void commit_max(const KParams& kp, const DuoDesc& d, int lane) {
        int m0 = M.x, m1 = M.y;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            m0 = max(m0, __shfl_xor(m0, off));
            m1 = max(m1, __shfl_xor(m1, off));
        }
        if (lane == 0) {
            if (m0 > 0) atomicMax(&kp.scores[d.out_idx[0]], m0);
            if (m1 > 0 && d.out_idx[1] >= 0) atomicMax(&kp.scores[d.out_idx[1]], m1);
        }
    }
};

// StripDuo with its row codes read from an LDS table (sw_duo_lds_kernel with TAB): the
// code selector of row r sits at tab[r + DUO_TAB_OFF], so position 0 of lane l takes the
// code of its row k - W*l at step k from tl[k] (tl = tab + DUO_TAB_OFF - W*l), 4 steps per
// 16-B read, instead of two DPP moves a step carrying the codes lane to lane.  The code of
// position p at chunk step K lives in R[(K - p) & 15]: a code enters at position 0 and
// stays in its register for the W steps it takes to cross the lane; the read for steps
// K+5..K+8 is issued at step K, into registers whose codes left the lane by step K-1.
template <int W, bool M3, bool LIN, bool RAW = false>
struct StripDuoT {
    static_assert(W % 4 == 0 && W <= 8, "16-B table reads per 4 steps; a code lives W steps in 16 registers");
    unsigned pA[W], pB[W];
    u16x2 aA[W], aB[W];
    u16x2 hg[W], eh[W], fh[W];
    unsigned R[16];
    u16x2 L0, M, P2;
    unsigned IOA, IOE;
    const unsigned* tl;

    __device__ __forceinline__ void setup(const KParams& kp, const DuoDesc& d, int strip, int lane, const unsigned* tab) {
        duo_columns<W, RAW>(kp, d, strip, lane, pA, pB);
        P2 = splat2(kp.match - kp.mismatch);
        const u16x2 ma2 = splat2(kp.match);
#pragma unroll
        for (int p = 0; p < W; ++p) {
            aA[p] = ma2; aB[p] = ma2; hg[p] = splat2(0); eh[p] = splat2(0); fh[p] = splat2(0);
        }
        L0 = ma2; M = splat2(0); IOA = as32(ma2); IOE = 0u;
        tl = tab + DUO_TAB_OFF - W * lane;
        // codes of steps -8..7 (rows below 0: the table's sentinels)
#pragma unroll
        for (int g = -2; g < 2; ++g) load_group(4 * g);
    }

    __device__ __forceinline__ void load_group(const int k) {   // k: a multiple of 4
        const u32x4 v = *reinterpret_cast<const u32x4*>(tl + k);
        const int j = k & 15;
        R[j] = v.x; R[(j + 1) & 15] = v.y; R[(j + 2) & 15] = v.z; R[(j + 3) & 15] = v.w;
    }

    // step K (0..15) of a 16-step group starting at strip step kb
    template <int K>
    __device__ __forceinline__ void step(u16x2 (&aCur)[W], const u16x2 (&aPrev)[W], const int kb, const u16x2 go2,
                                         const u16x2 ge2, const u16x2 ma2, const u16x2 gom2) {
        if constexpr ((K + 5) % 4 == 0) load_group(kb + K + 5);
        const u16x2 aL0 = as16((unsigned)dpp_shr1((int)IOA, (int)as32(aPrev[W - 1])));
        u16x2 ehL0 = splat2(0);
        if constexpr (!LIN) ehL0 = as16((unsigned)dpp_shr1((int)IOE, (int)as32(eh[W - 1])));
        const u16x2 hgL0 = vsubs2(aL0, gom2);
        u16x2 tOdd = splat2(0);
#pragma unroll
        for (int p = W - 1; p >= 0; --p) {
            const int q = p > 0 ? p - 1 : 0;
            const u16x2 hgL = p > 0 ? hg[q] : hgL0;
            const unsigned rL = R[(K - p + 16) & 15];
            const u16x2 aD = p > 0 ? aCur[q] : L0;
            const u16x2 pen = duo_pen<RAW>(pA[p], pB[p], rL, P2);
            const u16x2 t = vsubs2(aD, pen);
            u16x2 H;
            if constexpr (LIN) {
                H = vmax3h(t, hgL, hg[p]);
                if (p & 1) tOdd = t;
                else M = vmax3h(M, tOdd, t);
            } else {
                const u16x2 ehL = p > 0 ? eh[q] : ehL0;
                const u16x2 E = vmax2(ehL, hgL);
                const u16x2 F = vmax2(fh[p], hg[p]);
                if constexpr (M3) {
                    H = vmax3h(t, E, F);
                    if (p & 1) tOdd = t;
                    else M = vmax3h(M, tOdd, t);
                } else {
                    H = vmax2(vmax2(t, E), F);
                    M = vmax2(M, t);
                }
                eh[p] = vsubs2(E, ge2);
                fh[p] = vsubs2(F, ge2);
            }
            aCur[p] = add2(H, ma2);
            hg[p] = vsubs2(H, go2);
        }
        L0 = aL0;
        IOA = (unsigned)__builtin_amdgcn_update_dpp((int)as32(aCur[W - 1]), (int)IOA, DPP_WAVE_SHL1, 0xF, 0xF, false);
        if constexpr (!LIN)
            IOE = (unsigned)__builtin_amdgcn_update_dpp((int)as32(eh[W - 1]), (int)IOE, DPP_WAVE_SHL1, 0xF, 0xF, false);
    }

    template <int K>
    __device__ __forceinline__ void steps(const int kb, const u16x2 go2, const u16x2 ge2, const u16x2 ma2,
                                          const u16x2 gom2) {
        if constexpr (K < 16) {
            if constexpr (K % 2 == 0) step<K>(aA, aB, kb, go2, ge2, ma2, gom2);
            else step<K>(aB, aA, kb, go2, ge2, ma2, gom2);
            steps<K + 1>(kb, go2, ge2, ma2, gom2);
        }
    }

    // C steps from strip step k0 (a multiple of 16)
    template <int C>
    __device__ __forceinline__ void run(const int k0, const u16x2 go2, const u16x2 ge2, const u16x2 ma2,
                                        const u16x2 gom2) {
        static_assert(C % 16 == 0, "chunks of whole 16-step groups");
#pragma unroll
        for (int s = 0; s < C; s += 16) steps<0>(k0 + s, go2, ge2, ma2, gom2);
    }

    __device__ __forceinline__ void commit_max(const KParams& kp, const DuoDesc& d, int lane) {
        int m0 = M.x, m1 = M.y;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            m0 = max(m0, __shfl_xor(m0, off));
            m1 = max(m1, __shfl_xor(m1, off));
        }
        if (lane == 0) {
            if (m0 > 0) atomicMax(&kp.scores[d.out_idx[0]], m0);
            if (m1 > 0 && d.out_idx[1] >= 0) atomicMax(&kp.scores[d.out_idx[1]], m1);
        }
    }
};

__device__ __forceinline__ unsigned codes_duo(unsigned raw0, unsigned raw1, int k0, int lane, int C, const DuoDesc& d) {
    const int row = k0 + lane;
    const bool l0 = lane < C && row >= 0 && row < d.m[0];
    const bool l1 = lane < C && row >= 0 && row < d.m[1];
    const unsigned s0 = l0 ? (unsigned)dna_code(raw0) : 13u;
    const unsigned s1 = l1 ? (unsigned)dna_code(raw1) + 4u : 13u;
    return 0x0C000C00u | (s1 << 16) | s0;
}

// the row word of row k0 + lane for both pairs: DNA perm selectors, or RAW bytes (SENT_RAW)
template <bool RAW>
__device__ __forceinline__ unsigned codes_duo_t(unsigned raw0, unsigned raw1, int k0, int lane, int C, const DuoDesc& d) {
    if constexpr (RAW) {
        const int row = k0 + lane;
        const bool l0 = lane < C && row >= 0 && row < d.m[0];
        const bool l1 = lane < C && row >= 0 && row < d.m[1];
        return (l0 ? (raw0 & 0xFFu) << 8 : 0xFFu) | ((l1 ? (raw1 & 0xFFu) << 8 : 0xFFu) << 16);
    } else {
        return codes_duo(raw0, raw1, k0, lane, C, d);
    }
}

#ifndef SW_DUO_SLACK
#define SW_DUO_SLACK 0   // chunks a duo strip lets its producer lead by before it starts
#endif
template <int W, int C, bool M3, bool LIN, bool RAW = false>
__device__ void strip_pass_duo(const KParams& kp, const DuoDesc& d, const int strip, const int lane) {
    constexpr int SW = 64 * W;
    const int m = d.m_pad;
    const u16x2 go2 = splat2(kp.gap_init), ge2 = splat2(kp.gap_ext), ma2 = splat2(kp.match),
                gom2 = splat2(kp.gap_init + kp.match);
    StripDuo<W, M3, LIN, RAW> S;
    S.setup(kp, d, strip, lane);
    const bool has_in = strip > 0;
    const bool has_out = strip < d.strips - 1;
    Granule* in_base = kp.bnd + d.bnd_off + (uint64_t)(has_in ? strip - 1 : 0) * (uint64_t)m;
    Granule* out_base = kp.bnd + d.bnd_off + (uint64_t)strip * (uint64_t)m;
    const Edge in_e = linear_edge(in_base, m, kp.epoch);
    const Edge out_e = linear_edge(out_base, m, kp.epoch);
    const __amdgpu_buffer_rsrc_t r0 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + d.row_off[0]), 0, d.m[0], RSRC_FLAGS);
    const __amdgpu_buffer_rsrc_t r1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + d.row_off[1]), 0, d.m[1], RSRC_FLAGS);
    const int nchunks = (m + SW - 1 + C - 1) / C;
    bool failed = false;
    if constexpr (SW_DUO_SLACK > 0) {
        // start only once the producer strip has published chunk SW_DUO_SLACK: the lead keeps
        // every later chunk's granules (loaded one chunk ahead) published before they are read
        if (has_in && SW_DUO_SLACK * C < m) {
            u32x4 g0 = fetch_granules<C>(in_e, SW_DUO_SLACK * C, lane, m);
            await_granules<C>(kp, in_e, g0, SW_DUO_SLACK * C, lane, m, strip, failed);
        }
    }
    unsigned raw0_nxt = fetch_raw(r0, 0, lane, C, d.m[0]), raw1_nxt = fetch_raw(r1, 0, lane, C, d.m[1]);
    u32x4 g_nxt = has_in ? fetch_granules<C>(in_e, 0, lane, m) : u32x4{0u, 0u, 0u, 0u};
    for (int c = 0; c < nchunks; ++c) {
        const int k0 = c * C;
        const unsigned raw0 = raw0_nxt, raw1 = raw1_nxt;
        u32x4 g = g_nxt;
        raw0_nxt = fetch_raw(r0, k0 + C, lane, C, d.m[0]);
        raw1_nxt = fetch_raw(r1, k0 + C, lane, C, d.m[1]);
        if (has_in) await_granules<C>(kp, in_e, g, k0, lane, m, strip, failed);
        if (has_in) g_nxt = fetch_granules<C>(in_e, k0 + C, lane, m);
        const unsigned code = codes_duo_t<RAW>(raw0, raw1, k0, lane, C, d);
        if (lane < C) {
            const bool real = has_in && k0 + lane < m;
            S.IOA = real ? g.y : as32(ma2);
            S.IOE = real ? g.z : 0u;
            S.IOR = code;
        }
        S.template run<C>(go2, ge2, ma2, gom2);
        if (has_out) publish_granules<W, C>(out_e, k0, lane, m, (int)S.IOA, (int)S.IOE);
    }
    S.commit_max(kp, d, lane);
}

// Kernel 4 (DNA batches, 16-bit scores): workgroup b scores duos b, b+gridDim,
// ...; its DUO_WAVES waves run strips w, w+DUO_WAVES, ... of each duo (as
// sw_pairwg_kernel).  Four waves: eight (four per SIMD at C3) measured slower
// (r01 12.43 vs 12.06 ms; r03 7.57 vs 7.44 ms): the step is issue-bound, and its
// slow-class instructions (v_pk_*, v_perm, DPP) cost the SIMD ~1.8 ns at 2 waves
// and at 4 alike (tools/ubench_bank.hip).
// M3: H = max3 and the running max fold two positions per v_pk_maximum3_f16
// (scores below 0x7C00 only, LaunchCfg::duo_f16).
template <int W, int C, bool M3, bool LIN, bool RAW = false>
__global__ void __launch_bounds__(64 * DUO_WAVES) sw_duo_kernel(KParams kp) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int di = blockIdx.x; di < kp.npairs; di += gridDim.x) {
        const DuoDesc d = load_duo(kp, di);
        for (int strip = wave; strip < d.strips; strip += DUO_WAVES) strip_pass_duo<W, C, M3, LIN, RAW>(kp, d, strip, lane);
    }
}

// ---------------------------------------------------------------------------
// The duo kernel with every strip hand-off in LDS (LaunchCfg::duo_wrap > 0, C = 64):
// as sw_duo_kernel, wave w runs strips w, w + 4, ... of each duo, one per round, but
// strip s hands its right edge to strip s + 1 through the workgroup's LDS instead of
// HBM granules:
//   * wave w -> w + 1 (same round): a DUO_R-row ring, row r at slot (pos0 + r) mod R,
//     with back-pressure on the consumer's progress word;
//   * wave 3 -> wave 0 (next round): the wrap buffer, kp.wrap_rows >= m slots (dynamic
//     LDS), without back-pressure: wave 3 writes row r of round k + 1 only after waves
//     2, 1, 0 of round k + 1 have computed row r, so wave 0 has read row r of round k
//     by then (a back-pressure wait there would close the cycle 0 -> 1 -> 2 -> 3 -> 0).
// Positions: round k of the workgroup's duo sequence starts at the sum of the spans of
// the rounds before it (every wave walks the same rounds), so progress words grow
// monotonically across rounds and duos and the waves need no barrier between duos.
// A slot holds the edge's A (= H + MATCH) of both pairs, and with the affine step E too.
// ---------------------------------------------------------------------------
constexpr int DUO_R = 256;   // rows per in-round ring (a link's lag is ~C rows)
template <bool LIN> struct DuoSlotT { using T = uint2; };
template <> struct DuoSlotT<true> { using T = unsigned; };
template <bool LIN> using DuoSlot = typename DuoSlotT<LIN>::T;

template <bool LIN>
struct DuoLink {
    DuoSlot<LIN>* buf;   // ring or wrap buffer
    unsigned mask;       // row r at slot (off + r) & mask
    int off;
    int pb;              // position of row 0 in the progress words
    const int* prod;     // inflow: the producer's word (rows < *prod - pb are written)
    const int* cons;     // outflow ring: the consumer's word (positions < *cons are read); null: none
};

// TAB: the row codes come from the workgroup's LDS table (StripDuoT); `build` (the duo's
// strip 0, wave 0) writes the table as it goes, two chunks ahead of its own reads and so of
// every later strip's, after its first 128 rows (and the sentinels below row 0), then sets
// *ready_out (the other waves wait for it before their first read of this duo's table).
template <int W, int C, bool M3, bool LIN, bool TAB, bool RAW = false>
__device__ void strip_pass_duo_lds(const KParams& kp, const DuoDesc& d, const int strip, const int lane,
                                   const bool has_in, const DuoLink<LIN> in, const bool has_out,
                                   const DuoLink<LIN> out, int* const prod_out, int* const cons_out,
                                   DuoSlot<LIN>* const sink, unsigned* const tab, const bool build,
                                   int* const ready_out, const int ready_val, const int prio_par,
                                   const long long prio_t0) {
    constexpr int SW = 64 * W;
    static_assert(C == 64, "the LDS links move one row per lane and chunk");
    const int m = d.m_pad;
    const u16x2 go2 = splat2(kp.gap_init), ge2 = splat2(kp.gap_ext), ma2 = splat2(kp.match),
                gom2 = splat2(kp.gap_init + kp.match);
    const __amdgpu_buffer_rsrc_t r0 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + d.row_off[0]), 0, d.m[0], RSRC_FLAGS);
    const __amdgpu_buffer_rsrc_t r1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + d.row_off[1]), 0, d.m[1], RSRC_FLAGS);
    const int nchunks = (m + SW - 1 + C - 1) / C;
    unsigned raw0_nxt = 0u, raw1_nxt = 0u;
    if constexpr (TAB) {
        if (build) {
            // rows -DUO_TAB_OFF .. 127 now (sentinels below row 0), then 64 rows a chunk
            for (int i = lane; i < DUO_TAB_OFF + 128; i += 64) {
                const int row = i - DUO_TAB_OFF;
                const unsigned q0 = fetch_raw(r0, row, 0, 1, d.m[0]), q1 = fetch_raw(r1, row, 0, 1, d.m[1]);
                tab[i] = codes_duo_t<RAW>(q0, q1, row, 0, 1, d);
            }
            raw0_nxt = fetch_raw(r0, 128, lane, C, d.m[0]);
            raw1_nxt = fetch_raw(r1, 128, lane, C, d.m[1]);
            compiler_fence();
            *ready_out = ready_val;   // after the table writes (DS ops execute in order)
        }
    } else {
        raw0_nxt = fetch_raw(r0, 0, lane, C, d.m[0]);
        raw1_nxt = fetch_raw(r1, 0, lane, C, d.m[1]);
    }
    std::conditional_t<TAB, StripDuoT<W, M3, LIN, RAW>, StripDuo<W, M3, LIN, RAW>> S;
    if constexpr (TAB) S.setup(kp, d, strip, lane, tab);
    else S.setup(kp, d, strip, lane);
    const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
    [[maybe_unused]] int spin_n = 0;   // polls (spin_expired)
    bool failed = false;
    int cons_seen = 0;
    long long prio_t = t_start;   // the clock read one chunk ago (kp.duo_prio)
    for (int c = 0; c < nchunks; ++c) {
        const int k0 = c * C;
        const unsigned raw0 = raw0_nxt, raw1 = raw1_nxt;
        // kp.duo_prio = k: the CU's two workgroups (prio_par 0 / 1) take turns at issue priority in
        // slices of 2^k ticks of the 100 MHz clock from their start (the second-placed one first), so
        // neither runs alone on its SIMDs at the end: old-wave-first arbitration otherwise lets the
        // first one finish at ~3.4 ms and the second at ~6.4 on C3; at k = 17 both end at ~6.0-6.3
        // (profiles/r05_duo_prio.md). Slices under ~0.3 ms do not balance them.
        if (prio_par >= 0) {
            if ((((unsigned long long)(prio_t - prio_t0) >> kp.duo_prio) ^ (unsigned)prio_par) & 1u) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
            prio_t = (long long)__builtin_amdgcn_s_memrealtime();
        }
        if constexpr (TAB) {
            if (build) {   // table rows k0 + 128 .. k0 + 191 (bytes loaded a chunk ago), bytes of the next 64
                tab[DUO_TAB_OFF + k0 + 128 + lane] = codes_duo_t<RAW>(raw0, raw1, k0 + 128, lane, C, d);
                raw0_nxt = fetch_raw(r0, k0 + 192, lane, C, d.m[0]);
                raw1_nxt = fetch_raw(r1, k0 + 192, lane, C, d.m[1]);
            }
        } else {
            raw0_nxt = fetch_raw(r0, k0 + C, lane, C, d.m[0]);
            raw1_nxt = fetch_raw(r1, k0 + C, lane, C, d.m[1]);
        }
        unsigned va = as32(ma2), ve = 0u;   // no inflow / rows >= m: the border (H = E = 0)
        if (has_in) {
            // the progress word and the chunk's rows in one LDS round trip (a wave's DS ops
            // execute in order: rows read after a word that covers them are complete)
            const int need = in.pb + min(k0 + C, m);
            DuoSlot<LIN>* const src = &in.buf[(unsigned)(in.off + k0 + lane) & in.mask];
            int avail = lds_load(in.prod);
            compiler_fence();
            DuoSlot<LIN> v = *src;
            if (__builtin_amdgcn_readfirstlane(avail) < need && !failed) {
                do {
                    __builtin_amdgcn_s_sleep(1);
                    avail = lds_load(in.prod);
                    compiler_fence();
                    v = *src;
                    if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                        failed = true;
                        break;
                    }
                } while (__builtin_amdgcn_readfirstlane(avail) < need);
            }
            const bool real = k0 + lane < m;
            if constexpr (LIN) {
                va = real ? v : va;
            } else {
                va = real ? v.x : va;
                ve = real ? v.y : 0u;
            }
            compiler_fence();
            *cons_out = in.pb + k0 + C;   // after the ring read (DS ops execute in order)
        }
        S.IOA = va;
        S.IOE = ve;
        if constexpr (TAB) {
            S.template run<C>(k0, go2, ge2, ma2, gom2);
        } else {
            S.IOR = codes_duo_t<RAW>(raw0, raw1, k0, lane, C, d);
            S.template run<C>(go2, ge2, ma2, gom2);
        }
        if (has_out) {
            // lane L holds the outflow of step k0 + L: row k0 + L - (SW - 1)
            const int row_out = k0 + lane - (SW - 1);
            if (out.cons != nullptr) {
                // this chunk's last position reuses the slot of position last - R: read by now?
                const int floor_pos = out.pb + k0 + C - SW + 1 - DUO_R;
                if (cons_seen < floor_pos && !failed) {
                    cons_seen = __builtin_amdgcn_readfirstlane(lds_load(out.cons));
                    while (cons_seen < floor_pos) {
                        __builtin_amdgcn_s_sleep(1);
                        cons_seen = __builtin_amdgcn_readfirstlane(lds_load(out.cons));
                        if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                            failed = true;
                            break;
                        }
                    }
                }
            }
            const bool st = row_out >= 0 && row_out < m;
            DuoSlot<LIN>* const dst = st ? &out.buf[(unsigned)(out.off + row_out) & out.mask] : &sink[lane];
            if constexpr (LIN) *dst = S.IOA;
            else *dst = make_uint2(S.IOA, S.IOE);
            compiler_fence();
            *prod_out = out.pb + min(max(0, k0 + C - SW + 1), m);   // after the slot writes
        }
    }
    if (failed && lane == 0) {
        atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
        atomicMax(&kp.ctrl->err_item, (unsigned)strip);
    }
    S.commit_max(kp, d, lane);
}

// kp.wrap_rows: slots of the wrap buffer (a power of two >= every duo's m_pad); kp.ring_cons: per-CU
// words for the strip-role assignment (below), or null (roles by wave index); TAB: the row-code
// table follows it in the dynamic LDS (DUO_TAB_OFF + m_pad + DUO_TAB_TAIL words, host-sized).
// With TAB, one table serves the workgroup's current duo: wave 0 rewrites it for duo i only
// after every wave has reported done with duo i - 1 (done[]), and the other waves read it
// only after wave 0 has written its first rows (tabready).  Neither wait closes a cycle:
// the waves finishing duo i - 1 need nothing from wave 0's duo i.
template <int W, int C, bool M3, bool LIN, bool TAB, bool RAW = false>
__global__ void __launch_bounds__(64 * DUO_WAVES) sw_duo_lds_kernel(KParams kp) {
    static_assert(DUO_WAVES == 4, "the LDS links pair waves w -> w + 1 and 3 -> 0");
    using Slot = DuoSlot<LIN>;
    extern __shared__ __attribute__((aligned(16))) unsigned char duo_dyn[];
    Slot* const wrap = reinterpret_cast<Slot*>(duo_dyn);
    unsigned* const tab = reinterpret_cast<unsigned*>(duo_dyn + (size_t)kp.wrap_rows * sizeof(Slot));
    __shared__ Slot ring[3][DUO_R];
    __shared__ Slot sink[4][64];
    __shared__ int prod[4], cons[4], psink[4][64];
    __shared__ int done[4], tabready;
    __shared__ int s_simd[4], s_roles;
    const int lane = threadIdx.x & 63;
    const int hw = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const unsigned hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID: SIMD 5:4, CU 11:8, SH 12, SE 15:13
    const int my_simd = __builtin_amdgcn_readfirstlane((int)((hwid >> 4) & 3));
    if (threadIdx.x < 4) {
        prod[threadIdx.x] = 0;
        cons[threadIdx.x] = 0;
        done[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) tabready = 0;
    if (lane == 0) s_simd[hw] = my_simd;
    __syncthreads();
    // Strip roles (kp.ring_cons: one zeroed word per CU).  Two duo workgroups share a CU and its
    // 4 SIMDs; the older one gets most issue slots, and a role-r wave idles (r x 576 steps) until
    // the pipeline reaches it.  The second workgroup on a CU takes, on each SIMD, the role 3 - r
    // of the first one's wave there, so one wave of each SIMD starts early and one late.  Roles
    // follow the SIMDs only when this workgroup's 4 waves sit on 4 distinct SIMDs, so they are a
    // permutation of the waves whatever the placement (placement affects speed, never results).
    int wave = hw;
    if (kp.ring_cons != nullptr) {
        if (threadIdx.x == 0) {
            const int s0 = s_simd[0];
            int roles = -1;
            if (((1 << s0) | (1 << s_simd[1]) | (1 << s_simd[2]) | (1 << s_simd[3])) == 15) {
                const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;   // HW_REG_XCC_ID
                const unsigned key = (xcc << 8) | (((hwid >> 13) & 7u) << 5) | (((hwid >> 12) & 1u) << 4) | ((hwid >> 8) & 15u);
                const unsigned old = atomicCAS(kp.ring_cons + key, 0u, (1u << 16) | (unsigned)s0);
                if (old == 0u) roles = 0;                                   // first on this CU: its own order
                else if ((old >> 16) == 1u) {                               // second: mirror the first
                    atomicAdd(kp.ring_cons + key, 1u << 16);
                    roles = 16 | (int)(old & 3u);
                }
            }
            s_roles = roles;
        }
        __syncthreads();
        const int roles = s_roles;
        if (roles == 0) wave = (my_simd - s_simd[0]) & 3;
        else if (roles > 0) wave = 3 - ((my_simd - (roles & 3)) & 3);
    }
    wave = __builtin_amdgcn_readfirstlane(wave);
    // turn-taking parity (kp.duo_prio): the first workgroup on a CU 0, the second 1, else off
    int prio_par = -1;
    if (kp.ring_cons != nullptr && kp.duo_prio > 0) {
        const int roles = s_roles;
        prio_par = roles == 0 ? 0 : roles > 0 ? 1 : -1;
    }
    prio_par = __builtin_amdgcn_readfirstlane(prio_par);
    const unsigned wmask = (unsigned)kp.wrap_rows - 1u;
    // progress words: lane 0 writes the word, the others a sink (no exec-mask branch)
    int* const prod_out = lane == 0 ? &prod[wave] : &psink[wave][lane];
    int* const cons_out = lane == 0 ? &cons[wave] : &psink[wave][lane];
    int* const done_out = lane == 0 ? &done[wave] : &psink[wave][lane];
    int* const ready_out = lane == 0 ? &tabready : &psink[wave][lane];
    int base = 0, prev = 0;   // position bases of this round and the last
    int dseq = 0;             // duos this workgroup has begun
    // tools/probe_duo_simd.py: where each wave runs (HW_ID: SIMD, CU, SE; XCC_ID) and when
    const long long t_begin = (long long)__builtin_amdgcn_s_memrealtime();
    [[maybe_unused]] int spin_n = 0;   // polls (spin_expired)
    bool failed = false;
    for (int di = blockIdx.x; di < kp.npairs; di += gridDim.x, ++dseq) {
        const DuoDesc d = load_duo(kp, di);
        const int span = (d.m_pad + 64 * W - 1 + C - 1) / C * C + 128;
        if constexpr (TAB) {
            // wave 0: every wave done with the last duo's table; the others: this duo's first rows in
            if (wave < d.strips && !failed) {
                for (;;) {
                    const bool ok = wave == 0 ? min(min(lds_load(&done[1]), lds_load(&done[2])), lds_load(&done[3])) >= dseq
                                              : lds_load(&tabready) >= dseq + 1;
                    if (__builtin_amdgcn_readfirstlane((int)ok)) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (spin_expired(spin_n, t_begin, kp.timeout_ticks)) {
                        failed = true;
                        break;
                    }
                }
                compiler_fence();
            }
        }
        for (int r = 0; 4 * r < d.strips; ++r) {
            const int strip = 4 * r + wave;
            if (strip < d.strips) {
                const DuoLink<LIN> in{wave > 0 ? ring[wave - 1] : wrap, wave > 0 ? (unsigned)DUO_R - 1u : wmask,
                                      wave > 0 ? base : 0, wave > 0 ? base : prev, &prod[(wave + 3) & 3], nullptr};
                const DuoLink<LIN> out{wave < 3 ? ring[wave] : wrap, wave < 3 ? (unsigned)DUO_R - 1u : wmask,
                                       wave < 3 ? base : 0, base, nullptr, wave < 3 ? &cons[wave + 1] : nullptr};
                strip_pass_duo_lds<W, C, M3, LIN, TAB, RAW>(kp, d, strip, lane, strip > 0, in, strip + 1 < d.strips, out,
                                                       prod_out, cons_out, sink[wave], tab, strip == 0, ready_out,
                                                       dseq + 1, prio_par, t_begin);
            }
            // done with every position before the next round, read or not: a producer's back-pressure
            // must not wait on a consumer that skipped rounds (idle waves of a duo's last round) --
            // its word would stay below the producer's floor (found by a protocol simulation)
            compiler_fence();
            *cons_out = base + span;
            prev = base;
            base += span;
        }
        compiler_fence();
        *done_out = dseq + 1;   // this wave reads this duo's table no more
    }
    if (failed && lane == 0) atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
    if (kp.trace != nullptr && lane == 0) {
        unsigned long long* t = kp.trace + 4ull * (4u * blockIdx.x + (unsigned)wave);
        // HW_REG_HW_ID, and the strip role this wave ran at bit 40
        t[0] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((unsigned long long)wave << 40);
        t[1] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
        t[2] = (unsigned long long)t_begin;
        t[3] = __builtin_amdgcn_s_memrealtime();
    }
}

template <class K>
int occupancy_waves(K kernel, int threads = 256, int dyn = 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kernel, threads, dyn) != hipSuccess) return 4;
    return nb * threads / 64;
}

template <int W, int C, bool DNA>
hipError_t launch_t(const LaunchCfg& cfg, const KParams& kp, hipStream_t s) {
    switch (cfg.mode) {
        case MODE_STRIP: hipLaunchKernelGGL((sw_strip_kernel<W, C, DNA>), dim3(cfg.blocks), dim3(256), 0, s, kp); break;
        case MODE_PAIRWG: hipLaunchKernelGGL((sw_pairwg_kernel<W, C, DNA>), dim3(cfg.blocks), dim3(256), 0, s, kp); break;
        case MODE_CHAIN: hipLaunchKernelGGL((sw_chain_kernel<W, C, DNA>), dim3(cfg.blocks), dim3(256), 0, s, kp); break;
        case MODE_FLOW:
            if constexpr (DNA) {
                const int dyn = flow_stage_rows(cfg.max_m, W, C);
                if (dyn > flow_stage_max(W, C)) return hipErrorInvalidValue;
                if (dyn > 64 * 1024) {   // raise the dynamic-LDS limit (once per variant and device)
                    const hipError_t e = raise_dyn_lds((const void*)sw_flow_kernel<W, C>, flow_stage_max(W, C));
                    if (e != hipSuccess) return e;
                }
                hipLaunchKernelGGL((sw_flow_kernel<W, C>), dim3(cfg.blocks), dim3(256), (size_t)dyn, s, kp);
                break;
            }
            return hipErrorInvalidValue;
        case MODE_DUO:
            // byte batches (DNA false) run the same kernels with the penalty from the bytes (RAW)
            if constexpr (C == 64) {
                if (cfg.duo_wrap > 0) {   // every hand-off in LDS
                    const int dyn = duo_lds_dyn(cfg);
                    if (dyn > DUO_LDS_DYN_MAX) return hipErrorInvalidValue;
                    auto go = [&](auto kern) -> hipError_t {
                        // the wrap buffer, the code table and the static rings may pass 64 KB together
                        const hipError_t e = raise_dyn_lds((const void*)kern, DUO_LDS_DYN_MAX);
                        if (e != hipSuccess) return e;
                        hipLaunchKernelGGL(kern, dim3(cfg.blocks), dim3(64 * DUO_WAVES), (size_t)dyn, s, kp);
                        return hipGetLastError();
                    };
                    if constexpr (W % 4 == 0) {
                        if (cfg.duo_tab > 0) {
                            if (cfg.duo_f16 && cfg.f2_lin) return go(sw_duo_lds_kernel<W, C, true, true, true, !DNA>);
                            if (cfg.duo_f16) return go(sw_duo_lds_kernel<W, C, true, false, true, !DNA>);
                            return go(sw_duo_lds_kernel<W, C, false, false, true, !DNA>);
                        }
                    }
                    if (cfg.duo_f16 && cfg.f2_lin) return go(sw_duo_lds_kernel<W, C, true, true, false, !DNA>);
                    if (cfg.duo_f16) return go(sw_duo_lds_kernel<W, C, true, false, false, !DNA>);
                    return go(sw_duo_lds_kernel<W, C, false, false, false, !DNA>);
                }
            }
            {
                // the linear-gap step (G_INIT == G_EXT) is built with the f16-max3 form
                if (cfg.duo_f16 && cfg.f2_lin)
                    hipLaunchKernelGGL((sw_duo_kernel<W, C, true, true, !DNA>), dim3(cfg.blocks), dim3(64 * DUO_WAVES), 0, s, kp);
                else if (cfg.duo_f16)
                    hipLaunchKernelGGL((sw_duo_kernel<W, C, true, false, !DNA>), dim3(cfg.blocks), dim3(64 * DUO_WAVES), 0, s, kp);
                else
                    hipLaunchKernelGGL((sw_duo_kernel<W, C, false, false, !DNA>), dim3(cfg.blocks), dim3(64 * DUO_WAVES), 0, s, kp);
                break;
            }
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int W, int C, bool DNA>
int waves_t(const LaunchCfg& cfg) {
    const int mode = cfg.mode;
    if constexpr (C == 64) {
        if (mode == MODE_DUO && cfg.duo_wrap > 0) {
            const int dyn = duo_lds_dyn(cfg);
            if constexpr (W % 4 == 0) {
                if (cfg.duo_tab > 0)
                    return cfg.f2_lin    ? occupancy_waves(sw_duo_lds_kernel<W, C, true, true, true, !DNA>, 64 * DUO_WAVES, dyn)
                           : cfg.duo_f16 ? occupancy_waves(sw_duo_lds_kernel<W, C, true, false, true, !DNA>, 64 * DUO_WAVES, dyn)
                                         : occupancy_waves(sw_duo_lds_kernel<W, C, false, false, true, !DNA>, 64 * DUO_WAVES, dyn);
            }
            return cfg.f2_lin    ? occupancy_waves(sw_duo_lds_kernel<W, C, true, true, false, !DNA>, 64 * DUO_WAVES, dyn)
                   : cfg.duo_f16 ? occupancy_waves(sw_duo_lds_kernel<W, C, true, false, false, !DNA>, 64 * DUO_WAVES, dyn)
                                 : occupancy_waves(sw_duo_lds_kernel<W, C, false, false, false, !DNA>, 64 * DUO_WAVES, dyn);
        }
    }
    switch (mode) {
        case MODE_STRIP: return occupancy_waves(sw_strip_kernel<W, C, DNA>);
        case MODE_PAIRWG: return occupancy_waves(sw_pairwg_kernel<W, C, DNA>);
        case MODE_CHAIN: return occupancy_waves(sw_chain_kernel<W, C, DNA>);
        case MODE_FLOW:
            if constexpr (DNA) return occupancy_waves(sw_flow_kernel<W, C>);
            return 0;
        case MODE_DUO:
            return occupancy_waves(sw_duo_kernel<W, C, true, false, !DNA>, 64 * DUO_WAVES);
        default: return 4;
    }
}

}  // namespace

#define SW_VARIANTS(X) X(1, 16) X(1, 32) X(2, 32) X(4, 64) X(8, 64)

bool variant_exists(int W, int C) {
#define SW_EXISTS(w, c) if (W == w && C == c) return true;
    SW_VARIANTS(SW_EXISTS)
#undef SW_EXISTS
    return false;
}

hipError_t launch_sw_strip(const LaunchCfg& cfg, const KParams& kp, hipStream_t stream) {
#define SW_LAUNCH(w, c)                                                           \
    if (cfg.W == w && cfg.C == c)                                                 \
        return cfg.dna ? launch_t<w, c, true>(cfg, kp, stream) : launch_t<w, c, false>(cfg, kp, stream);
    SW_VARIANTS(SW_LAUNCH)
#undef SW_LAUNCH
    return hipErrorInvalidValue;
}

int kernel_waves_per_cu(const LaunchCfg& cfg) {
#define SW_OCC(w, c) \
    if (cfg.W == w && cfg.C == c) return cfg.dna ? waves_t<w, c, true>(cfg) : waves_t<w, c, false>(cfg);
    SW_VARIANTS(SW_OCC)
#undef SW_OCC
    return 4;
}

}  // namespace swmi
