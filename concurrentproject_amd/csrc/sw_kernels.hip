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
// Work decomposition (Kernel):
//   * a WAVE owns a strip of 64*W consecutive columns; lane l holds columns
//     [l*W, l*W+W) of the strip in registers;
//   * the wave sweeps the strip's rows as an anti-diagonal wavefront: at step k
//     every (lane, position) computes the cell of anti-diagonal k, so the W
//     cells of a lane are independent (ILP) and the left neighbour of position
//     0 is the previous step's position W-1 of lane l-1: ONE wave_shr:1 DPP
//     move per flowing quantity (H-G_INIT, E-G_EXT, row code) per step;
//   * the strip's left column enters at lane 0 and its right column leaves at
//     lane 63 through one "combined" register per quantity that is rotated by
//     wave_shl:1 every step (lane 0 consumes the next inflow, lane 63 collects
//     the outflow), so C rows of hand-off cost one 16-byte load and one
//     16-byte store per lane per C steps;
//   * strips hand off through tagged 16-byte granules (write-through sc1
//     stores, sc1 polls; no fences), and waves claim (pair, strip) items
//     strictly in order from one atomic counter, so a consumer's producer has
//     always been claimed by a running wave: no co-residency assumption, no
//     deadlock, any grid size.
#include "sw_internal.h"

namespace swmi {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int DPP_WAVE_SHL1 = 0x130;
constexpr int DPP_WAVE_SHR1 = 0x138;
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
__device__ __forceinline__ int dpp_shl1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, DPP_WAVE_SHL1, 0xF, 0xF, false);
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// 'A','C','G','T' -> 0,1,2,3  (only used when the host verified the alphabet)
__device__ __forceinline__ int dna_code(unsigned c) { return (int)(((c >> 1) ^ (c >> 2)) & 3u); }

// One anti-diagonal step for the W positions of a lane.
//   hgCur : on entry H-G_INIT two steps ago (diagonal source); on exit this step's
//   hgPrev: H-G_INIT of the previous step (left source for p>0, up source for F)
//   eh, r : E-G_EXT and row code of the previous step, updated in place
//   fh    : F-G_EXT of the previous step (own column), updated in place
// Positions are processed from W-1 down to 0 so that the in-place arrays still
// hold the previous step's value of p-1 when position p reads it.
template <int W, bool DNA>
__device__ __forceinline__ void sw_step(int (&hgCur)[W], const int (&hgPrev)[W], int (&eh)[W], int (&r)[W],
                                        int (&fh)[W], const int (&prof)[W], const int (&tb)[W], int& L0,
                                        int& IOH, int& IOE, int& IOR, int& M, const int go, const int ge,
                                        const int ma, const int mi) {
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
        const int t = hgD + s + tb[p];                 // H[i-1][j-1] + s(q_j, d_i)   (v_add3_u32)
        const int E = max3i(ehL, hgL, 0);              // clamped E
        const int F = max3i(fh[p], hgPrev[p], 0);      // clamped F
        const int H = max3i(t, E, F);
        M = max(M, t);
        hgCur[p] = H - go;
        eh[p] = E - ge;
        fh[p] = F - ge;
        r[p] = rL;
    }
    L0 = hgL0;
    IOH = dpp_shl1(hgCur[W - 1], IOH);   // lane 63 <- this step's right-edge output
    IOE = dpp_shl1(eh[W - 1], IOE);
    IOR = dpp_shl1(IOR, IOR);
}

struct RowFetch {
    int code;
    u32x4 g;
};

template <int W, int C, bool DNA>
__device__ __forceinline__ RowFetch fetch_rows(const __amdgpu_buffer_rsrc_t row_rsrc, const __amdgpu_buffer_rsrc_t in_rsrc,
                                               bool has_in, int k0, int lane, int m) {
    RowFetch f;
    const int row = k0 + lane;
    const bool live = lane < C && row < m;
    const unsigned ch = __builtin_amdgcn_raw_buffer_load_b8(row_rsrc, live ? (unsigned)row : OOR, 0, 0);
    if constexpr (DNA) f.code = live ? (dna_code(ch) | 0x0C0C0C00) : SENT_DNA;
    else f.code = live ? (int)ch : SENT_BYTE;
    if (has_in) {
        f.g = __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, live ? (unsigned)row * 16u : OOR, 0, AUX_SC1);
    } else {
        f.g = u32x4{0u, 0u, 0u, 0u};
    }
    return f;
}

__device__ __forceinline__ bool granule_ok(const u32x4& g, unsigned epoch, int row) {
    return g.x == epoch && g.w == granule_chk(epoch, (int)g.y, (int)g.z, row);
}

template <int W, int C, bool DNA>
__device__ void sw_item(const KParams& kp, const PairDesc& pd, const int strip, const int lane) {
    constexpr int SW = 64 * W;
    static_assert(C % 4 == 0 && C <= 64, "chunk");
    const int n = pd.n, m = pd.m;
    const int go = kp.gap_init, ge = kp.gap_ext, ma = kp.match, mi = kp.mismatch;
    const unsigned epoch = kp.epoch;
    const unsigned char* colseq = kp.seq + pd.col_off;

    // ---- column state (fixed for the strip) --------------------------------
    int prof[W], tb[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
        const int c = strip * SW + lane * W + p;
        if (c < n) {
            const unsigned ch = colseq[c];
            if constexpr (DNA) {
                const int code = dna_code(ch);
                const unsigned pw = code == 0 ? kp.prof[0] : code == 1 ? kp.prof[1] : code == 2 ? kp.prof[2] : kp.prof[3];
                prof[p] = (int)pw;
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

    // ---- DP state: everything starts at the border (H = E = F = 0) --------
    int hgA[W], hgB[W], eh[W], r[W], fh[W];
    const int sent = DNA ? SENT_DNA : SENT_BYTE;
#pragma unroll
    for (int p = 0; p < W; ++p) {
        hgA[p] = -go; hgB[p] = -go; eh[p] = -ge; fh[p] = -ge; r[p] = sent;
    }
    int L0 = -go, M = 0;
    int IOH = -go, IOE = -ge, IOR = sent;

    const bool has_in = strip > 0;
    const bool has_out = strip < pd.strips - 1;
    Granule* in_base = kp.bnd + pd.bnd_off + (uint64_t)(has_in ? strip - 1 : 0) * (uint64_t)m;
    Granule* out_base = kp.bnd + pd.bnd_off + (uint64_t)strip * (uint64_t)m;
    const __amdgpu_buffer_rsrc_t in_rsrc = __builtin_amdgcn_make_buffer_rsrc(in_base, 0, m * 16, RSRC_FLAGS);
    const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(out_base, 0, m * 16, RSRC_FLAGS);
    const __amdgpu_buffer_rsrc_t row_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + pd.row_off), 0, m, RSRC_FLAGS);

    const int total_steps = m + SW - 1;
    const int nchunks = (total_steps + C - 1) / C;
    bool failed = false;

    RowFetch nxt = fetch_rows<W, C, DNA>(row_rsrc, in_rsrc, has_in, 0, lane, m);
    for (int c = 0; c < nchunks; ++c) {
        const int k0 = c * C;
        RowFetch cur = nxt;
        const int row = k0 + lane;
        if (has_in && !failed) {
            bool ok = lane >= C || row >= m || granule_ok(cur.g, epoch, row);
            if (!__all(ok)) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                for (;;) {
                    __builtin_amdgcn_s_sleep(1);
                    if (!ok) cur.g = __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, (unsigned)row * 16u, 0, AUX_SC1);
                    ok = lane >= C || row >= m || granule_ok(cur.g, epoch, row);
                    if (__all(ok)) break;
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks) {
                        if (lane == 0) {
                            atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
                            atomicMax(&kp.ctrl->err_item, (unsigned)strip);
                        }
                        failed = true;
                        break;
                    }
                }
            }
        }
        // next chunk's rows in flight while this chunk computes
        if (c + 1 < nchunks) nxt = fetch_rows<W, C, DNA>(row_rsrc, in_rsrc, has_in, k0 + C, lane, m);

        if (lane < C) {
            const bool real = has_in && row < m;
            IOH = real ? (int)cur.g.y : -go;
            IOE = real ? (int)cur.g.z : -ge;
            IOR = cur.code;
        }

#pragma unroll 2
        for (int s = 0; s < C; s += 2) {
            sw_step<W, DNA>(hgA, hgB, eh, r, fh, prof, tb, L0, IOH, IOE, IOR, M, go, ge, ma, mi);
            sw_step<W, DNA>(hgB, hgA, eh, r, fh, prof, tb, L0, IOH, IOE, IOR, M, go, ge, ma, mi);
        }

        if (has_out) {
            // lanes [64-C, 64) hold the right-edge (H-G_INIT, E-G_EXT) of steps k0..k0+C-1,
            // i.e. rows k - (SW-1).
            const int row_out = k0 + (lane - (64 - C)) - (SW - 1);
            const bool st = lane >= 64 - C && row_out >= 0 && row_out < m;
            u32x4 g;
            g.x = epoch;
            g.y = (unsigned)IOH;
            g.z = (unsigned)IOE;
            g.w = granule_chk(epoch, IOH, IOE, row_out);
            __builtin_amdgcn_raw_buffer_store_b128(g, out_rsrc, st ? (unsigned)row_out * 16u : OOR, 0, AUX_SC1);
        }
    }

    // wave max, then one device-scope atomic per (pair, strip)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) M = max(M, __shfl_xor(M, off));
    if (lane == 0 && M > 0) atomicMax(&kp.scores[pd.out_idx], M);
}

template <int W, int C, bool DNA>
__global__ void __launch_bounds__(256) sw_strip_kernel(KParams kp) {
    const int lane = threadIdx.x & 63;
    for (;;) {
        unsigned item = 0;
        if (lane == 0) item = atomicAdd(&kp.ctrl->next_item, 1u);
        item = __builtin_amdgcn_readfirstlane(item);
        if ((int)item >= kp.total_items) return;
        int lo = 0, hi = kp.npairs - 1;   // last pair with item_base <= item
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (kp.item_base[mid] <= (int)item) lo = mid; else hi = mid - 1;
        }
        // every field made provably wave-uniform: the buffer descriptors built
        // from them must live in SGPRs (no waterfall loops, guide T20)
        const PairDesc raw = kp.pairs[lo];
        PairDesc pd;
        pd.col_off = uniform64(raw.col_off);
        pd.row_off = uniform64(raw.row_off);
        pd.bnd_off = uniform64(raw.bnd_off);
        pd.n = __builtin_amdgcn_readfirstlane(raw.n);
        pd.m = __builtin_amdgcn_readfirstlane(raw.m);
        pd.strips = __builtin_amdgcn_readfirstlane(raw.strips);
        pd.out_idx = __builtin_amdgcn_readfirstlane(raw.out_idx);
        const int strip = __builtin_amdgcn_readfirstlane((int)item - kp.item_base[lo]);
        sw_item<W, C, DNA>(kp, pd, strip, lane);
    }
}

template <int W, int C, bool DNA>
hipError_t launch_t(const LaunchCfg& cfg, const KParams& kp, hipStream_t s) {
    hipLaunchKernelGGL((sw_strip_kernel<W, C, DNA>), dim3(cfg.blocks), dim3(256), 0, s, kp);
    return hipGetLastError();
}

template <int W, int C, bool DNA>
int waves_t() {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)sw_strip_kernel<W, C, DNA>, 256, 0) != hipSuccess)
        return 4;
    return nb * 4;
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
    if (cfg.W == w && cfg.C == c) return cfg.dna ? waves_t<w, c, true>() : waves_t<w, c, false>();
    SW_VARIANTS(SW_OCC)
#undef SW_OCC
    return 4;
}

}  // namespace swmi
