// sw_flow2.hip -- the single-long-pair kernel (BASELINE config 2: one DNA pair,
// N = 65536) for gfx950.  Same recurrence and clamped arithmetic as
// sw_kernels.hip (main.cpp:54-66, DESIGN.md "Arithmetic"); what changes is how
// few instructions one anti-diagonal step costs.  For one long pair the time is
// (m + strips x lag) steps of ONE wave per SIMD issuing alone (one VALU instruction
// every ~2.05 ns, ~1.7 ns more per s_nop or SALU between two of them:
// tools/ubench_bank.hip), so every instruction of the step is on the critical path.
// The kernels that run many strips per SIMD (streamed, ring, slab, PWG) are bound
// by VALU issue instead (roofline.issue).
//
// The affine one-column step is described here; the linear-gap step (LIN) and the
// two-columns-per-lane step (W2, the automatic choice at G_INIT == G_EXT) below.
//
// Layout: a wave owns a strip of 64 columns, lane l = column 63*s + l.  Strips
// OVERLAP by one column: lane 0 of strip s+1 recomputes column 63*(s+1), the
// column of lane 63 of strip s.  Its left inputs (H - G_INIT, E - G_EXT of
// column 63s+62) are then exactly the values lane 63 of strip s computes in its
// own DPP step, so the hand-off needs no extra arithmetic.
//
// One step (lane l, row i = k - l), 10.5 VALU for 64 cells:
//   t    = L0 + s               L0 = last step's hgL (the diagonal); s is a
//                               signed byte s(q,d) + G_INIT, taken with an SDWA
//                               byte select from a v_perm_b32 of 4 rows' codes
//   IOx' = wave_shl1(IOx), lane 63 <- last step's (hgL, ehL)
//                               rotating I/O registers: lanes [0, C) enter a
//                               chunk holding the inflow rows, lanes [64-C, 64)
//                               leave it holding the outflow rows (one LDS read
//                               and one LDS write per chunk, not per step)
//   hgL  = v_add_u32_dpp(old = IOH, H, -G_INIT)   lanes 1..63: H[l-1] - G_INIT,
//   ehL  = v_add_u32_dpp(old = IOE, E, -G_EXT)    lane 0 keeps the inflow row
//   E    = max3(ehL, hgL, 0)    clamped E (H never sees E < 0)
//   F    = max3(fh, hgO, 0),  fh = F - G_EXT,  hgO = H - G_INIT
//   H    = max3(t, E, F),  M = max(M, t)
//
// Hand-offs: wave w -> w+1 of a workgroup through an LDS ring with progress
// words (as sw_flow_kernel); the workgroup edges through tagged HBM granules
// (sw_device.h).  Work items (groups of 4 strips) are claimed in order, so a
// producer is always resident: no co-residency assumption, any grid size (ring
// mode deals them statically instead, every block resident; PWG claims whole
// pairs).  Every spin is bounded by s_memrealtime and reports ERR_TIMEOUT.
#include <algorithm>
#include <type_traits>

#include "sw_device.h"

namespace swmi {
namespace {

constexpr int F2_R = 256;   // ring rows per link (power of two, >= 2C + 64)
#ifndef SW_F2_GPREF
#define SW_F2_GPREF 1       // cross-workgroup granules are loaded this many chunks ahead
#endif
#ifndef SW_F2_SPEC
#define SW_F2_SPEC 0        // >0: the next chunk's LDS inflow is read speculatively SW_F2_SPEC steps (a multiple of 4)
                            // before the chunk ends (C2 W2: off 3.153, 4 steps 3.26, 8 steps 3.146, 12 steps 3.21 ms)
#endif
#ifndef SW_F2_GPOS
#define SW_F2_GPOS 1        // chunk c+SW_F2_GPREF's granules are loaded after SW_F2_GPOS/4 of chunk c's steps
#endif
#ifndef SW_F2_HALFPUB
#define SW_F2_HALFPUB 1     // workgroup-edge strips publish granules every half chunk
#endif
#ifndef SW_F2_HALFLDS
#define SW_F2_HALFLDS 0     // 1: in-workgroup links hand off every half chunk (C2 3.63 -> 3.85 ms: slower)
#endif
#ifndef SW_F2_LOADER
#define SW_F2_LOADER 1      // staged kernel: a fifth wave loads the workgroup's granule inflow into LDS
#endif
#ifndef SW_F2_LDQ
#define SW_F2_LDQ 1         // loader: granule polls in flight (C2: 1 3.456, 2 3.473, 4 3.484 ms)
#endif
#ifndef SW_F2_LDSLEEP
#define SW_F2_LDSLEEP 0     // loader: s_sleep units between polls of a round
#endif
#ifndef SW_F2_LDIDLE
#define SW_F2_LDIDLE 0      // loader: s_sleep units after a round that moved nothing
#endif
#ifndef SW_F2_HALFIN_AHEAD
#define SW_F2_HALFIN_AHEAD 4   // steps before mid-chunk at which the second half's inflow is read
#endif

// v_add_u32_dpp wave_shr:1 with the destination tied to 'old': lanes 1..63 get
// src[l-1] + k, lane 0 (no source, bound_ctrl off) keeps old.  Inline asm because
// no builtin ties a DPP-VOP2 destination to a live register.  The hazard a VALU
// write of src -> DPP read of src needs (2 wait states) is invisible to the
// compiler inside asm, so the asm takes 'after', a value computed from src
// through >= 2 dependent instructions: the asm cannot issue sooner.
__device__ __forceinline__ int dpp_add_shr1_tied(int old, int src, int k, int after) {
    asm("v_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf ; dep %3"
        : "+v"(old) : "v"(src), "v"(k), "v"(after));
    return old;
}
// LIN: the I/O rotation ioh = wave_shl1(IOH) (lane 63 <- L0) and the tied DPP-add
// of hgL in one asm: the rotation, which does not depend on H, is the second
// instruction between the write of src (H) and its DPP read
__device__ __forceinline__ int rot_dpp_add(int io, int& rot, int src, int k, int after) {
    int old = io;
    asm("v_mov_b32_dpp %1, %0 wave_shl:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_add_u32_dpp %0, %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf ; dep %4"
        : "+v"(old), "+v"(rot) : "v"(src), "v"(k), "v"(after));
    return old;
}
#ifndef SW_F2_PRIO
#define SW_F2_PRIO 0        // staged kernel: s_setprio of the compute waves (the loader stays at 0)
#endif
#ifndef SW_F2_VISMAX
#define SW_F2_VISMAX 0      // 1: the staged W2 step's maxima compiler-visible (no asm-result nops; see step_lin2)
#endif
// max3: compiler-visible (VIS) or the inline-asm v_max3_i32 (sw_device.h vmax3)
template <bool VIS>
__device__ __forceinline__ int max3_sel(int a, int b, int c) {
    if constexpr (VIS) return max(max(a, b), c);
    else return vmax3(a, b, c);
}
// max(H - G, 0) for H >= 0 in one instruction (unsigned subtract, clamped at 0)
__device__ __forceinline__ int sub_clamp0(int h, int g) {
    return (int)__builtin_elementwise_sub_sat((unsigned)h, (unsigned)g);
}

// s_memrealtime with its wait inside the asm: nothing SMEM stays outstanding, so
// the compiler's LDS wait counts around a stamp stay exact (tools only)
__device__ __forceinline__ long long realtime_waited() {
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// gfx950 LDS serves unaligned dword reads (ds_read_b32 at any byte address)
__device__ __forceinline__ unsigned load_u32_unaligned(const unsigned char* p) {
    unsigned v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

#ifndef SW_F2_WIDECODES
#define SW_F2_WIDECODES 1   // a chunk's row codes in 16-B LDS reads (2 per 32 rows) instead of 4-B ones
#endif
// the C row codes lane l steps through in a chunk, C/4 dwords from p (any byte address)
template <int C>
__device__ __forceinline__ void load_codes(unsigned (&D)[C / 4], const unsigned char* p) {
    if constexpr (SW_F2_WIDECODES) {
        static_assert(C % 16 == 0, "16-B code reads");
#pragma unroll
        for (int u = 0; u < C / 4; u += 4) {
            u32x4 v;
            __builtin_memcpy(&v, p + 4 * u, 16);   // ds_read_b128 (unaligned LDS access)
            D[u] = v.x;
            D[u + 1] = v.y;
            D[u + 2] = v.z;
            D[u + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < C / 4; ++u) D[u] = load_u32_unaligned(p + 4 * u);
    }
}

// signed byte b of w (SDWA src_sel:BYTE_b with sext)
template <int B>
__device__ __forceinline__ int sbyte(unsigned w) {
    if constexpr (B == 3) return (int)w >> 24;
    else return (int)(signed char)(w >> (8 * B));
}

// STREAM (rows too long to stage, e.g. C5's 2^20): instead of the pair's staged
// codes, each wave keeps its own ring of F2_CR row codes in LDS -- row r in slot
// (r + 64) mod F2_CR, slots [0, C) mirrored behind the ring so that a lane's
// unaligned 4-row read never wraps -- and refills it one chunk ahead: C lanes load
// the raw bytes of chunk c+3 (buffer_load_ubyte, one chunk of latency cover) and
// store the codes of chunk c+2 (two ds_write_b8).  The step loop is unchanged.
constexpr int F2_CR = 256;

// RING: ring-mode edges (KParams::ring_rows > 0).  SLAB: a column slab with edges
// to / from other GPUs (KParams::slab_in / slab_out, system-scope hand-off loops).
// Separate instantiations, both with streamed codes, so the single-GPU linear-edge
// kernel (C2) carries none of their code.
//
// LIN: G_INIT == G_EXT (the reference's default constants, main.cpp:20-23).  Then
// E(i,j) = H(i,j-1) - G and F(i,j) = H(i-1,j) - G exactly: by induction
// E(i,j-1) <= H(i,j-1) (H is a max over E), so max(E(i,j-1) - G, H(i,j-1) - G)
// is the second term; the same for F.  The step keeps H only:
//   t   = H(i-1,j-1) + s            (SDWA add, as above)
//   hgL = v_add_u32_dpp(old = IOH, H, -G)   lanes 1..63: H(i,j-1) - G; lane 0 the inflow row
//   H   = max3(hgL, hgO, t)         hgO = max(H(i-1,j) - G, 0) of this lane's last step
//   hgO = max(H - G, 0)             v_sub_u32 with clamp (H >= 0): the floor at 0
// 5.5 VALU per step instead of 10.7; edges carry (H - G, H - G), which is also
// the exact (H - G_INIT, E - G_EXT) an affine consumer expects at G_INIT == G_EXT.
// LOADER (the staged kernel): the workgroup's first strip does not poll HBM for
// its inflow granules itself.  A fifth wave (no strip of its own) keeps
// SW_F2_LDQ granule loads of the next 64 rows in flight, spaced SW_F2_LDSLEEP
// apart, and moves every valid prefix into an LDS ring with a progress word, so
// wave 0 takes its inflow like any in-workgroup link (half chunks, one LDS round
// trip).  A published granule is then seen one load latency after it lands
// instead of a sleep + reload round trip after wave 0 next looks.
template <bool STREAM>
constexpr bool f2_loader() { return SW_F2_LOADER && !STREAM; }
template <bool STREAM>
constexpr int f2_threads() { return f2_loader<STREAM>() ? 320 : 256; }

// W2: two columns per lane (LIN only).  Strip s covers columns [126s, 126s + 128),
// lane l columns A = 126s + 2l and B = A + 1; strips overlap by two columns (lane 0
// of strip s+1 recomputes lane 63's pair), so the hand-off is exactly W = 1's: the
// outflow is lane 63's hgL_A = H(i, A - 1) - G, the left input of the next strip's
// lane 0.  Inside a lane B's left neighbour is A (same row, same step); A's left is
// lane l-1's B through the tied DPP-add.  10 VALU per step for 128 columns instead of
// 5.5 for 64, and half the strips: the wavefront's column term and the number of
// strip hops both halve.
//
// PWG (batches of pairs whose scores need int32, sw_engine.hip plan_flow2): a workgroup
// claims a whole pair and its 4 waves run all of its strips in rounds (wave w: strips w,
// w + 4, ...), every hand-off through the LDS rings (wave 3 -> wave 0 of the next round
// included): no granules, no cross-workgroup waits, so any grid size works.  Streamed codes.
template <int C, bool STREAM, bool RING, bool SLAB, bool LIN, bool W2 = false, bool PWG = false>
__global__ void __launch_bounds__(f2_threads<STREAM>()) sw_flow2_kernel(KParams kp) {
    static_assert(!(RING || SLAB) || STREAM, "ring and slab kernels stream the row codes");
    static_assert(!W2 || LIN, "two columns per lane: the linear-gap step only");
    static_assert(!PWG || (STREAM && !RING && !SLAB), "pair per workgroup: streamed codes, LDS links only");
    static_assert(!PWG || !SW_F2_HALFLDS, "pair per workgroup: whole-chunk LDS reads");
    static_assert(C % 4 == 0 && 64 % C == 0 && 2 * C + 64 <= F2_R, "chunk");
    // STREAM ring: during chunk c the reads span rows [k0 + C - 63, k0 + 2C) and the
    // writes rows [k0 + 2C, k0 + 3C): no slot is rewritten while still read
    static_assert(!STREAM || 3 * C + 63 <= F2_CR, "code ring");
    static_assert(SW_F2_SPEC % 4 == 0 && SW_F2_SPEC < C, "speculative inflow read");
    static_assert(!SW_F2_HALFLDS || (SW_F2_SPEC == 0 && SW_F2_HALFIN_AHEAD % 4 == 0 && SW_F2_HALFIN_AHEAD <= C / 2),
                  "half-chunk LDS links");
    // rows per LDS hand-off: the consumer needs rows [k0, k0 + HL) at the start of a
    // chunk and [k0 + HL, k0 + C) at its middle, so a link's lag is 64 + C/2 steps, not 64 + C
    constexpr int HL = SW_F2_HALFLDS ? C / 2 : C;
    constexpr int R = F2_R;
    constexpr bool LD = f2_loader<STREAM>();
    constexpr int NT = f2_threads<STREAM>();
    constexpr int NR = LD ? 5 : 4;           // LDS rings: one per compute wave (+ the loader's)
    constexpr int CRB = F2_CR + C + 64;      // STREAM ring + mirror + per-lane sinks, bytes per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char rc[];   // rc[row + 64]: 4..7 = A,C,G,T; 0 = no row (staged mode)
    __shared__ __attribute__((aligned(16))) unsigned char cring[STREAM ? 4 : 1][STREAM ? CRB : 16];
    __shared__ int2 ring[NR][R];             // ring w: outflow rows of wave w (row r in slot r mod R)
    __shared__ int2 sink[NR][64];            // lanes that publish nothing write here
    __shared__ int prod[NR], cons[NR], psink[NR][64];
    __shared__ int s_item;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const int go = kp.gap_init, ge = kp.gap_ext;
    for (int it = 0;; ++it) {
        // items are claimed in order (any grid size), or in ring mode dealt statically:
        // block j runs items j, j + G, j + 2G, ... (every block resident, see group_edge)
        if (tid == 0) s_item = RING ? (int)blockIdx.x + it * (int)gridDim.x : (int)atomicAdd(&kp.ctrl->next_item, 1u);
        __syncthreads();   // every wave is done with the previous item
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= kp.total_items) return;
        const int pi = PWG ? item : find_pair(kp, item);
        const PairDesc pd = load_pair(kp, pi);
        const int m = pd.m;
        const int group = item - kp.item_base[pi];
        const int nloc = (m + 64 + C - 1) / C;   // lane 63's last row is out at step m + 63
        if (tid < NR) { prod[tid] = 0; cons[tid] = 0; }
        for (int i = tid; i < NR * R; i += NT) ring[i / R][i % R] = make_int2(-go, -ge);
        const __amdgpu_buffer_rsrc_t row_rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(kp.seq + pd.row_off), 0, m, RSRC_FLAGS);
        if constexpr (!STREAM) {
            // 16 rows per thread and load (the first group's staging delays the whole
            // chain): rc[i .. i+16) = codes of rows i-64 .. i-49, 4 + code, 0 = no row
            const int nst = flow2_stage_bytes(m, C);   // a multiple of 16
            for (int i = tid * 16; i < nst; i += 16 * NT) {
                const int row0 = i - 64;
                u32x4 w = u32x4{0u, 0u, 0u, 0u};
                if (row0 >= 0 && row0 + 16 <= m) {
                    const u32x4 raw = __builtin_amdgcn_raw_buffer_load_b128(row_rsrc, (unsigned)row0, 0, 0);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        w[q] = (((raw[q] >> 1) ^ (raw[q] >> 2)) & 0x03030303u) | 0x04040404u;   // dna_code per byte
                } else if (row0 < m && row0 + 16 > 0) {   // the block holding row m-1: byte by byte
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const int row = row0 + j;
                        const bool live = row >= 0 && row < m;
                        const unsigned ch = __builtin_amdgcn_raw_buffer_load_b8(row_rsrc, live ? (unsigned)row : OOR, 0, 0);
                        w[j >> 2] |= (live ? 4u + (unsigned)dna_code(ch) : 0u) << (8 * (j & 3));
                    }
                }
                *reinterpret_cast<u32x4*>(rc + i) = w;
            }
        }
        __syncthreads();
        if (LD && wave == 4) {   // the loader wave: granule inflow of strip 4 * group (not group 0)
            if (group > 0 && 4 * group < pd.strips) {
                const Edge le = group_edge(kp, pd, group - 1, (pd.strips + 3) / 4);
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                [[maybe_unused]] int spin_n = 0;   // polls (spin_expired)
                int2* const lring = ring[4];
                int* const lprod = lane == 0 ? &prod[4] : &psink[4][lane];
                int base = 0, sent = 0, cseen = 0;
                bool lfail = false;
                // rounds of SW_F2_LDQ polls of the current 64-row window, spaced SW_F2_LDSLEEP
                // apart, then checked in issue order (no load crosses a round: a load whose
                // destination is carried around the loop would be copied, and the copy waits for it)
                while (base < m) {
                    const int b0 = base, sent0 = sent;
                    u32x4 q[SW_F2_LDQ];
#pragma unroll
                    for (int i = 0; i < SW_F2_LDQ; ++i) {
                        q[i] = fetch_granules<64>(le, b0, lane, m);
                        if (i + 1 < SW_F2_LDQ) __builtin_amdgcn_s_sleep(SW_F2_LDSLEEP);
                    }
#pragma unroll
                    for (int i = 0; i < SW_F2_LDQ; ++i) {
                        if (base == b0) {
                            const int row = b0 + lane;
                            const bool live = row < m;
                            const bool ok = (!live) | granule_ok(q[i], le, row);
                            const unsigned long long bal = __ballot(ok);
                            const int lead = bal == ~0ull ? 64 : (int)__builtin_ctzll(~bal);
                            if (b0 + lead > sent) {
                                int2* const dst = ok && live ? &lring[row & (R - 1)] : &sink[4][lane];
                                *dst = make_int2((int)q[i].y, (int)q[i].z);
                                compiler_fence();
                                sent = min(b0 + lead, m);
                                *lprod = sent;   // after the ring writes (in-order DS)
                            }
                            if (lead == 64) base = b0 + 64;
                        }
                    }
                    if (SW_F2_LDIDLE > 0 && sent == sent0) __builtin_amdgcn_s_sleep(SW_F2_LDIDLE);
                    // the next window's slots: rows < base + 64 - R must be consumed by wave 0
                    const int floor_rows = min(base, m) + 64 - R;
                    // the expiry is recorded where it is seen: a second spin_expired call after
                    // the loop would count one more poll and miss it (n no longer 0 mod 64)
                    while (cseen < floor_rows) {
                        cseen = __builtin_amdgcn_readfirstlane(lds_load(&cons[0]));
                        if (cseen >= floor_rows) break;
                        __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                        if (spin_expired(spin_n, t0, kp.timeout_ticks)) {
                            lfail = true;
                            break;
                        }
                    }
                    // the granule polls above are bounded the same way: the window's rows never
                    // arriving (a producer that failed) ends the loader as well
                    if (!lfail && sent == sent0 && spin_expired(spin_n, t0, kp.timeout_ticks)) lfail = true;
                    if (lfail) break;
                }
                if (lfail && lane == 0) {
                    atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
                    atomicMax(&kp.ctrl->err_item, (unsigned)(4 * group));
                }
            }
            continue;
        }
        if (item == kp.stall_item) continue;   // tests: this item's edges are never published
        // PWG: this workgroup runs every strip of the pair, wave w the strips w, w + 4, ...
        // (one per round); wave 3 hands off to wave 0 of the next round through LDS too.
        // Positions on every link: row r of round k at k * span + 128 + r (span = the
        // rows a round spans, so rounds never share a position, and a producer's first
        // publishes of round k need only what its consumer has read of round k - 1).
        const int nrounds = PWG ? (pd.strips + 3) / 4 : 1;
        const int span = PWG ? nloc * C : 0;
        for (int round = 0; round < nrounds; ++round) {
            const int strip = PWG ? 4 * round + wave : 4 * group + wave;
            if (strip >= pd.strips) break;
            if constexpr (LD && SW_F2_PRIO > 0) __builtin_amdgcn_s_setprio(SW_F2_PRIO);   // ahead of the loader on SIMD 0
            const int pb_out = PWG ? round * span + 128 : 0;                       // positions this strip publishes at
            const int pb_in = PWG ? (wave > 0 ? round : round - 1) * span + 128 : 0;   // and reads at
            const int col = W2 ? 126 * strip + 2 * lane : 63 * strip + lane;
            const unsigned prof = col < pd.n ? kp.prof2[dna_code(kp.seq[pd.col_off + col])] : 0x80808080u;
            // W2 column B takes its diagonal as H_A (not H_A - G): raw score bytes s
            const unsigned profB = W2 && col + 1 < pd.n ? kp.prof3[dna_code(kp.seq[pd.col_off + col + 1])] : 0x80808080u;
            // a multi-GPU column slab: the first strip takes the previous slab's edge, the
            // last one hands its lane-62 column (the next slab's left neighbour) on
            const int ngroups = (pd.strips + 3) / 4;
            const int in_kind = PWG ? (strip == 0 ? FLOW_NONE : wave == 0 ? FLOW_WRAP : FLOW_LDS)
                                : wave > 0 || (LD && strip > 0) ? FLOW_LDS
                                : strip > 0                     ? FLOW_GRANULE
                                : kp.slab_in != nullptr         ? FLOW_PEER
                                                                : FLOW_NONE;
            // the ring an LDS inflow comes from (4: the loader's; PWG wave 0: wave 3's, last round)
            const int in_w = wave > 0 ? wave - 1 : PWG ? 3 : 4;
            const int out_kind = strip + 1 >= pd.strips ? (kp.slab_out != nullptr ? FLOW_PEER : FLOW_NONE)
                                 : wave < 3             ? FLOW_LDS
                                 : PWG                  ? FLOW_WRAP
                                                        : FLOW_GRANULE;
            // PWG: the wave 3 -> wave 0 link holds a whole round in the dynamic LDS (the rows
            // of round k - 1 stay until wave 0 of round k has read them: wave 3 writes row x
            // of round k only after wave 0 of round k has computed row x, so it needs no
            // back-pressure, which would close a cycle of waits 0 -> 1 -> 2 -> 3 -> 0)
            int2* const wrapbuf = reinterpret_cast<int2*>(rc);   // affine: (H - G_INIT, E - G_EXT)
            int* const wrapbuf1 = reinterpret_cast<int*>(rc);    // LIN: H - G
            const Edge in_e = group_edge(kp, pd, group - 1, ngroups);
            const Edge out_e = group_edge(kp, pd, group, ngroups);
            // ring mode: the consumer of ring j reports the positions it has consumed in
            // ring_cons[j]; the producer never overwrites a slot whose position is not
            // consumed yet (back-pressure).  The wrap ring holds >= m rows and needs none:
            // its consumer (block 0, round k+1) has read row r of round k before the chain
            // of round k+1 lets block G-1 produce row r again.
            unsigned* cons_in = nullptr;
            unsigned* bp_word = nullptr;
            if constexpr (RING) {
                const int G = (int)gridDim.x;
                if (group > 0 && (group - 1) % G != G - 1) cons_in = kp.ring_cons + ((group - 1) % G) * RING_CONS_STRIDE;
                if (group < ngroups - 1 && group % G != G - 1) bp_word = kp.ring_cons + (group % G) * RING_CONS_STRIDE;
            }
            const bool cons_live = cons_in != nullptr;
            const __amdgpu_buffer_rsrc_t cons_rsrc = __builtin_amdgcn_make_buffer_rsrc(cons_live ? cons_in : nullptr, 0,
                                                                                        cons_live ? 4 : 0, RSRC_FLAGS);
            const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
            [[maybe_unused]] int spin_n = 0;   // polls (spin_expired)
            bool failed = false;
            long long t_first = t_start;
            int nslow = 0;   // chunks whose inflow took the slow path (trace only)
            int fail_in = -1, fail_bp = -1;   // RING trace: chunk whose inflow / back-pressure wait timed out
            long long tl[5] = {0, 0, 0, 0, 0};   // SW_TIMELINE: wall clock at chunks 1, 2, 3, 50, 1000
            // LIN keeps hgO clamped at 0 (see the step)
            int H = 0, E = 0, fh = -ge, hgO = LIN ? 0 : -go, L0 = -go, ehP = -ge, M = 0;
            int HB = 0, hgOB = 0;                     // W2: column B of the lane
            int IOH = -go, IOE = -ge;                 // rotating I/O registers (see the step)
            // -G_INIT, -G_EXT kept in VGPRs (operands of the DPP-adds, which take no SGPR)
            int neggo, negge;
            asm volatile("v_mov_b32 %0, %1" : "=v"(neggo) : "s"(-go));
            asm volatile("v_mov_b32 %0, %1" : "=v"(negge) : "s"(-ge));
            // progress words are written by every lane: lane 0 to the word, the others to sinks
            // (no exec-mask branch, so the compiler counts LDS operations exactly)
            int* const prod_out = lane == 0 ? &prod[wave] : &psink[wave][lane];
            int* const cons_out = lane == 0 ? &cons[wave] : &psink[wave][lane];
            int2* const in_ring = ring[in_w < NR ? in_w : 0];
            int2* const out_ring = ring[wave];
            // per-lane code address: lane l reads rows k - l .. k - l + 3 (unaligned dword)
            const unsigned char* const code_base = rc + 64 - lane;
            // STREAM: this wave's code ring; codes of chunk cc's rows from their raw bytes
            unsigned char* const cr = cring[STREAM ? wave : 0];
            auto raw_of = [&](const int cc) __attribute__((always_inline)) {
                const int row = cc * C + lane;
                return __builtin_amdgcn_raw_buffer_load_b8(row_rsrc, lane < C && row < m ? (unsigned)row : OOR, 0, 0);
            };
            auto put_codes = [&](const unsigned raw, const int cc) __attribute__((always_inline)) {
                const int row = cc * C + lane;
                const bool wl = lane < C;
                const unsigned char code = (unsigned char)(wl && row < m ? 4u + (unsigned)dna_code(raw) : 0u);
                const int s1 = wl ? ((row + 64) & (F2_CR - 1)) : F2_CR + C + lane;
                const int s2 = wl && s1 < C ? F2_CR + s1 : F2_CR + C + lane;
                cr[s1] = code;
                cr[s2] = code;
            };
            // where lane l's reads of chunk k0's rows start (STREAM: in the ring)
            auto code_at = [&](const int k0) __attribute__((always_inline)) -> const unsigned char* {
                if constexpr (STREAM) return cr + ((k0 + 64 - lane) & (F2_CR - 1));
                else return code_base + k0;
            };
            // STREAM: the raw bytes of chunk c+2, loaded during chunk c-1: one register
            // instead of a rotated pair (copying an in-flight load's destination makes the
            // compiler wait for that load; C5 430 -> 422 ms)
            unsigned rq0 = 0;
            if constexpr (STREAM) {
                for (int i = lane; i < CRB / 4; i += 64) reinterpret_cast<unsigned*>(cr)[i] = 0u;   // rows < 0: no row
                const unsigned r0 = raw_of(0), r1 = raw_of(1);
                put_codes(r0, 0);
                put_codes(r1, 1);
                rq0 = raw_of(2);
            }

            auto flow_loop = [&](auto in_c, auto out_c) __attribute__((always_inline)) {
                constexpr int IN = decltype(in_c)::value, OUT = decltype(out_c)::value;
                constexpr int AIN = flow_aux(IN), AOUT = flow_aux(OUT);
                // granule prefetch queue: gq[i] holds the loads for chunk c + i (issued SW_F2_GPREF chunks ahead)
                u32x4 gq[SW_F2_GPREF];
    #pragma unroll
                for (int i = 0; i < SW_F2_GPREF; ++i)
                    gq[i] = flow_granule(IN) ? fetch_granules<C, AIN>(in_e, i * C, lane, m) : u32x4{0u, 0u, 0u, 0u};
                unsigned D[C / 4];
                load_codes<C>(D, code_at(0));
                int cons_seen = 0;
                int h_avail = 0;                     // SW_F2_HALFLDS: the mid-chunk inflow read
                int2 h_v = make_int2(0, 0);
                int spec_avail = -1;                 // progress word read with spec_v (-1: none)
                int2 spec_v = make_int2(0, 0);
                // granule outflow at step k0 (chunk start, or mid-chunk with SW_F2_HALFPUB):
                // lane L >= 64 - C holds row k0 - 128 + L; with half-chunk publishing only
                // lanes >= 64 - C/2 are new
                unsigned bp_seen = 0;   // ring mode: last value read of the consumer's progress word
                auto publish_granules_half = [&](const int k0) __attribute__((always_inline)) {
                    const int row_out = k0 - 128 + lane;
                    constexpr int LO = SW_F2_HALFPUB ? 64 - C / 2 : 64 - C;
                    const bool st = lane >= LO && row_out >= 0 && row_out < m;
                    if (RING && bp_word != nullptr) {
                        // rows <= k0 - 65 go out: positions <= pos0 + k0 - 65 - R must be consumed.
                        // Also at the start of a round (k0 - 64 <= R): the slots then still hold the
                        // previous round's last rows, which the consumer (one hop behind, in that
                        // round) may not have read yet; `need` is then below pos0, in wrap-safe
                        // unsigned arithmetic, and in round 0 below 0, so always met.
                        const unsigned need = out_e.pos0 + (unsigned)(k0 - 64 - kp.ring_rows);
                        if ((int)(bp_seen - need) < 0) {
                            bp_seen = __builtin_amdgcn_readfirstlane(
                                __hip_atomic_load(bp_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                            while ((int)(bp_seen - need) < 0) {
                                __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                bp_seen = __builtin_amdgcn_readfirstlane(
                                    __hip_atomic_load(bp_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                                if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                    failed = true;
                                    if (fail_bp < 0) fail_bp = k0;
                                    break;
                                }
                            }
                        }
                    }
                    edge_publish<AOUT>(out_e, row_out, st, IOH, LIN ? IOH : IOE);
                };
                // ---- publish the last chunk's outflow: lane L >= 64 - C holds row k0 - 128 + L
                auto publish = [&](const int k0) __attribute__((always_inline)) {
                    const int row_out = k0 - 128 + lane;
                    if constexpr (OUT == FLOW_WRAP) {
                        const bool st = lane >= 64 - HL && row_out >= 0;
                        if constexpr (LIN) {   // (H - G, H - G): one int per row
                            int* const dst = st ? &wrapbuf1[row_out] : &psink[wave][lane];
                            *dst = IOH;
                        } else {
                            int2* const dst = st ? &wrapbuf[row_out] : &sink[wave][lane];
                            *dst = make_int2(IOH, IOE);
                        }
                        compiler_fence();
                        *prod_out = pb_out + max(0, k0 - 64);   // after the buffer writes (in-order DS)
                    } else if constexpr (OUT == FLOW_LDS) {
                        // ring slots of rows < k0 - 64 - R must have been read
                        const int floor_rows = pb_out + k0 - 64 - R;
                        int* const cons_next = &cons[(wave + 1) & 3];   // PWG wave 3: wave 0 of the next round
                        if (cons_seen < floor_rows) {
                            cons_seen = __builtin_amdgcn_readfirstlane(lds_load(cons_next));
                            while (cons_seen < floor_rows) {
                                __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                cons_seen = __builtin_amdgcn_readfirstlane(lds_load(cons_next));
                                if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                    failed = true;
                                    break;
                                }
                            }
                        }
                        int2* const dst = lane >= 64 - HL ? &out_ring[(pb_out + row_out) & (R - 1)] : &sink[wave][lane];
                        *dst = make_int2(IOH, LIN ? IOH : IOE);
                        compiler_fence();
                        *prod_out = pb_out + max(0, k0 - 64);   // after the ring writes (in-order DS)
                    } else if constexpr (flow_granule(OUT)) {
                        publish_granules_half(k0);
                    }
                };
                for (int c = 0; c < nloc; ++c) {
                    const int k0 = c * C;
    #ifdef SW_TIMELINE
                    if (c == 1 || c == 2 || c == 3 || c == 50 || c == 1000)
                        tl[c == 1 ? 0 : c == 2 ? 1 : c == 3 ? 2 : c == 50 ? 3 : 4] = realtime_waited();
    #endif
                    // ---- inflow rows [k0, k0 + C), for lanes [0, C) of the I/O registers
                    int newH, newE;
                    if constexpr (flow_granule(IN)) {
                        u32x4 g = gq[0];
                        if (kp.trace != nullptr) {   // tools: count chunks whose granules were not there yet
                            const int row = k0 + lane;
                            const bool need = lane < C && row < m;
                            nslow += __all((!need) | granule_ok(g, in_e, row)) ? 0 : 1;
                        }
                        await_granules<C, AIN>(kp, in_e, g, k0, lane, m, strip, failed);
                        if constexpr (RING) {
                            if (kp.trace != nullptr && failed && fail_in < 0) fail_in = k0;
                        }
                        // ring mode: rows < k0 + C are consumed (reported every 4th chunk and at
                        // the last).  An unconditional store, dropped (offset OOR) where there is
                        // nothing to report: no branch around a memory op in the chunk loop.
                        if constexpr (RING)
                            __builtin_amdgcn_raw_buffer_store_b32(
                                in_e.pos0 + (unsigned)min(k0 + C, m), cons_rsrc,
                                cons_live && lane == 0 && ((c & 3) == 3 || c == nloc - 1) ? 0u : OOR, 0, AUX_SC1);
    #pragma unroll
                        for (int i = 0; i + 1 < SW_F2_GPREF; ++i) gq[i] = gq[i + 1];
                        if constexpr (SW_F2_GPOS == 0)
                            gq[SW_F2_GPREF - 1] = fetch_granules<C, AIN>(in_e, k0 + SW_F2_GPREF * C, lane, m);
                        const bool live = k0 + lane < m;
                        newH = live ? (int)g.y : -go;
                        newE = live ? (int)g.z : -ge;
                    } else if constexpr (IN == FLOW_LDS || IN == FLOW_WRAP) {
                        const int need = pb_in + min(k0 + HL, m);
                        // the rows' slots: the producer's ring, or (WRAP) the round buffer
                        auto in_slot = [&](const int row) __attribute__((always_inline)) -> int2 {
                            if constexpr (IN == FLOW_WRAP && LIN) {
                                const int h = wrapbuf1[row];
                                return make_int2(h, h);
                            } else if constexpr (IN == FLOW_WRAP) {
                                return wrapbuf[row];
                            } else {
                                return in_ring[(pb_in + row) & (R - 1)];
                            }
                        };
                        int2 v;
                        if constexpr (SW_F2_SPEC > 0 && IN == FLOW_LDS) {
                            // the rows were read speculatively during the last chunk, behind a read
                            // of the progress word; only if that word did not cover them, poll and re-read
                            v = spec_v;
                            if (__builtin_amdgcn_readfirstlane(spec_avail) < need) {
                                ++nslow;
                                int avail = __builtin_amdgcn_readfirstlane(lds_load(&prod[in_w]));
                                while (avail < need) {
                                    __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                    avail = __builtin_amdgcn_readfirstlane(lds_load(&prod[in_w]));
                                    if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                        failed = true;
                                        break;
                                    }
                                }
                                compiler_fence();
                                v = in_slot(k0 + (lane & (C - 1)));
                            }
                        } else {
                            // the progress word and the chunk's rows in one LDS round trip (DS ops
                            // of a wave execute in order: rows read after a word that covers them
                            // are complete); re-read both until the word covers the chunk
                            int avail = lds_load(&prod[in_w]);
                            compiler_fence();
                            v = in_slot(k0 + (lane & (HL - 1)));
                            if (__builtin_amdgcn_readfirstlane(avail) < need) {
                                ++nslow;
                                do {
                                    __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                    avail = lds_load(&prod[in_w]);
                                    compiler_fence();
                                    v = in_slot(k0 + (lane & (HL - 1)));
                                    if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                        failed = true;
                                        break;
                                    }
                                } while (__builtin_amdgcn_readfirstlane(avail) < need);
                            }
                        }
                        newH = v.x;
                        newE = v.y;
                        if constexpr (IN == FLOW_WRAP) {
                            // rows >= m of the round buffer may hold anything (never written in
                            // this pass): the border values instead, as for granule inflow
                            const bool live = k0 + lane < m;
                            newH = live ? newH : -go;
                            newE = live ? newE : -ge;
                        }
                    } else {
                        newH = -go;
                        newE = -ge;
                    }
                    // ---- scores of the chunk's rows: one v_perm_b32 per 4 rows
                    unsigned P[C / 4], PB[W2 ? C / 4 : 1];
    #pragma unroll
                    for (int u = 0; u < C / 4; ++u) P[u] = __builtin_amdgcn_perm(prof, 0x80808080u, D[u]);
                    if constexpr (W2) {
    #pragma unroll
                        for (int u = 0; u < C / 4; ++u) PB[u] = __builtin_amdgcn_perm(profB, 0x80808080u, D[u]);
                    }
                    // take the inflow (and the scores) into registers before this chunk's LDS
                    // writes are issued, so the waits for them do not also wait for the writes
                    asm volatile("" : "+v"(newH), "+v"(newE));
                    if (c > 0) publish(k0);
                    IOH = newH;
                    IOE = newE;
                    if constexpr (IN == FLOW_LDS || IN == FLOW_WRAP) {
                        compiler_fence();
                        *cons_out = pb_in + k0 + HL;   // after the ring read (DS ops execute in order)
                    }
    #ifdef SW_TIMELINE
                    if (c == 0) t_first = realtime_waited();
    #endif
                    if constexpr (STREAM) {   // refill the ring: codes of chunk c+2, raw bytes of chunk c+3
                        put_codes(rq0, c + 2);
                        rq0 = raw_of(c + 3);
                    }
                    load_codes<C>(D, code_at(k0 + C));
                    // ---- C anti-diagonal steps
    #pragma unroll
                    for (int j = 0; j < C; j += 4) {
                        if constexpr (flow_granule(IN) && SW_F2_GPOS > 0) {
                            if (j == SW_F2_GPOS * C / 4) gq[SW_F2_GPREF - 1] = fetch_granules<C, AIN>(in_e, k0 + SW_F2_GPREF * C, lane, m);
                        }
                        if constexpr (flow_granule(OUT) && SW_F2_HALFPUB) {
                            // lanes [64 - C/2, 64) hold this chunk's first C/2 outflow rows
                            if (j == C / 2) publish_granules_half(k0 + C / 2);
                        }
                        if constexpr (OUT == FLOW_LDS && SW_F2_HALFLDS) {
                            if (j == C / 2) publish(k0 + C / 2);
                        }
                        if constexpr (IN == FLOW_LDS && SW_F2_HALFLDS) {
                            // the second half of the chunk's inflow: rows [k0 + C/2, k0 + C) go into
                            // lanes [0, C/2) of the I/O registers just before step C/2, when lanes
                            // [C/2, C) of the chunk start have rotated down there
                            if (j == C / 2 - SW_F2_HALFIN_AHEAD) {
                                h_avail = lds_load(&prod[in_w]);
                                compiler_fence();
                                h_v = in_ring[(pb_in + k0 + HL + (lane & (HL - 1))) & (R - 1)];
                            }
                            if (j == C / 2) {
                                const int need = pb_in + min(k0 + C, m);
                                if (__builtin_amdgcn_readfirstlane(h_avail) < need) {
                                    ++nslow;
                                    do {
                                        __builtin_amdgcn_s_sleep(SW_SPIN_SLEEP);
                                        h_avail = lds_load(&prod[in_w]);
                                        compiler_fence();
                                        h_v = in_ring[(pb_in + k0 + HL + (lane & (HL - 1))) & (R - 1)];
                                        if (spin_expired(spin_n, t_start, kp.timeout_ticks)) {
                                            failed = true;
                                            break;
                                        }
                                    } while (__builtin_amdgcn_readfirstlane(h_avail) < need);
                                }
                                IOH = lane < HL ? h_v.x : IOH;
                                if constexpr (!LIN) IOE = lane < HL ? h_v.y : IOE;
                                compiler_fence();
                                *cons_out = pb_in + k0 + C;   // after the ring read
                            }
                        }
                        if constexpr (IN == FLOW_LDS && SW_F2_SPEC > 0) {
                            if (j == C - SW_F2_SPEC) {   // speculative read of the next chunk's inflow
                                spec_avail = lds_load(&prod[in_w]);
                                compiler_fence();
                                spec_v = in_ring[(pb_in + k0 + C + (lane & (C - 1))) & (R - 1)];
                                compiler_fence();
                            }
                        }
                        auto step_lin = [&](auto b_c) __attribute__((always_inline)) {
                            constexpr int b = decltype(b_c)::value;
                            // 5.5 VALU: hgO = max(H - G, 0) in one clamped subtract carries the floor
                            // at 0, so H = max(t, hgL, H_up - G, 0) = max3(hgL, hgO, t); hgL is a
                            // tied DPP-add straight out of H, so the chain is H -> DPP-add -> max3
                            // (C2 4.21 -> 3.64 ms, C5 285 -> 251 ms against H = max(max3(hgL, hgO, 0), t)
                            // with hgO = H - G and hgL shifted out of hgO)
                            const int t = L0 + sbyte<b>(P[j >> 2]);
                            int ioh = L0;
                            const int hgL = rot_dpp_add(IOH, ioh, H, neggo, hgO);
                            IOH = ioh;
                            H = vmax3(hgL, hgO, t);
                            hgO = sub_clamp0(H, go);
                            M = max(M, t);
                            L0 = hgL;
                        };
                        auto step_lin2 = [&](auto b_c) __attribute__((always_inline)) {
                            constexpr int b = decltype(b_c)::value;
                            // 9 VALU for 128 cells.  Column A: as step_lin, with H_B of lane l-1 as
                            // the left input.  Column B: diagonal = H_A of the last row taken
                            // unshifted with the raw score byte (tB = H_A + s), left = max(H_A - G, 0)
                            // of this row, which is hgO_A: the clamp only adds the 0 that
                            // H = max(0, ...) has anyway, so no separate H_A - G is needed
                            // The maxima stay inline asm (vmax3) although the compiler pads a read of an
                            // asm result in the next instruction with s_nop 0 (it assumes a 16-bit dst_sel
                            // write).  Compiler-visible maxima removed C2's 16-20 nops per 32 steps but the
                            // kernel got slower (3.15 -> 3.30 ms: a lone wave's 4-step body times the same
                            // either way, tools/ubench_w2seq.hip, and the rest of the chunk scheduled worse),
                            // and the streamed kernels grew from 93 to 135 VGPRs (ring mode needs <= 128).
                            const int tA = L0 + sbyte<b>(P[j >> 2]);
                            const int tB = H + sbyte<b>(PB[j >> 2]);
                            int ioh = L0;
                            const int hgL = rot_dpp_add(IOH, ioh, HB, neggo, hgOB);   // HB -> hgOB -> DPP
                            IOH = ioh;
                            H = max3_sel<SW_F2_VISMAX && !STREAM>(hgL, hgO, tA);
                            hgO = sub_clamp0(H, go);
                            HB = max3_sel<SW_F2_VISMAX && !STREAM>(hgO, hgOB, tB);
                            hgOB = sub_clamp0(HB, go);
                            M = max3_sel<SW_F2_VISMAX && !STREAM>(M, tA, tB);
                            L0 = hgL;
                        };
                        auto step = [&](auto b_c) __attribute__((always_inline)) {
                            constexpr int b = decltype(b_c)::value;
                            if constexpr (W2) {
                                step_lin2(b_c);
                            } else if constexpr (LIN) {
                                step_lin(b_c);
                            } else {
                                const int t = L0 + sbyte<b>(P[j >> 2]);
                                // rotate the I/O registers down one lane; lane 63 takes last step's
                                // (hgL, ehL) = row k - 64 of the next strip's lane 0
                                const int ioh = __builtin_amdgcn_update_dpp(L0, IOH, DPP_WAVE_SHL1, 0xF, 0xF, false);
                                const int ioe = __builtin_amdgcn_update_dpp(ehP, IOE, DPP_WAVE_SHL1, 0xF, 0xF, false);
                                const int F = max3i(fh, hgO, 0);
                                const int hgL = dpp_add_shr1_tied(IOH, H, neggo, F);     // H -> hgO -> F -> DPP
                                const int ehL = dpp_add_shr1_tied(IOE, E, negge, hgO);   // E -> H -> hgO -> DPP
                                IOH = ioh;
                                IOE = ioe;
                                E = max3i(ehL, hgL, 0);
                                fh = F - ge;
                                H = vmax3(t, E, F);
                                hgO = H - go;
                                M = max(M, t);
                                L0 = hgL;
                                ehP = ehL;
                            }
                        };
                        step(std::integral_constant<int, 0>{});
                        step(std::integral_constant<int, 1>{});
                        step(std::integral_constant<int, 2>{});
                        step(std::integral_constant<int, 3>{});
                    }
                }
                publish(nloc * C);
            };
            dispatch_kinds<PWG ? KINDS_LDS : SLAB ? KINDS_PEER : KINDS_GRANULE>(in_kind, out_kind, flow_loop);
            if (kp.trace != nullptr && lane == 0) {
                unsigned long long* t = kp.trace + 16ull * (unsigned)strip;
                t[0] = (unsigned long long)t_start;
                t[1] = (unsigned long long)t_first;
                t[3] = (unsigned long long)nslow;
                t[13] = (unsigned long long)(long long)fail_in;
                t[14] = (unsigned long long)(long long)fail_bp;
                t[2] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
                t[7] = (unsigned long long)nloc;
                for (int q = 0; q < 5; ++q) t[8 + q] = (unsigned long long)tl[q];
            }
            if (failed && lane == 0) {
                atomicOr(&kp.ctrl->error, ERR_TIMEOUT);
                atomicMax(&kp.ctrl->err_item, (unsigned)strip);
            }
    #pragma unroll
            for (int off = 32; off > 0; off >>= 1) M = max(M, __shfl_xor(M, off));
            if (lane == 0 && M > 0) atomicMax(&kp.scores[pd.out_idx], M);
        }
    }
}

// Dynamic LDS of a launch (*lim: the most it may be).  At least half the CU's LDS
// for the staged kernel: one workgroup per CU, so no strip ever shares a SIMD with
// another (a co-resident waiting workgroup's polls steal issue slots from a strip
// on the critical path); STREAM stages nothing, the rest is padding that admits
// cfg.f2_wgs workgroups per CU (LDS just above 1/(wgs+1) of the CU's).
template <int C, bool STREAM>
int flow2_dyn_lds(const LaunchCfg& cfg, int* lim) {
    const int wgs = STREAM ? std::max(1, std::min(cfg.f2_wgs, F2_WGS_MAX)) : 1;
    const int pad = LDS_PER_CU / (wgs + 1) + 1024 - flow2_static_lds(C, f2_loader<STREAM>() ? 5 : 4);
    static_assert(F2_CR == 256, "flow2_stream_dyn_max assumes 256-row code rings");
    *lim = STREAM ? flow2_stream_dyn_max(C) : flow2_stage_max(C);
    if (STREAM && cfg.f2_pwg)   // the round buffer
        return std::max(pad, flow2_pwg_row_bytes(cfg.f2_lin) * flow2_pwg_rows(cfg.max_m, C));
    return STREAM ? pad : std::max(flow2_stage_bytes(cfg.max_m, C), pad);
}

template <int C, bool STREAM, bool RING = false, bool SLAB = false, bool LIN = false, bool W2 = false,
          bool PWG = false>
hipError_t prepare_c(const LaunchCfg& cfg, int* dyn) {
    int lim = 0;
    *dyn = flow2_dyn_lds<C, STREAM>(cfg, &lim);
    if (*dyn > lim) return hipErrorInvalidValue;
    if (*dyn > 64 * 1024)   // raise the dynamic-LDS limit (once per variant and device)
        return raise_dyn_lds((const void*)sw_flow2_kernel<C, STREAM, RING, SLAB, LIN, W2, PWG>, lim);
    return hipSuccess;
}

template <int C, bool STREAM, bool RING = false, bool SLAB = false, bool LIN = false, bool W2 = false,
          bool PWG = false>
hipError_t launch_c(const LaunchCfg& cfg, const KParams& kp, hipStream_t s) {
    int dyn = 0;
    const hipError_t e = prepare_c<C, STREAM, RING, SLAB, LIN, W2, PWG>(cfg, &dyn);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((sw_flow2_kernel<C, STREAM, RING, SLAB, LIN, W2, PWG>), dim3(cfg.blocks),
                       dim3(f2_threads<STREAM>()), (size_t)dyn, s, kp);
    return hipGetLastError();
}

// Workgroups per CU the runtime will keep resident for the streamed instantiation a
// launch of cfg would run (its registers, waves and the LDS of cfg.f2_wgs): what
// ring mode's static deal must not exceed (every block resident).  -1 on error.
template <int C, bool RING, bool SLAB, bool LIN, bool W2>
int resident_c(const LaunchCfg& cfg) {
    int dyn = 0, nb = 0;
    if (prepare_c<C, true, RING, SLAB, LIN, W2>(cfg, &dyn) != hipSuccess) return -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)sw_flow2_kernel<C, true, RING, SLAB, LIN, W2>,
                                                     f2_threads<true>(), (size_t)dyn) != hipSuccess)
        return -1;
    return nb;
}
template <int C, bool LIN, bool W2 = false>
int resident_v(const LaunchCfg& cfg, bool ring, bool slab) {
    if (slab) return ring ? resident_c<C, true, true, LIN, W2>(cfg) : resident_c<C, false, true, LIN, W2>(cfg);
    return ring ? resident_c<C, true, false, LIN, W2>(cfg) : resident_c<C, false, false, LIN, W2>(cfg);
}

// the instantiation a launch needs: ring edges, slab edges, streamed or staged codes
template <int C, bool LIN, bool W2 = false>
hipError_t launch_v(const LaunchCfg& cfg, const KParams& kp, hipStream_t s) {
    const bool ring = kp.ring_rows > 0, slab = kp.slab_in != nullptr || kp.slab_out != nullptr;
    if (slab)
        return ring ? launch_c<C, true, true, true, LIN, W2>(cfg, kp, s) : launch_c<C, true, false, true, LIN, W2>(cfg, kp, s);
    if (ring) return launch_c<C, true, true, false, LIN, W2>(cfg, kp, s);
    return cfg.f2_stream ? launch_c<C, true, false, false, LIN, W2>(cfg, kp, s)
                         : launch_c<C, false, false, false, LIN, W2>(cfg, kp, s);
}

template <int C>
int waves_c() {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)sw_flow2_kernel<C, false, false, false, false>,
                                                     f2_threads<false>(), 0) != hipSuccess)
        return 4;
    return nb * 4;
}

}  // namespace

bool flow2_variant_exists(int C) { return C == 16 || C == 32 || C == 64; }

hipError_t launch_sw_flow2(const LaunchCfg& cfg, const KParams& kp, hipStream_t stream) {
    // a pair per workgroup (batches needing int32 scores): 64-row chunks, throughput-bound,
    // the two-column linear-gap step or the one-column affine step
    if (cfg.f2_pwg) {
        if (cfg.C != 64) return hipErrorInvalidValue;
        return cfg.f2_w2 && cfg.f2_lin ? launch_c<64, true, false, false, true, true, true>(cfg, kp, stream)
               : !cfg.f2_w2 && !cfg.f2_lin ? launch_c<64, true, false, false, false, false, true>(cfg, kp, stream)
                                           : hipErrorInvalidValue;
    }
    switch (cfg.C) {
        // the linear-gap step (G_INIT == G_EXT) is built for 32-row (latency-bound pairs) and
        // 64-row chunks (ring mode, throughput-bound)
        case 16: return launch_v<16, false>(cfg, kp, stream);
        // two columns per lane (cfg.f2_w2) with the linear-gap step only
        case 32:
            return cfg.f2_w2 && cfg.f2_lin ? launch_v<32, true, true>(cfg, kp, stream)
                   : cfg.f2_lin            ? launch_v<32, true>(cfg, kp, stream)
                                           : launch_v<32, false>(cfg, kp, stream);
        case 64:
            return cfg.f2_w2 && cfg.f2_lin ? launch_v<64, true, true>(cfg, kp, stream)
                   : cfg.f2_lin            ? launch_v<64, true>(cfg, kp, stream)
                                           : launch_v<64, false>(cfg, kp, stream);
        default: return hipErrorInvalidValue;
    }
}

int flow2_stream_resident(const LaunchCfg& cfg, bool ring, bool slab) {
    switch (cfg.C) {
        case 16: return resident_v<16, false>(cfg, ring, slab);
        case 32:
            return cfg.f2_w2 && cfg.f2_lin ? resident_v<32, true, true>(cfg, ring, slab)
                   : cfg.f2_lin            ? resident_v<32, true>(cfg, ring, slab)
                                           : resident_v<32, false>(cfg, ring, slab);
        case 64:
            return cfg.f2_w2 && cfg.f2_lin ? resident_v<64, true, true>(cfg, ring, slab)
                   : cfg.f2_lin            ? resident_v<64, true>(cfg, ring, slab)
                                           : resident_v<64, false>(cfg, ring, slab);
        default: return -1;
    }
}

int flow2_waves_per_cu(int C) {
    switch (C) {
        case 16: return waves_c<16>();
        case 32: return waves_c<32>();
        case 64: return waves_c<64>();
        default: return 4;
    }
}

}  // namespace swmi
