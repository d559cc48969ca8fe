// sw_internal.h -- structures shared by the gfx950 kernels (sw_kernels.hip) and
// the C++ host layer (sw_engine.hip).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swmi {

// One pair after orientation: the "column" sequence (length n) runs across the
// lanes of a wave, the "row" sequence (length m) streams through it.  The score
// is symmetric in (seq1, seq2), so the host picks the orientation.
struct PairDesc {
    uint64_t col_off;   // byte offset of the column sequence in the sequence arena
    uint64_t row_off;   // byte offset of the row sequence
    uint64_t bnd_off;   // granule offset of this pair's strip-boundary buffers
    int n;              // columns (> 0)
    int m;              // rows    (> 0)
    int strips;         // ceil(n / (64*W))
    int out_idx;        // slot in the score array
};

// Two pairs scored in lock step by the packed-u16 "duo" kernel: lane values
// hold pair 0 in the low and pair 1 in the high 16 bits.  Both are padded to
// (n_pad, m_pad) with dead columns / sentinel rows.
struct DuoDesc {
    uint64_t col_off[2];
    uint64_t row_off[2];
    uint64_t bnd_off;   // granule offset of the duo's strip-boundary buffers (m_pad rows each)
    int n[2], m[2];
    int n_pad, m_pad;
    int strips;         // ceil(n_pad / (64*W))
    int out_idx[2];     // out_idx[1] == -1: no second pair
};

// Per-launch control block (zeroed by hipMemsetAsync before every launch).
struct Ctrl {
    unsigned int next_item;   // work-claim counter (items claimed strictly in order)
    unsigned int error;       // nonzero: a bounded spin gave up (see ERR_*)
    unsigned int err_item;
    unsigned int pad;
};

enum : unsigned { ERR_TIMEOUT = 1u };

// A strip boundary hand-off granule: written ONCE per launch with a single
// 16-byte write-through (sc1) store by the producer wave, read with sc1 loads
// by the consumer wave.  `tag` carries the launch epoch, `chk` detects a torn
// or stale read.  (MI355X_MICROARCH.md, Workgroup dispatch ... R2 granules.)
struct alignas(16) Granule {
    unsigned int tag;
    int hg;      // H - G_INIT of the strip's last column at this row
    int eh;      // E - G_EXT  of the strip's last column at this row
    unsigned int chk;
};

// Torn-read guard of a 16-B granule {tag, hg, eh, chk}: injective in each of
// tag, hg and eh for fixed others, so a granule mixing dwords of two writes
// (different epoch, or a stale value) fails the check.  Multiply-free: XORs
// and one rotate (v_xor3 / v_alignbit), on the consumer's critical path.
__host__ __device__ inline unsigned granule_chk(unsigned tag, int hg, int eh, int row) {
    const unsigned e = (unsigned)eh;
    return tag ^ (unsigned)hg ^ ((e << 13) | (e >> 19)) ^ ((unsigned)row << 7) ^ 0x5BD1E995u;
}

struct KParams {
    const unsigned char* seq;     // sequence arena (raw bytes)
    const PairDesc* pairs;
    const int* item_base;         // npairs+1 prefix sums of strips
    Granule* bnd;                 // strip-boundary granule arena
    Ctrl* ctrl;
    int* scores;
    int npairs;
    int total_items;
    unsigned epoch;               // != 0, unique per launch
    int match, mismatch, gap_init, gap_ext;
    unsigned prof[4];             // DNA mode: per column code, 4 biased score bytes (row code 0..3)
    unsigned prof2[4];            // flow2 mode: per column code, 4 signed score bytes s + G_INIT (row code 0..3)
    unsigned prof3[4];            // flow2 W2: per column code, 4 signed score bytes s (row code 0..3)
    unsigned pen[4];              // duo mode: per column code, 4 penalty bytes MATCH - s (row code 0..3)
    // a pair over an alphabet of up to seven byte values (flow3 staged, LaunchCfg::hep): the symbol
    // 0..6 of each byte value, and per column symbol the perm's high word (row symbols 0..3) and low
    // word (byte 0: the no-row 0x80; bytes 1..3: row symbols 4..6), as signed bytes s + G_INIT (hp2,
    // hq2) and s (hp3, hq3)
    unsigned char hsym[256];
    unsigned hp2[7], hq2[7], hp3[7], hq3[7];
    const unsigned char* hrows;   // ring mode (sw_flow3r3h / ra3h_kernel): the pair's rows as perm selectors
    const DuoDesc* duos;          // duo mode: nduos descriptors (npairs counts duos)
    long long timeout_ticks;      // s_memrealtime ticks (100 MHz) before a spin gives up
    unsigned long long* trace;    // optional (tools/trace_flow.py): per-strip timestamps, else null
    // Column slab of a pair split across GPUs (grouped modes, one pair per launch):
    // the first group's inflow comes from slab_in (the previous slab's last
    // column, written by the previous GPU over xGMI), the last group's outflow
    // goes to slab_out (the next GPU's slab_in, mapped here by IPC).  Both use
    // slab_epoch, agreed by all ranks; null = an ordinary pair edge.
    Granule* slab_in;
    Granule* slab_out;
    unsigned slab_epoch;
    // flow2 ring mode (one pair; sw_flow2.hip): 0 = linear edges (one m-row
    // granule buffer per group boundary, written once).  Else block j of the
    // G-block grid runs groups j, j+G, j+2G, ...; boundary k*G+j streams through
    // ring j (ring_rows rows, j < G-1) or the wrap ring (wrap_rows >= m rows,
    // j = G-1), so the boundary state is O(G*ring_rows + m), not O(groups*m).
    int ring_rows;
    int wrap_rows;
    unsigned* ring_cons;          // ring j's consumer progress (positions consumed), RING_CONS_STRIDE apart;
                                  // duo LDS kernel: DUO_CU_WORDS zeroed role words (or null)
    int duo_prio;                 // duo LDS kernel with roles: 0 = off, k in 6..20 = the CU's two workgroups
                                  // take turns at issue priority every 2^k ticks of s_memrealtime (s_setprio)
    int w45_s4;                   // flow3 ring at four / five columns per lane (sw_flow3r45_kernel): strips below
                                  // this index have 252 new columns, the rest 315 (a multiple of 4); -1 otherwise
    int stall_item;               // tests only (option stall_item): flow2's compute waves skip this item, so its
                                  // edges are never published and its consumers' bounded waits must expire; -1 = none
    // (the duo kernel with LDS hand-offs takes its wrap-buffer slots from wrap_rows)
};

constexpr int RING_CONS_STRIDE = 32;   // dwords between consumer progress words (one 128-B line each)

// Grid organisations (sw_kernels.hip):
//   MODE_STRIP  independent waves claim (pair, strip) items in order
//   MODE_PAIRWG one workgroup per pair, its 4 waves interleave the strips
//   MODE_CHAIN  one workgroup per group of 4 consecutive strips, LDS hand-offs
//   MODE_DUO    one workgroup per two pairs, packed u16 (DNA, small scores)
//   MODE_FLOW   as MODE_CHAIN, free-running waves with LDS progress words
//   MODE_FLOW2  W=1 DNA single pairs: overlapping 64-column strips, DPP-add
//               hand-offs, 11 instructions per step (sw_flow2.hip)
enum : int { MODE_STRIP = 0, MODE_PAIRWG = 1, MODE_CHAIN = 2, MODE_DUO = 3, MODE_FLOW = 4, MODE_FLOW2 = 5 };
inline bool grouped_mode(int mode) { return mode == MODE_CHAIN || mode == MODE_FLOW || mode == MODE_FLOW2; }

#ifndef SW_DUO_WAVES
#define SW_DUO_WAVES 4
#endif
constexpr int DUO_WAVES = SW_DUO_WAVES;   // waves per workgroup of the duo kernel (one workgroup per duo)

// Host-side launch (sw_kernels.hip).
struct LaunchCfg {
    int W;          // columns per lane
    int C;          // rows per hand-off chunk
    bool dna;       // 2-bit ACGT profile path (else raw-byte compare)
    int blocks;     // persistent workgroups (256 threads = 4 waves)
    int mode;       // MODE_*
    int max_m;      // longest row sequence (MODE_FLOW stages it in LDS)
    bool duo_f16 = false;   // MODE_DUO: max3 through v_pk_maximum3_f16 (every value < 0x7C00)
    bool f2_stream = false; // MODE_FLOW2: row codes streamed through per-wave LDS rings (rows too long to stage)
    int f2_wgs = 1;         // MODE_FLOW2 streamed: workgroups per CU (LDS pad sized to admit exactly this many)
    bool f2_lin = false;    // G_INIT == G_EXT, the exact linear-gap step: MODE_FLOW2 at C = 32 or 64 (sw_flow2.hip
                            // LIN) and MODE_DUO with duo_f16 (sw_kernels.hip StripDuo LIN)
    bool f2_w2 = false;     // MODE_FLOW2 with f2_lin: two columns per lane (126 new columns per strip)
    bool f2_pwg = false;    // MODE_FLOW2 batch: a pair per workgroup, all hand-offs in LDS (C = 64, streamed)
    bool f3 = false;        // MODE_FLOW2 staged two-column linear-gap launch on the flow3 kernel (sw_flow3.hip)
    bool f3_hl = false;     // flow3 staged at C = 32: in-workgroup links hand off every half chunk
    bool f3a = false;       // MODE_FLOW2 staged one-column launch with the affine step on flow3 (sw_flow3a_kernel)
    bool f3p = false;       // flow3 staged on the pool loops (sw_flow3p_kernel: C = 32, f3_hl, no I/O rotation)
    bool hep = false;       // flow3 staged launch of a pair over up to seven byte values (sw_flow3h / ah_kernel, KParams::hsym)
    bool f3_w3 = false;     // flow3 ring mode at three columns per lane (sw_flow3r3_kernel / sw_flow3r3s_kernel)
    bool f3_w45 = false;    // flow3 ring mode at four and five columns per lane (sw_flow3r45_kernel, KParams::w45_s4)
    bool f3_pwg = false;    // flow3 three-column ring step, a pair per workgroup (sw_flow3r3p_kernel; int32 batches)
    bool f3ra = false;      // MODE_FLOW2 ring-mode two-column launch with the affine step on flow3 (sw_flow3ra_kernel)
    bool f3_slab = false;   // flow3 ring launch of a column slab (sw_flow3rs_kernel / sw_flow3ras_kernel)
    int duo_wrap = 0;       // MODE_DUO at C = 64: > 0 = strip hand-offs in LDS (sw_duo_lds_kernel), this many
                            // wrap-buffer slots (a power of two >= every m_pad); 0 = HBM granules
    int duo_tab = 0;        // with duo_wrap, W % 4 == 0: > 0 = row codes from an LDS table of this many words
};
// the duo LDS kernel's wrap buffer: slots for rows of m_pad up to m, and its dynamic LDS
inline int duo_wrap_slots(int m) {
    int w = 64;
    while (w < m) w *= 2;
    return w;
}
// the duo LDS kernel's row-code table (sw_kernels.hip StripDuoT): rows -DUO_TAB_OFF .. m_pad + DUO_TAB_TAIL
constexpr int DUO_TAB_OFF = 528;     // rows below row 0: lane 63's W = 8 positions and a read group ahead
constexpr int DUO_TAB_TAIL = 768;    // rows past m_pad: the last chunk's steps, the build's two chunks ahead
// the duo LDS kernel's dynamic LDS: the wrap buffer, then the code table (words, 16-B rounded)
inline int duo_lds_dyn(const LaunchCfg& cfg) {
    return cfg.duo_wrap * (cfg.f2_lin ? 4 : 8) + ((cfg.duo_tab * 4 + 15) & ~15);
}
constexpr int DUO_LDS_DYN_MAX = 72 * 1024;   // attribute limit of the duo LDS kernel's dynamic LDS
constexpr int DUO_CU_WORDS = 8 * 256;         // duo strip roles: a word per (XCC, SE, SH, CU) of HW_ID
// the most dynamic LDS that still admits two workgroups per CU beside the static LDS (rings, sinks:
// ~5 KB at the linear-gap step's 4-B slots, ~9 KB affine)
inline int duo_lds_fit(bool lin) { return lin ? 72 * 1024 : 68 * 1024; }
constexpr int F2_WGS_MAX = 4;   // flow2 streamed kernel: most workgroups per CU (launch_c sizes the LDS pad)

// MODE_FLOW stages a pair's row codes in LDS: one byte per row plus the
// prefetch tail; pairs whose rows do not fit use MODE_CHAIN.
constexpr int LDS_PER_CU = 160 * 1024;
__host__ __device__ constexpr int flow_stage_rows(int m, int W, int C) { return ((m + 64 * W + 2 * C + 64) + 15) & ~15; }
__host__ __device__ constexpr int flow_ring_rows(int W, int C) {
    int r = 256;
    while (r < 2 * 64 * W + 4 * C) r *= 2;
    return r;
}
// static LDS of sw_flow_kernel<W,C> (rings + sinks + words), rounded up
__host__ __device__ constexpr int flow_static_lds(int W, int C) { return 3 * flow_ring_rows(W, C) * 8 + 4096; }
__host__ __device__ constexpr int flow_stage_max(int W, int C) { return LDS_PER_CU - flow_static_lds(W, C); }

// MODE_FLOW2 (sw_flow2.hip): strip s covers columns [63s, 63s + 64); the row
// codes of the pair are staged in LDS (one byte per row, 64 rows of border in
// front, a chunk of prefetch behind).
__host__ __device__ constexpr int flow2_strips(int n) { return n <= 64 ? 1 : (n - 1 + 62) / 63; }
// two columns per lane (LaunchCfg::f2_w2): strip s covers columns [126s, 126s + 128)
__host__ __device__ constexpr int flow2_strips_w2(int n) { return n <= 128 ? 1 : (n - 2 + 125) / 126; }
// three columns per lane (flow3 ring mode): strips of 189 new columns overlapping by three
__host__ __device__ constexpr int flow2_strips_w3(int n) { return n <= 192 ? 1 : (n - 3 + 188) / 189; }
__host__ __device__ constexpr int flow2_stage_bytes(int m, int C) {
    return (64 + ((m + 64 + C - 1) / C + 1) * C + 8 + 15) & ~15;
}
// (rings: 4, or 5 with the staged kernel's loader wave, whose static LDS bounds the staged rows)
__host__ __device__ constexpr int flow2_static_lds(int C, int rings = 5) { return rings * (256 * 8 + 64 * 8 + 64 * 4) + 64 + 0 * C; }
__host__ __device__ constexpr int flow2_stage_max(int C) { return LDS_PER_CU - flow2_static_lds(C) - 256; }
// the most dynamic LDS a streamed flow2 launch may take (sw_flow2.hip flow2_dyn_lds): the staged
// limit less the 4 per-wave code rings (F2_CR = 256 rows + a chunk + 64 sinks each)
__host__ __device__ constexpr int flow2_stream_dyn_max(int C) { return flow2_stage_max(C) - 4 * (256 + C + 64); }
// flow2 pair per workgroup (LaunchCfg::f2_pwg): the wave 3 -> wave 0 buffer holds a round's
// rows (int2 each) in the dynamic LDS; workgroups per CU that fit beside the static LDS
// (4 rings) and the 4 streamed code rings
// (4 B per row at the linear-gap step, whose edges carry H - G twice)
__host__ __device__ constexpr int flow2_pwg_rows(int m, int C) { return (m + 64 + C - 1) / C * C; }
__host__ __device__ constexpr int flow2_pwg_row_bytes(bool lin) { return lin ? 4 : 8; }
__host__ __device__ constexpr int flow2_pwg_wgs(int m, int C, bool lin) {
    return LDS_PER_CU /
           (flow2_pwg_row_bytes(lin) * flow2_pwg_rows(m, C) + flow2_static_lds(C, 4) + 4 * (256 + C + 64) + 1024);
}
// sets the calling thread's sw_last_error() text (sw_engine.hip)
void report_error(const char* msg);
// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) once per (kernel, device) (sw_engine.hip)
hipError_t raise_dyn_lds(const void* fn, int bytes);

hipError_t launch_sw_flow2(const LaunchCfg& cfg, const KParams& kp, hipStream_t stream);
// flow3 (sw_flow3.hip): flow2's staged W2 linear-gap kernel with hand-scheduled chunk loops
hipError_t launch_sw_flow3(const LaunchCfg& cfg, const KParams& kp, hipStream_t stream);
bool flow3_fits(int max_m, int C, bool aff = false);
// workgroups per CU resident for a flow3 ring-mode launch (its LDS pad of cfg.f2_wgs), -1 on error
int flow3_ring_resident(const LaunchCfg& cfg);
int flow2_waves_per_cu(int C);
// workgroups per CU resident for the streamed flow2 kernel cfg selects (ring / slab
// instantiation, LDS pad of cfg.f2_wgs); -1 on error (sw_flow2.hip)
int flow2_stream_resident(const LaunchCfg& cfg, bool ring, bool slab);
bool flow2_variant_exists(int C);

hipError_t launch_sw_strip(const LaunchCfg& cfg, const KParams& kp, hipStream_t stream);
int kernel_waves_per_cu(const LaunchCfg& cfg);     // residency of the chosen variant
bool variant_exists(int W, int C);

}  // namespace swmi
