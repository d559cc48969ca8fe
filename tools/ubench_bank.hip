// ubench_bank.hip -- gfx950 VALU issue cost vs VGPR bank placement of the source
// operands (tools only).  Each probe issues 8 independent instructions per
// iteration on fixed physical registers (inline asm with clobbers), so the bank
// of every source (register number mod 4) is chosen here, not by the compiler:
//   "spread": the sources of each instruction sit in different banks
//   "same":   every source of an instruction sits in one bank
// Prints cycles per instruction per SIMD at 1, 2, 4 and 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_bank.hip -o build/ubench_bank
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define ITERS 16384

// v20..v27: destinations (banks 0..3 twice); sources from v28..v43
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", \
             "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43"

#define INIT                                                                                                   \
    asm volatile(                                                                                              \
        "v_mov_b32 v28, 1\n v_mov_b32 v29, 2\n v_mov_b32 v30, 3\n v_mov_b32 v31, 4\n v_mov_b32 v32, 5\n"        \
        "v_mov_b32 v33, 6\n v_mov_b32 v34, 7\n v_mov_b32 v35, 8\n v_mov_b32 v36, 9\n v_mov_b32 v37, 10\n"      \
        "v_mov_b32 v38, 11\n v_mov_b32 v39, 12\n v_mov_b32 v40, 13\n v_mov_b32 v41, 14\n v_mov_b32 v42, 15\n"  \
        "v_mov_b32 v43, 16\n" ::: CLOB);

// 3-source ops: spread = (b1, b2, b3) distinct banks; same = all bank 0 (v28, v32, v36 / v40, ...)
#define OP3_SPREAD(op)                                                                                         \
    op " v20, v29, v30, v31\n" op " v21, v33, v34, v35\n" op " v22, v37, v38, v39\n" op " v23, v41, v42, v43\n" \
    op " v24, v29, v30, v31\n" op " v25, v33, v34, v35\n" op " v26, v37, v38, v39\n" op " v27, v41, v42, v43\n"
#define OP3_SAME(op)                                                                                           \
    op " v20, v28, v32, v36\n" op " v21, v29, v33, v37\n" op " v22, v30, v34, v38\n" op " v23, v31, v35, v39\n" \
    op " v24, v32, v36, v40\n" op " v25, v33, v37, v41\n" op " v26, v34, v38, v42\n" op " v27, v35, v39, v43\n"
#define OP3_TWO(op)                                                                                            \
    op " v20, v28, v32, v29\n" op " v21, v29, v33, v30\n" op " v22, v30, v34, v31\n" op " v23, v31, v35, v28\n" \
    op " v24, v32, v36, v29\n" op " v25, v33, v37, v30\n" op " v26, v34, v38, v31\n" op " v27, v35, v39, v28\n"
#define OP2_SPREAD(op)                                                                                         \
    op " v20, v29, v30\n" op " v21, v33, v34\n" op " v22, v37, v38\n" op " v23, v41, v42\n"                     \
    op " v24, v31, v28\n" op " v25, v35, v32\n" op " v26, v39, v36\n" op " v27, v43, v40\n"
#define OP2_SAME(op)                                                                                           \
    op " v20, v28, v32\n" op " v21, v29, v33\n" op " v22, v30, v34\n" op " v23, v31, v35\n"                     \
    op " v24, v32, v36\n" op " v25, v33, v37\n" op " v26, v34, v38\n" op " v27, v35, v39\n"

// SDWA byte operand, DPP (wave_shr:1 / wave_shl:1), VOP1 moves, clamped subtract
#define SD(d, a, b) " v" #d ", v" #a ", sext(v" #b ") dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define OP2_SDWA(op) op SD(20, 29, 30) op SD(21, 33, 34) op SD(22, 37, 38) op SD(23, 41, 42) op SD(24, 31, 28) \
    op SD(25, 35, 32) op SD(26, 39, 36) op SD(27, 43, 40)
#define DP(d, a, b) " v" #d ", v" #a ", v" #b " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define OP2_DPP(op) op DP(20, 29, 30) op DP(21, 33, 34) op DP(22, 37, 38) op DP(23, 41, 42) op DP(24, 31, 28) \
    op DP(25, 35, 32) op DP(26, 39, 36) op DP(27, 43, 40)
#define D1(d, a) " v" #d ", v" #a " wave_shl:1 row_mask:0xf bank_mask:0xf\n"
#define OP1_DPP(op) op D1(20, 29) op D1(21, 33) op D1(22, 37) op D1(23, 41) op D1(24, 31) op D1(25, 35) op D1(26, 39) op D1(27, 43)
#define M1(d, a) " v" #d ", v" #a "\n"
#define OP1(op) op M1(20, 29) op M1(21, 33) op M1(22, 37) op M1(23, 41) op M1(24, 31) op M1(25, 35) op M1(26, 39) op M1(27, 43)
#define CL(d, a, b) " v" #d ", v" #a ", v" #b " clamp\n"
#define OP2_CLAMP(op) op CL(20, 29, 30) op CL(21, 33, 34) op CL(22, 37, 38) op CL(23, 41, 42) op CL(24, 31, 28) \
    op CL(25, 35, 32) op CL(26, 39, 36) op CL(27, 43, 40)

#define NOPS(op) op " v20, v29, v30, v31\n s_nop 0\n" op " v21, v33, v34, v35\n s_nop 0\n" op " v22, v37, v38, v39\n s_nop 0\n" \
    op " v23, v41, v42, v43\n s_nop 0\n" op " v24, v29, v30, v31\n s_nop 0\n" op " v25, v33, v34, v35\n s_nop 0\n" \
    op " v26, v37, v38, v39\n s_nop 0\n" op " v27, v41, v42, v43\n s_nop 0\n"
#define SALUS(op) op " v20, v29, v30, v31\n s_add_u32 s40, s40, 1\n" op " v21, v33, v34, v35\n s_add_u32 s41, s41, 1\n" \
    op " v22, v37, v38, v39\n s_add_u32 s40, s40, 1\n" op " v23, v41, v42, v43\n s_add_u32 s41, s41, 1\n" \
    op " v24, v29, v30, v31\n s_add_u32 s40, s40, 1\n" op " v25, v33, v34, v35\n s_add_u32 s41, s41, 1\n" \
    op " v26, v37, v38, v39\n s_add_u32 s40, s40, 1\n" op " v27, v41, v42, v43\n s_add_u32 s41, s41, 1\n"
// every instruction reads the previous one's result (latency of a dependent chain)
#define CHAIN(op) op " v20, v27, v30, v31\n" op " v21, v20, v34, v35\n" op " v22, v21, v38, v39\n" op " v23, v22, v42, v43\n" \
    op " v24, v23, v30, v31\n" op " v25, v24, v34, v35\n" op " v26, v25, v38, v39\n" op " v27, v26, v42, v43\n"
// two interleaved dependent chains
#define CHAIN2(op) op " v20, v26, v30, v31\n" op " v21, v27, v34, v35\n" op " v22, v20, v38, v39\n" op " v23, v21, v42, v43\n" \
    op " v24, v22, v30, v31\n" op " v25, v23, v34, v35\n" op " v26, v24, v38, v39\n" op " v27, v25, v42, v43\n"

// producer writing v20 / v21 / v22 / v23 (one per pair), consumer max3 reading it
#define DPPW(d) "v_add_u32_dpp v" #d ", v29, v30 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define SDWAW(d) "v_add_u32_sdwa v" #d ", v29, sext(v30) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define MAXW(d) "v_max3_i32 v" #d ", v29, v30, v31\n"
#define USE(d) "v_max3_i32 v24, v" #d ", v33, v34\n"
#define FILL "v_max3_i32 v25, v37, v38, v39\n"
#define DIST1(W) W(20) USE(20) W(21) USE(21) W(22) USE(22) W(23) USE(23)
#define DIST2(W) W(20) FILL USE(20) W(21) FILL USE(21) W(22) FILL USE(22) W(23) FILL USE(23)
#define DIST3(W) W(20) FILL FILL USE(20) W(21) FILL FILL USE(21) W(22) FILL FILL USE(22) W(23) FILL FILL USE(23)

template <int KIND>
__global__ void bank(int* out, unsigned long long* cyc) {
    INIT
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (KIND == 0) asm volatile(OP3_SPREAD("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 1) asm volatile(OP3_SAME("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 2) asm volatile(OP3_TWO("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 3) asm volatile(OP3_SPREAD("v_pk_maximum3_f16") ::: CLOB);
        if constexpr (KIND == 4) asm volatile(OP3_SAME("v_pk_maximum3_f16") ::: CLOB);
        if constexpr (KIND == 5) asm volatile(OP3_TWO("v_pk_maximum3_f16") ::: CLOB);
        if constexpr (KIND == 6) asm volatile(OP3_SPREAD("v_perm_b32") ::: CLOB);
        if constexpr (KIND == 7) asm volatile(OP3_SAME("v_perm_b32") ::: CLOB);
        if constexpr (KIND == 8) asm volatile(OP2_SPREAD("v_pk_sub_u16") ::: CLOB);
        if constexpr (KIND == 9) asm volatile(OP2_SAME("v_pk_sub_u16") ::: CLOB);
        if constexpr (KIND == 10) asm volatile(OP2_SPREAD("v_add_u32") ::: CLOB);
        if constexpr (KIND == 11) asm volatile(OP2_SAME("v_add_u32") ::: CLOB);
        if constexpr (KIND == 12) asm volatile(OP2_SPREAD("v_pk_add_u16") ::: CLOB);
        if constexpr (KIND == 13) asm volatile(OP2_SAME("v_pk_add_u16") ::: CLOB);
        if constexpr (KIND == 14) asm volatile(OP2_SPREAD("v_sub_u32_e64") ::: CLOB);
        if constexpr (KIND == 15) asm volatile(OP2_SAME("v_sub_u32_e64") ::: CLOB);
        if constexpr (KIND == 16) asm volatile(OP3_SPREAD("v_add3_u32") ::: CLOB);
        if constexpr (KIND == 17) asm volatile(OP3_SAME("v_add3_u32") ::: CLOB);
        if constexpr (KIND == 18) asm volatile(OP3_SPREAD("v_fma_f32") ::: CLOB);
        if constexpr (KIND == 19) asm volatile(OP2_SPREAD("v_max_i32") ::: CLOB);
        if constexpr (KIND == 20) asm volatile(OP2_SDWA("v_add_u32_sdwa") ::: CLOB);
        if constexpr (KIND == 21) asm volatile(OP2_DPP("v_add_u32_dpp") ::: CLOB);
        if constexpr (KIND == 22) asm volatile(OP1_DPP("v_mov_b32_dpp") ::: CLOB);
        if constexpr (KIND == 23) asm volatile(OP1("v_mov_b32") ::: CLOB);
        if constexpr (KIND == 24) asm volatile(OP2_CLAMP("v_sub_u32_e64") ::: CLOB);
        if constexpr (KIND == 25) asm volatile("v_pk_add_f32 v[20:21], v[28:29], v[30:31]\n v_pk_add_f32 v[22:23], v[32:33], v[34:35]\n v_pk_add_f32 v[24:25], v[36:37], v[38:39]\n v_pk_add_f32 v[26:27], v[40:41], v[42:43]\n" "v_pk_add_f32 v[20:21], v[30:31], v[28:29]\n v_pk_add_f32 v[22:23], v[34:35], v[32:33]\n v_pk_add_f32 v[24:25], v[38:39], v[36:37]\n v_pk_add_f32 v[26:27], v[42:43], v[40:41]\n" ::: CLOB);
        if constexpr (KIND == 26) asm volatile(OP2_SPREAD("v_add_f32") ::: CLOB);
        if constexpr (KIND == 27) asm volatile(OP2_SPREAD("v_max_u16") ::: CLOB);
        if constexpr (KIND == 28) asm volatile(OP3_SPREAD("v_max3_u16") ::: CLOB);
        // lone-wave issue: VALU interleaved with s_nop / SALU, dependent chains
        if constexpr (KIND == 29) asm volatile(NOPS("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 30) asm volatile(SALUS("v_max3_i32") ::: CLOB, "s40", "s41", "scc");
        if constexpr (KIND == 31) asm volatile(CHAIN("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 32) asm volatile(CHAIN2("v_max3_i32") ::: CLOB);
        // a DPP / SDWA / VOP3 result read 1, 2 or 3 instructions later (4 pairs of 2..4 instructions)
        if constexpr (KIND == 33) asm volatile(DIST1(DPPW) ::: CLOB);
        if constexpr (KIND == 34) asm volatile(DIST2(DPPW) ::: CLOB);
        if constexpr (KIND == 35) asm volatile(DIST3(DPPW) ::: CLOB);
        if constexpr (KIND == 36) asm volatile(DIST1(SDWAW) ::: CLOB);
        if constexpr (KIND == 37) asm volatile(DIST2(SDWAW) ::: CLOB);
        if constexpr (KIND == 38) asm volatile(DIST1(MAXW) ::: CLOB);
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    int r;
    asm volatile("v_add_u32 %0, v20, v27" : "=v"(r)::CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int KIND>
void run(const char* name, int wps, int per_iter = 8) {
    int* out;
    unsigned long long* cyc;
    const int threads = wps * 256 > 1024 ? 1024 : wps * 256;   // waves per SIMD: 4*wps waves per CU
    const int blocks = 256 * (wps * 256 / threads), waves = blocks * threads / 64;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, waves * 8);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(bank<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(bank<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(waves);
    hipMemcpy(h.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto v : h) avg += v;
    avg /= waves;
    const double per_wave = avg / (ITERS * (double)per_iter);
    // wall-clock cost too: ns per instruction per SIMD from the event time
    const double ns_simd = ms * 1e6 / (ITERS * (double)per_iter * wps);
    printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_simd\": %.2f, \"ns_per_instr_per_simd\": %.3f, "
           "\"ms\": %.3f}\n", name, wps, per_wave / wps, ns_simd, ms);
    fflush(stdout);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int t : {1, 2}) {   // lone-wave issue of VALU + s_nop / SALU, dependent chains
        run<0>("v_max3_i32 (8 independent)", t);
        run<29>("v_max3_i32 + s_nop 0 each", t);
        run<30>("v_max3_i32 + s_add_u32 each", t);
        run<31>("v_max3_i32 one dependent chain", t);
        run<32>("v_max3_i32 two dependent chains", t);
        run<33>("dpp_add -> use at distance 1", t, 8);
        run<34>("dpp_add -> use at distance 2", t, 12);
        run<35>("dpp_add -> use at distance 3", t, 16);
        run<36>("sdwa_add -> use at distance 1", t, 8);
        run<37>("sdwa_add -> use at distance 2", t, 12);
        run<38>("max3 -> use at distance 1", t, 8);
    }
    if (getenv("UB_LONE_ONLY")) return 0;
    for (int t : {1, 2, 4, 8}) {   // waves per SIMD
        run<18>("v_fma_f32", t);
        run<19>("v_max_i32", t);
        run<20>("v_add_u32_sdwa", t);
        run<21>("v_add_u32_dpp", t);
        run<22>("v_mov_b32_dpp", t);
        run<23>("v_mov_b32", t);
        run<24>("v_sub_u32_e64 clamp", t);
        run<25>("v_pk_add_f32", t);
        run<26>("v_add_f32", t);
        run<27>("v_max_u16", t);
        run<28>("v_max3_u16", t);
        run<0>("v_max3_i32 spread", t);
        run<1>("v_max3_i32 same", t);
        run<2>("v_max3_i32 two", t);
        run<3>("v_pk_maximum3_f16 spread", t);
        run<4>("v_pk_maximum3_f16 same", t);
        run<5>("v_pk_maximum3_f16 two", t);
        run<6>("v_perm_b32 spread", t);
        run<7>("v_perm_b32 same", t);
        run<8>("v_pk_sub_u16 spread", t);
        run<9>("v_pk_sub_u16 same", t);
        run<10>("v_add_u32 spread", t);
        run<11>("v_add_u32 same", t);
        run<12>("v_pk_add_u16 spread", t);
        run<13>("v_pk_add_u16 same", t);
        run<14>("v_sub_u32_e64 spread", t);
        run<15>("v_sub_u32_e64 same", t);
        run<16>("v_add3_u32 spread", t);
        run<17>("v_add3_u32 same", t);
    }
    return 0;
}
