// ubench_fclass.hip -- gfx950 VALU issue cost of candidate replacements for the slow-class
// integer max / SDWA / DPP forms of the wavefront steps (tools only), and a correctness check of
// float maxima over non-negative int32 bit patterns.
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_fclass.hip -o build/ubench_fclass
//
// Issue cost: as tools/ubench_bank.hip (8 independent instructions per iteration on fixed
// registers, 1 / 2 / 4 waves per SIMD, ns per instruction per SIMD from the event time).
// Check: v_max_f32 / v_max3_f32 on int32 bit patterns against the integer maximum, for operand
// triples where at least one operand is a non-negative int (the steps' clamped H - G, or 0): the
// IEEE order of positive floats (denormals included, if the mode keeps them) is the integer order
// of their bit patterns, negative ints are negative floats or NaNs, which maxNum drops.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define ITERS 16384
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", \
             "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43"
#define INIT                                                                                                   \
    asm volatile(                                                                                              \
        "v_mov_b32 v28, 1\n v_mov_b32 v29, 2\n v_mov_b32 v30, 3\n v_mov_b32 v31, 4\n v_mov_b32 v32, 5\n"        \
        "v_mov_b32 v33, 6\n v_mov_b32 v34, 7\n v_mov_b32 v35, 8\n v_mov_b32 v36, 9\n v_mov_b32 v37, 10\n"      \
        "v_mov_b32 v38, 11\n v_mov_b32 v39, 12\n v_mov_b32 v40, 13\n v_mov_b32 v41, 14\n v_mov_b32 v42, 15\n"  \
        "v_mov_b32 v43, 16\n" ::: CLOB);
#define OP3(op)                                                                                                \
    op " v20, v29, v30, v31\n" op " v21, v33, v34, v35\n" op " v22, v37, v38, v39\n" op " v23, v41, v42, v43\n" \
    op " v24, v29, v30, v31\n" op " v25, v33, v34, v35\n" op " v26, v37, v38, v39\n" op " v27, v41, v42, v43\n"
#define OP2(op)                                                                                                \
    op " v20, v29, v30\n" op " v21, v33, v34\n" op " v22, v37, v38\n" op " v23, v41, v42\n"                     \
    op " v24, v31, v28\n" op " v25, v35, v32\n" op " v26, v39, v36\n" op " v27, v43, v40\n"
#define OP2S(op, sfx)                                                                                          \
    op " v20, v29, v30" sfx "\n" op " v21, v33, v34" sfx "\n" op " v22, v37, v38" sfx "\n" op " v23, v41, v42" sfx "\n" \
    op " v24, v31, v28" sfx "\n" op " v25, v35, v32" sfx "\n" op " v26, v39, v36" sfx "\n" op " v27, v43, v40" sfx "\n"
#define OP1S(op, sfx)                                                                                          \
    op " v20, v29" sfx "\n" op " v21, v33" sfx "\n" op " v22, v37" sfx "\n" op " v23, v41" sfx "\n"             \
    op " v24, v31" sfx "\n" op " v25, v35" sfx "\n" op " v26, v39" sfx "\n" op " v27, v43" sfx "\n"
#define SDB " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
#define WSHR " wave_shr:1 row_mask:0xf bank_mask:0xf"
#define RSHR " row_shr:1 row_mask:0xf bank_mask:0xf"
#define QP " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"

template <int KIND>
__global__ void probe(int* out) {
    INIT
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (KIND == 0) asm volatile(OP3("v_max3_i32") ::: CLOB);
        if constexpr (KIND == 1) asm volatile(OP3("v_max3_f32") ::: CLOB);
        if constexpr (KIND == 2) asm volatile(OP2("v_max_f32") ::: CLOB);
        if constexpr (KIND == 3) asm volatile(OP2S("v_max_f32_e64", "") ::: CLOB);
        if constexpr (KIND == 4) asm volatile(OP3("v_med3_f32") ::: CLOB);
        if constexpr (KIND == 5) asm volatile(OP2("v_max_u32") ::: CLOB);
        if constexpr (KIND == 6) asm volatile(OP2("v_min_u32") ::: CLOB);
        if constexpr (KIND == 7) asm volatile(OP2("v_max_i32") ::: CLOB);
        if constexpr (KIND == 8) asm volatile(OP2("v_max_i16") ::: CLOB);
        if constexpr (KIND == 9) asm volatile(OP2("v_sub_f32") ::: CLOB);
        if constexpr (KIND == 10) asm volatile(OP2S("v_add_u32_e64", " clamp") ::: CLOB);
        if constexpr (KIND == 11) asm volatile(OP2("v_sub_u32") ::: CLOB);
        if constexpr (KIND == 12) asm volatile(OP2S("v_add_f32_e64", " clamp") ::: CLOB);
        if constexpr (KIND == 13) asm volatile(OP3("v_maximum3_f32") ::: CLOB);
        if constexpr (KIND == 14) asm volatile(OP3("v_bfe_i32") ::: CLOB);
        if constexpr (KIND == 15) asm volatile(OP3("v_and_or_b32") ::: CLOB);
        if constexpr (KIND == 16) asm volatile(OP3("v_lshl_add_u32") ::: CLOB);
        if constexpr (KIND == 17) asm volatile(OP2S("v_add_u32_sdwa", SDB) ::: CLOB);
        if constexpr (KIND == 18) asm volatile(OP2S("v_add_u32_dpp", WSHR) ::: CLOB);
        if constexpr (KIND == 19) asm volatile(OP2S("v_add_u32_dpp", RSHR) ::: CLOB);
        if constexpr (KIND == 20) asm volatile(OP1S("v_mov_b32_dpp", QP) ::: CLOB);
        if constexpr (KIND == 21) asm volatile(OP2S("v_max_f32_dpp", WSHR) ::: CLOB);
        if constexpr (KIND == 22) asm volatile(OP2S("v_add_f32_dpp", WSHR) ::: CLOB);
        if constexpr (KIND == 23) asm volatile(OP2("v_cndmask_b32") ::: CLOB, "vcc");
        if constexpr (KIND == 24) asm volatile(OP3("v_fma_f32") ::: CLOB);
        if constexpr (KIND == 25) asm volatile(OP2S("v_max_f32_sdwa", " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD") ::: CLOB);
        if constexpr (KIND == 26) asm volatile(OP2S("v_mul_u32_u24", "") ::: CLOB);
        if constexpr (KIND == 27) asm volatile(OP3("v_mad_u32_u24") ::: CLOB);
        if constexpr (KIND == 28) asm volatile(OP2("v_subrev_u32") ::: CLOB);
        if constexpr (KIND == 29) asm volatile(OP3("v_perm_b32") ::: CLOB);
        if constexpr (KIND == 30) asm volatile(OP2("v_lshrrev_b32") ::: CLOB);
        if constexpr (KIND == 31) asm volatile(OP2("v_xor_b32") ::: CLOB);
        if constexpr (KIND == 32) asm volatile(OP3("v_min3_f32") ::: CLOB);
        if constexpr (KIND == 33) asm volatile(OP2("v_add_f16") ::: CLOB);
        if constexpr (KIND == 34) asm volatile(OP2("v_max_f16") ::: CLOB);
        if constexpr (KIND == 35) asm volatile(OP2S("v_sub_u16_e64", " clamp") ::: CLOB);
        if constexpr (KIND == 36) asm volatile(OP2S("v_add_u16_e64", " clamp") ::: CLOB);
        if constexpr (KIND == 37) asm volatile(OP3("v_max3_u32") ::: CLOB);
    }
    int r;
    asm volatile("v_add_u32 %0, v20, v27" : "=v"(r)::CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int KIND>
void run(const char* name, int wps) {
    int* out;
    const int threads = wps * 256 > 1024 ? 1024 : wps * 256;
    const int blocks = 256 * (wps * 256 / threads);
    hipMalloc(&out, blocks * threads * 4);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(threads), 0, 0, out);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(threads), 0, 0, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"ns_per_instr_per_simd\": %.3f, \"ms\": %.3f}\n", name, wps,
           ms * 1e6 / (ITERS * 8.0 * wps), ms);
    fflush(stdout);
    hipFree(out);
}

// v_max_f32 / v_max3_f32 of int32 bit patterns, and the MODE register this kernel runs with
__global__ void fcheck(const int* a, const int* b, const int* c, int n, int* m2, int* m3, unsigned* mode) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *mode = __builtin_amdgcn_s_getreg((31 << 11) | 1);   // HW_REG_MODE, all 32 bits
    if (i >= n) return;
    int r2, r3;
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r2) : "v"(a[i]), "v"(b[i]));
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r3) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
    m2[i] = r2;
    m3[i] = r3;
}

static int check() {
    // operand values: the steps' range (|x| < 2^28) incl. denormal patterns (< 2^23), 0, negatives
    std::vector<int> vals = {0, 1, 2, 3, 7, 8, 100, 255, 256, 65535, 65536, 119470, (1 << 23) - 1, 1 << 23, (1 << 23) + 1,
                             (1 << 24) + 3, (1 << 27) + 5, (1 << 28) - 1, -1, -2, -3, -5, -128, -255, -65536,
                             -(1 << 23), -(1 << 28), (int)0x80000000u, (int)0x80000001u, 0x7F7FFFFF};
    for (int k = 0; k < 2000; ++k) vals.push_back((int)((unsigned)rand() % (1u << 28)) - (k % 3 == 0 ? (1 << 27) : 0));
    std::vector<int> A, B, C;
    for (size_t i = 0; i < vals.size(); ++i)
        for (size_t j = 0; j < 64 && j < vals.size(); ++j)
            for (size_t k = 0; k < 8; ++k) {
                A.push_back(vals[i]);
                B.push_back(vals[(i * 7 + j * 13 + 1) % vals.size()]);
                C.push_back(vals[(j * 31 + k * 101 + i) % vals.size()]);
            }
    // one operand of every triple non-negative (the clamped H - G of the steps): put it in C
    for (size_t i = 0; i < C.size(); ++i) C[i] = C[i] < 0 ? -C[i] & 0x0FFFFFFF : C[i];
    const int n = (int)A.size();
    int *da, *db, *dc, *d2, *d3;
    unsigned* dm;
    hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&d2, n * 4); hipMalloc(&d3, n * 4);
    hipMalloc(&dm, 4);
    hipMemcpy(da, A.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, C.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(fcheck, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dc, n, d2, d3, dm);
    std::vector<int> r2(n), r3(n);
    unsigned mode = 0;
    hipMemcpy(r2.data(), d2, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r3.data(), d3, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&mode, dm, 4, hipMemcpyDeviceToHost);
    long bad2 = 0, bad3 = 0, n2 = 0;
    for (int i = 0; i < n; ++i) {
        if (A[i] >= 0 || B[i] >= 0) {   // max of two with a non-negative one
            ++n2;
            if (r2[i] != std::max(A[i], B[i])) {
                if (bad2 < 5) printf("max2 mismatch: %d %d -> %d\n", A[i], B[i], r2[i]);
                ++bad2;
            }
        }
        if (r3[i] != std::max(std::max(A[i], B[i]), C[i])) {
            if (bad3 < 5) printf("max3 mismatch: %d %d %d -> %d\n", A[i], B[i], C[i], r3[i]);
            ++bad3;
        }
    }
    printf("{\"check\": \"v_max_f32 / v_max3_f32 on int32 patterns, one operand >= 0\", \"cases_max2\": %ld, "
           "\"bad_max2\": %ld, \"cases_max3\": %d, \"bad_max3\": %ld, \"mode\": \"0x%08x\", \"fp_denorm_bits\": %u}\n",
           n2, bad2, n, bad3, mode, (mode >> 4) & 0xF);
    return (bad2 || bad3) ? 1 : 0;
}

int main() {
    const int bad = check();
    for (int t : {1, 2, 4}) {
        run<0>("v_max3_i32", t);
        run<1>("v_max3_f32", t);
        run<37>("v_max3_u32", t);
        run<2>("v_max_f32", t);
        run<3>("v_max_f32_e64", t);
        run<4>("v_med3_f32", t);
        run<32>("v_min3_f32", t);
        run<13>("v_maximum3_f32", t);
        run<5>("v_max_u32", t);
        run<6>("v_min_u32", t);
        run<7>("v_max_i32", t);
        run<8>("v_max_i16", t);
        run<34>("v_max_f16", t);
        run<33>("v_add_f16", t);
        run<9>("v_sub_f32", t);
        run<10>("v_add_u32_e64 clamp", t);
        run<35>("v_sub_u16_e64 clamp", t);
        run<36>("v_add_u16_e64 clamp", t);
        run<11>("v_sub_u32", t);
        run<28>("v_subrev_u32", t);
        run<12>("v_add_f32_e64 clamp", t);
        run<14>("v_bfe_i32", t);
        run<15>("v_and_or_b32", t);
        run<16>("v_lshl_add_u32", t);
        run<17>("v_add_u32_sdwa", t);
        run<25>("v_max_f32_sdwa", t);
        run<18>("v_add_u32_dpp wave_shr", t);
        run<19>("v_add_u32_dpp row_shr", t);
        run<20>("v_mov_b32_dpp quad_perm", t);
        run<21>("v_max_f32_dpp wave_shr", t);
        run<22>("v_add_f32_dpp wave_shr", t);
        run<23>("v_cndmask_b32", t);
        run<24>("v_fma_f32", t);
        run<26>("v_mul_u32_u24", t);
        run<27>("v_mad_u32_u24", t);
        run<29>("v_perm_b32", t);
        run<30>("v_lshrrev_b32", t);
        run<31>("v_xor_b32", t);
    }
    return bad;
}
