// ubench_tput.hip -- gfx950 VALU issue cost per instruction class (tools only).
// Each probe runs 8 independent chains of one instruction (inline asm, so the
// compiler cannot fold them) for ITERS iterations; cycles per instruction per
// wave and per SIMD are printed for 1, 2, 4 and 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_tput.hip -o build/ubench_tput
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

#define ITERS 2048

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ void tput(int* out, unsigned long long* cyc, int seed) {
    int v0 = threadIdx.x + seed, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6,
        v7 = v0 + 7;
    const int a = seed * 3 + 1, b = seed ^ 0x5555;
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < ITERS; ++i) {
#define OP(k)                                                                                                   \
    if constexpr (KIND == 0) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));           \
    if constexpr (KIND == 1) asm volatile("v_max_i32 %0, %0, %1" : "+v"(v##k) : "v"(a));                       \
    if constexpr (KIND == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));           \
    if constexpr (KIND == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));           \
    if constexpr (KIND == 4) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(v##k) : "v"(a));                    \
    if constexpr (KIND == 5) asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(v##k) : "v"(a));              \
    if constexpr (KIND == 6) asm volatile("v_subrev_u32 %0, %1, %0" : "+v"(v##k) : "v"(a));                   \
    if constexpr (KIND == 7) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v##k) : "v"(a)); \
    if constexpr (KIND == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v##k) : "v"(a) : "vcc");       \
    if constexpr (KIND == 9) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));           \
    if constexpr (KIND == 10) asm volatile("v_pk_add_u16 %0, %0, %1 clamp" : "+v"(v##k) : "v"(a));             \
    if constexpr (KIND == 11) asm volatile("v_max_u16 %0, %0, %1" : "+v"(v##k) : "v"(a));                      \
    if constexpr (KIND == 12) asm volatile("v_sub_u32 %0, %0, %1 clamp" : "+v"(v##k) : "v"(a));                \
    if constexpr (KIND == 13) asm volatile("v_max3_i16 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));           \
    if constexpr (KIND == 14) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));   \
    if constexpr (KIND == 15) asm volatile("v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(v##k) : "v"(a)); \
    if constexpr (KIND == 16) asm volatile("v_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v##k) : "v"(a), "v"(b)); \
    if constexpr (KIND == 17) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v##k) : "v"(a), "v"(b));            \
    if constexpr (KIND == 18) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v##k) : "v"(a));                       \
    if constexpr (KIND == 19) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v##k) : "v"(a));
        REP8(OP)
#undef OP
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int KIND>
void run(const char* name, int threads) {
    int* out;
    unsigned long long* cyc;
    const int blocks = 256, waves = blocks * threads / 64;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, waves * 8);
    hipLaunchKernelGGL(tput<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(tput<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 2);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(waves);
    hipMemcpy(h.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : h) avg += v; avg /= waves;
    const double per_wave = avg / (ITERS * 8.0);
    const int wps = threads / 256 > 0 ? threads / 256 : 1;   // waves per SIMD (one block per CU)
    printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_wave\": %.2f, \"cyc_per_instr_per_simd\": %.2f, "
           "\"ms\": %.3f, \"ghz\": %.2f}\n", name, threads < 256 ? 0 : wps, per_wave, per_wave / (threads < 256 ? 1 : wps), ms,
           avg / (ms * 1e6));
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int t : {256, 512, 1024}) {   // 1, 2, 4 waves per SIMD (one 4..16-wave block per CU)
        run<0>("v_max3_i32", t);
        run<9>("v_max3_u32", t);
        run<1>("v_max_i32", t);
        run<2>("v_add3_u32", t);
        run<3>("v_perm_b32", t);
        run<6>("v_subrev_u32", t);
        run<12>("v_sub_u32_clamp", t);
        run<4>("v_pk_max_u16", t);
        run<5>("v_pk_sub_u16_clamp", t);
        run<10>("v_pk_add_u16_clamp", t);
        run<11>("v_max_u16", t);
        run<13>("v_max3_i16", t);
        run<7>("v_mov_dpp_wave_shr", t);
        run<8>("v_cndmask_vcc", t);
        run<14>("v_pk_maximum3_f16", t);
        run<15>("v_add_u32_sdwa", t);
        run<16>("v_add_u32_dpp", t);
        run<17>("v_fma_f32", t);
        run<18>("v_add_f32", t);
        run<19>("v_add_u32", t);
    }
    return 0;
}
