// ubench_dpplat.hip -- lone-wave latency of a loop-carried chain through a DPP source
// read (tools only): max3 writes X, k independent fillers, DPP-add reads X as its
// source and writes Y, max3 reads Y ... (the flow2 W2 recurrence HB -> DPP-add -> H).
// Prints ns per chain link pair for k = 2..8 fillers, and the same chain with a plain
// v_add in place of the DPP-add.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 8192
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32"
#define F "v_max3_i32 v25, v26, v27, v28\n"
#define F2 F F
#define F4 F2 F2
#define M3 "v_max3_i32 v20, v21, v30, v31\n"
#define DPP "v_add_u32_dpp v21, v20, v32 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define ADD "v_add_u32 v21, v20, v32\n"
template <int K>
__global__ void lat(int* o) {
    asm volatile("v_mov_b32 v20, 1\n v_mov_b32 v21, 2\n v_mov_b32 v26, 3\n v_mov_b32 v27, 4\n v_mov_b32 v28, 5\n"
                 "v_mov_b32 v30, 6\n v_mov_b32 v31, 7\n v_mov_b32 v32, 8\n" ::: CLOB);
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (K == 2) asm volatile(M3 F2 DPP M3 F2 DPP M3 F2 DPP M3 F2 DPP ::: CLOB);
        if constexpr (K == 3) asm volatile(M3 F2 F DPP M3 F2 F DPP M3 F2 F DPP M3 F2 F DPP ::: CLOB);
        if constexpr (K == 4) asm volatile(M3 F4 DPP M3 F4 DPP M3 F4 DPP M3 F4 DPP ::: CLOB);
        if constexpr (K == 6) asm volatile(M3 F4 F2 DPP M3 F4 F2 DPP M3 F4 F2 DPP M3 F4 F2 DPP ::: CLOB);
        if constexpr (K == 8) asm volatile(M3 F4 F4 DPP M3 F4 F4 DPP M3 F4 F4 DPP M3 F4 F4 DPP ::: CLOB);
        if constexpr (K == 102) asm volatile(M3 F2 ADD M3 F2 ADD M3 F2 ADD M3 F2 ADD ::: CLOB);
        if constexpr (K == 100) asm volatile(M3 ADD M3 ADD M3 ADD M3 ADD ::: CLOB);
        if constexpr (K == 200) asm volatile(M3 "s_nop 1\n" DPP M3 "s_nop 1\n" DPP M3 "s_nop 1\n" DPP M3 "s_nop 1\n" DPP ::: CLOB);
    }
    int r;
    asm volatile("v_mov_b32 %0, v21" : "=v"(r)::CLOB);
    o[blockIdx.x * 64 + threadIdx.x] = r;
}
template <int K>
void run(const char* n, int per_link_instr) {
    int* o;
    hipMalloc(&o, 256 * 64 * 4);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(lat<K>, dim3(256), dim3(64), 0, 0, o);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(lat<K>, dim3(256), dim3(64), 0, 0, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double per_pair = ms * 1e6 / (ITERS * 4.0);
    printf("{\"probe\": \"%s\", \"ns_per_max3_dpp_pair\": %.2f, \"instr_per_pair\": %d, \"ns_per_instr\": %.3f}\n", n, per_pair,
           per_link_instr, per_pair / per_link_instr);
    fflush(stdout);
    hipFree(o);
}
int main() {
    for (int rep = 0; rep < 2; ++rep) {
        run<200>("max3 -> s_nop 1 -> dpp_add(src) -> max3", 3);
        run<2>("max3 -> 2 fillers -> dpp_add(src)", 4);
        run<3>("max3 -> 3 fillers -> dpp_add(src)", 5);
        run<4>("max3 -> 4 fillers -> dpp_add(src)", 6);
        run<6>("max3 -> 6 fillers -> dpp_add(src)", 8);
        run<8>("max3 -> 8 fillers -> dpp_add(src)", 10);
        run<100>("max3 -> v_add (no dpp)", 2);
        run<102>("max3 -> 2 fillers -> v_add", 4);
    }
    return 0;
}
