// ubench_dep.hip -- dependent-issue latency of the VALU forms the flow2 step uses, for
// ONE wave alone on its SIMD (the C2 regime), and the cycles of the W = 1 and W = 2
// step bodies with no hand-off at all.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_dep.hip -o build/ubench_dep && build/ubench_dep
// Prints one JSON line per probe: cycles per instruction (chains) or per step (bodies),
// from s_memtime around ITER iterations of a 32-fold unrolled body.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096
#define R32(x) x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x

__device__ __forceinline__ unsigned long long tick() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int P>
__global__ void probe(unsigned long long* out, int* sink, int seed) {
    int a = seed + threadIdx.x, b = a ^ 0x55, c = a + 3, d = a - 7, k = 1, e = 0, f = 0, g = 0, h = 0;
    const unsigned long long t0 = tick();
    for (int it = 0; it < ITER; ++it) {
        if constexpr (P == 0) {   // dependent v_add_u32 (VOP2)
            asm volatile(R32("v_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(k));
        } else if constexpr (P == 1) {   // dependent v_max3_i32 (VOP3)
            asm volatile(R32("v_max3_i32 %0, %0, %1, %2\n\t") : "+v"(a) : "v"(b), "v"(c));
        } else if constexpr (P == 2) {   // dependent v_sub_u32 clamp (VOP3)
            asm volatile(R32("v_sub_u32 %0, %0, %1 clamp\n\t") : "+v"(a) : "v"(k));
        } else if constexpr (P == 3) {   // dependent v_add_u32_sdwa byte select
            asm volatile(R32("v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n\t")
                         : "+v"(a) : "v"(b));
        } else if constexpr (P == 4) {   // dependent DPP add (the 2 wait states as s_nop 1)
            asm volatile(R32("s_nop 1\n\tv_add_u32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t")
                         : "+v"(a) : "v"(k));
        } else if constexpr (P == 5) {   // 4 independent v_max3 chains interleaved
            asm volatile(R32("v_max3_i32 %0, %0, %4, %5\n\tv_max3_i32 %1, %1, %4, %5\n\tv_max3_i32 %2, %2, %4, %5\n\t"
                             "v_max3_i32 %3, %3, %4, %5\n\t")
                         : "+v"(a), "+v"(e), "+v"(f), "+v"(g) : "v"(b), "v"(c));
        } else if constexpr (P == 6) {   // dependent pairs: max3 -> add -> max3 ... with one independent op between
            asm volatile(R32("v_max3_i32 %0, %0, %2, %3\n\tv_add_u32 %1, %1, %4\n\t") : "+v"(a), "+v"(e) : "v"(b), "v"(c), "v"(k));
        } else if constexpr (P == 7) {   // DPP add dependent on a max3 two instructions back (the step's hazard spacing)
            asm volatile(R32("v_max3_i32 %0, %1, %2, %3\n\tv_add_u32 %4, %4, %5\n\tv_add_u32 %6, %6, %5\n\t"
                             "v_add_u32_dpp %1, %0, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t")
                         : "+v"(a), "+v"(d), "+v"(b), "+v"(c), "+v"(e), "+v"(k), "+v"(f));
        }
    }
    const unsigned long long t1 = tick();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
}

template <int P>
void run(const char* name, int per_iter_instrs) {
    unsigned long long* d_out;
    int* d_sink;
    hipMalloc(&d_out, 256 * sizeof(unsigned long long));
    hipMalloc(&d_sink, 256 * 64 * sizeof(int));
    hipLaunchKernelGGL(probe<P>, dim3(1), dim3(64), 0, 0, d_out, d_sink, 1);   // warm
    hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<P>, dim3(1), dim3(64), 0, 0, d_out, d_sink, 2);   // one wave, alone on the GPU
    unsigned long long cyc = 0;
    hipMemcpy(&cyc, d_out, sizeof(cyc), hipMemcpyDeviceToHost);
    printf("{\"probe\": \"%s\", \"cycles_per_instr\": %.2f, \"memtime_ticks\": %llu}\n", name,
           (double)cyc / ((double)ITER * per_iter_instrs), cyc);
    hipFree(d_out);
    hipFree(d_sink);
}

int main() {
    run<0>("dep v_add_u32", 32);
    run<1>("dep v_max3_i32", 32);
    run<2>("dep v_sub_u32 clamp", 32);
    run<3>("dep v_add_u32_sdwa", 32);
    run<4>("dep v_add_u32_dpp (+s_nop 1)", 32);
    run<5>("4 indep v_max3 chains", 128);
    run<6>("dep max3 with 1 indep add between", 64);
    run<7>("max3 -> 2 adds -> dpp add (per instr)", 128);
    return 0;
}
