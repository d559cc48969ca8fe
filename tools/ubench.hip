// ubench.hip -- gfx950 latency/throughput probes for the SW step's instruction
// mix (tools only; not part of the engine).  One kernel per probe; each wave
// times N iterations with s_memtime and writes cycles/iteration.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o build/ubench && build/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

#define ITERS 4096

__device__ __forceinline__ unsigned long long tick() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int KIND>
__global__ void probe(int* out, unsigned long long* cyc, int seed) {
    int a = threadIdx.x + seed, b = a * 3 + 1, c = a ^ 5, d = a + 7;
    int e = a * 11, f = a - 3, g = a + 9, h = a * 5;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = tick();
#pragma unroll 16
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (KIND == 0) {            // dependent v_max3_i32 chain
            a = max(max(a, b), c);
            a = max(max(a, d), e);
        } else if constexpr (KIND == 1) {     // dependent v_add3 chain
            a = a + b + c;
            a = a + d + e;
        } else if constexpr (KIND == 2) {     // dependent DPP wave_shr chain + one VALU (dpp needs a VALU producer)
            a = __builtin_amdgcn_update_dpp(b, a, 0x138, 0xF, 0xF, false);
            a = a + c;
        } else if constexpr (KIND == 3) {     // dependent DPP row_shr:1 (0x111) + VALU
            a = __builtin_amdgcn_update_dpp(b, a, 0x111, 0xF, 0xF, false);
            a = a + c;
        } else if constexpr (KIND == 4) {     // 8 independent max3 chains (ILP 8)
            a = max(max(a, b), c); d = max(max(d, b), c); e = max(max(e, b), c); f = max(max(f, b), c);
            g = max(max(g, b), c); h = max(max(h, b), c); b = max(max(b, a), c); c = max(max(c, a), d);
        } else if constexpr (KIND == 5) {     // dependent chain: max3 -> sub (the SW E/H/Hg chain shape)
            a = max(max(a, b), 0);
            a = a - c;
        } else if constexpr (KIND == 6) {     // dependent ds_swizzle / shfl_up-like via ds_bpermute
            a = __builtin_amdgcn_ds_bpermute((int)((threadIdx.x + 63) & 63) << 2, a);
            a = a + c;
        } else if constexpr (KIND == 7) {     // v_perm dependent chain
            a = (int)__builtin_amdgcn_perm((unsigned)b, (unsigned)a, 0x0C0C0C01u);
            a = a + c;
        }
    }
    const unsigned long long t1 = tick();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int KIND>
void run(const char* name, int ops_per_iter, int blocks, int threads) {
    int* out; unsigned long long* cyc;
    const int waves = blocks * threads / 64;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, waves * 8);
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 2);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(waves);
    hipMemcpy(h.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : h) avg += v; avg /= waves;
    printf("{\"probe\": \"%s\", \"blocks\": %d, \"threads\": %d, \"cyc_per_iter\": %.2f, \"cyc_per_op\": %.2f, "
           "\"ms\": %.4f, \"clock_ghz_est\": %.2f}\n",
           name, blocks, threads, avg / ITERS, avg / ITERS / ops_per_iter, ms, avg / (ms * 1e6));
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int t : {64, 128, 256, 512}) {   // 1, 2, 4, 8 waves per CU (threads/64 spread over 4 SIMDs)
        run<0>("max3_dep", 2, 256, t);
        run<1>("add3_dep", 2, 256, t);
        run<2>("dpp_wave_shr_dep", 2, 256, t);
        run<3>("dpp_row_shr_dep", 2, 256, t);
        run<4>("max3_ilp8", 8, 256, t);
        run<5>("max3_sub_dep", 2, 256, t);
        run<6>("bpermute_dep", 2, 256, t);
        run<7>("perm_dep", 2, 256, t);
    }
    return 0;
}
