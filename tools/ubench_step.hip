// ubench_step.hip -- cycles per anti-diagonal step of the flow2 step body
// (sw_flow2.hip) with no hand-off waits: one wave per SIMD (256 blocks x 4
// waves), each running CHUNKS x 32 steps with constant inflow registers.
// Variants isolate what one step costs: the full body, without the per-step
// outflow ds_write, without the DPP (plain adds), and the dependency chain only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_step.hip -o build/ubench_step && build/ubench_step
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHUNKS 512
constexpr int C = 32;

__device__ __forceinline__ unsigned long long tick() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ int dpp_add_shr1(int src, int k) {
    return __builtin_amdgcn_update_dpp(0, src, 0x138, 0xF, 0xF, false) + k;
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
__device__ __forceinline__ int vmax3(int a, int b, int c) {
    int d;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// v_add_u32_dpp with the destination tied to 'old': lanes 1..63 get src[l-1] + k,
// lane 0 (no wave_shr source) keeps old.  The s_nop 1 covers the VALU -> DPP
// read hazard the compiler cannot see inside inline asm.
template <bool NOP>
__device__ __forceinline__ int dpp_add_tied(int old, int src, int k) {
    if constexpr (NOP)
        asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(old) : "v"(src), "v"(k));
    else
        asm("v_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(old) : "v"(src), "v"(k));
    return old;
}

// tied DPP-add whose VALU->DPP read hazard is covered by data dependence: 'after'
// is computed >= 2 instructions after 'src', so the asm cannot issue earlier.
__device__ __forceinline__ int dpp_add_dep(int old, int src, int k, int after) {
    asm("v_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf ; after %3" : "+v"(old) : "v"(src), "v"(k), "v"(after));
    return old;
}
constexpr int DPP_WAVE_SHL1 = 0x130;

template <int B>
__device__ __forceinline__ int sbyte(unsigned w) {
    if constexpr (B == 3) return (int)w >> 24;
    else return (int)(signed char)(w >> (8 * B));
}

// V: 0 full step; 1 no ds_write; 2 no DPP (plain add); 3 no DPP, no write;
//    4 full step with s_setprio 3;
//    5 chunk model: lane-0-only K reads, tied asm DPP (+s_nop 1), lane-63-only
//      quad writes of the DPP results at chunk end;  6 as 5 without the s_nop;
//    8 rotation model: per step wave_shl deposit + tied DPP-add per quantity,
//      one ds_read2_b32 / ds_write2_b32 per chunk;
//    7 chunk model with all-lane K reads (lanes 1..63 read constants), combined
//      DPP, lane-63-only quad writes at chunk end
template <int V>
__global__ void __launch_bounds__(256) step_probe(int* out, unsigned long long* cyc, int go, int ge, unsigned seed) {
    __shared__ int2 sink[4][64 + C];
    __shared__ __attribute__((aligned(16))) int4 kring[4][C / 2];
    __shared__ __attribute__((aligned(16))) int4 kconst[C / 2];
    if (threadIdx.x < C / 2) kconst[threadIdx.x] = make_int4(-go, -ge, -go, -ge);
    if ((threadIdx.x & 63) < C / 2) kring[threadIdx.x >> 6][threadIdx.x & 63] = make_int4(-2, -3, -4, -5);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (V == 4) __builtin_amdgcn_s_setprio(3);
    int H = 0, E = 0, fh = -ge, L0 = -go, ehP = -ge, M = 0;
    const unsigned prof = 0x00020002u ^ seed;
    unsigned P[C / 4];
    for (int u = 0; u < C / 4; ++u) P[u] = __builtin_amdgcn_perm(prof, 0x80808080u, 0x04050607u + u + lane);
    // distinct registers per row, as ds_read_b128 gives them in the kernel
    int4 K[C / 2];
    const int4* kin = reinterpret_cast<const int4*>(out) + (lane == 0 ? 0 : C / 2);
    for (int u = 0; u < C / 2; ++u) K[u] = kin[u];
    int2* const wb = &sink[wave][lane];
    const int neggo = -go, negge = -ge;
    const unsigned long long t0 = tick();
    for (int c = 0; c < CHUNKS; ++c) {
        if constexpr (V >= 5) {
            if constexpr (V == 7) {
                const int4* kb = lane == 0 ? kring[wave] : kconst;
#pragma unroll
                for (int u = 0; u < C / 2; ++u) K[u] = kb[u];
            } else if (lane == 0) {
#pragma unroll
                for (int u = 0; u < C / 2; ++u) K[u] = kring[wave][u];
            }
        }
#pragma unroll
        for (int j = 0; j < C; j += 4) {
            auto step = [&](auto b_c) __attribute__((always_inline)) {
                constexpr int b = decltype(b_c)::value;
                const int jj = j + b;
                const int kh = (jj & 1) ? K[jj >> 1].z : K[jj >> 1].x;
                const int ke = (jj & 1) ? K[jj >> 1].w : K[jj >> 1].y;
                int hgL, ehL;
                if constexpr (V == 2 || V == 3) { hgL = H + kh; ehL = E + ke; }
                else if constexpr (V == 5 || V == 6) {
                    hgL = dpp_add_tied<V == 5>(kh, H, neggo); ehL = dpp_add_tied<V == 5>(ke, E, negge);
                    if (jj & 1) { K[jj >> 1].z = hgL; K[jj >> 1].w = ehL; } else { K[jj >> 1].x = hgL; K[jj >> 1].y = ehL; }
                } else {
                    hgL = dpp_add_shr1(H, kh); ehL = dpp_add_shr1(E, ke);
                    if constexpr (V == 7) {
                        if (jj & 1) { K[jj >> 1].z = hgL; K[jj >> 1].w = ehL; } else { K[jj >> 1].x = hgL; K[jj >> 1].y = ehL; }
                    }
                }
                if constexpr (V <= 4 && V != 1 && V != 3) wb[jj] = make_int2(L0, ehP);
                const int t = L0 + sbyte<b>(P[j >> 2]);
                const int hgO = H - go;
                E = max3i(ehL, hgL, 0);
                const int F = max3i(fh, hgO, 0);
                fh = F - ge;
                H = vmax3(t, E, F);
                M = max(M, t);
                L0 = hgL;
                ehP = ehL;
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
        }
        if constexpr (V >= 5) {
            if (lane == 63) {
#pragma unroll
                for (int u = 0; u < C / 2; ++u) reinterpret_cast<int4*>(&sink[wave][0])[u] = K[u];
            }
        }
        __asm__ __volatile__("" ::: "memory");
    }
    const unsigned long long t1 = tick();
    out[1024 + blockIdx.x * blockDim.x + threadIdx.x] = M + H + E + fh;
    if (lane == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

__global__ void __launch_bounds__(256) rot_probe(int* out, unsigned long long* cyc, int go, int ge, unsigned seed) {
    __shared__ int2 ring[4][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 1024; i += 256) ring[i / 256][i % 256] = make_int2(-go, -ge);
    __syncthreads();
    int H = 0, E = 0, fh = -ge, L0 = -go, ehP = -ge, M = 0;
    const unsigned prof = 0x00020002u ^ seed;
    unsigned P[C / 4];
    for (int u = 0; u < C / 4; ++u) P[u] = __builtin_amdgcn_perm(prof, 0x80808080u, 0x04050607u + u + lane);
    const int neggo = -go, negge = -ge;
    int IOH = -go, IOE = -ge;
    int hgO = -go;
    const unsigned long long t0 = tick();
    for (int c = 0; c < CHUNKS; ++c) {
        {   // outflow of the last chunk (lanes 64-C..63), inflow of this one (lanes 0..C-1)
            int2* wp = &ring[wave][(lane + c * C) & 255];
            wp->x = IOH; wp->y = IOE;
            __asm__ __volatile__("" ::: "memory");
            const int2 v = ring[wave][(lane + c * C + 64) & 255];
            IOH = v.x; IOE = v.y;
        }
#pragma unroll
        for (int j = 0; j < C; j += 4) {
            auto step = [&](auto b_c) __attribute__((always_inline)) {
                constexpr int b = decltype(b_c)::value;
                const int t = L0 + sbyte<b>(P[j >> 2]);
                const int ioh = __builtin_amdgcn_update_dpp(L0, IOH, DPP_WAVE_SHL1, 0xF, 0xF, false);
                const int ioe = __builtin_amdgcn_update_dpp(ehP, IOE, DPP_WAVE_SHL1, 0xF, 0xF, false);
                const int F = max3i(fh, hgO, 0);
                const int hgL = dpp_add_dep(IOH, H, neggo, F);      // H -> hgO -> F -> DPP
                const int ehL = dpp_add_dep(IOE, E, negge, hgO);    // E -> H -> hgO -> DPP
                IOH = ioh; IOE = ioe;
                E = max3i(ehL, hgL, 0);
                fh = F - ge;
                H = vmax3(t, E, F);
                hgO = H - go;
                M = max(M, t);
                L0 = hgL;
                ehP = ehL;
            };
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
        }
        __asm__ __volatile__("" ::: "memory");
    }
    const unsigned long long t1 = tick();
    out[1024 + blockIdx.x * blockDim.x + threadIdx.x] = M + H + E + fh + IOH + IOE;
    if (lane == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int V>
void run(const char* name, int blocks) {
    int* out; unsigned long long* cyc;
    const int waves = blocks * 4;
    hipMalloc(&out, blocks * 256 * 4 + 4096);
    {
        std::vector<int> kv(2 * C * 2);
        for (int u = 0; u < C / 2; ++u) {   // lane 0's inflow rows, then the constants of lanes 1..63
            kv[4 * u] = -1 - (u & 3); kv[4 * u + 1] = -1 - (u & 1); kv[4 * u + 2] = -1 - (u & 2); kv[4 * u + 3] = -1;
            kv[2 * C + 4 * u] = -1; kv[2 * C + 4 * u + 1] = -1; kv[2 * C + 4 * u + 2] = -1; kv[2 * C + 4 * u + 3] = -1;
        }
        hipMemcpy(out, kv.data(), kv.size() * 4, hipMemcpyHostToDevice);
    }
    hipMalloc(&cyc, waves * 8);
    auto kern = V == 8 ? rot_probe : step_probe<V>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, cyc, 1, 1, 1u);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, cyc, 1, 1, 2u);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(waves);
    hipMemcpy(h.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : h) avg += v; avg /= waves;
    const double steps = (double)CHUNKS * C;
    printf("{\"probe\": \"%s\", \"blocks\": %d, \"cyc_per_step\": %.2f, \"ns_per_step\": %.3f, \"clock_ghz_est\": %.2f}\n",
           name, blocks, avg / steps, ms * 1e6 / steps, avg / (ms * 1e6));
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int b : {1, 256}) {
        run<0>("flow2_step", b);
        run<1>("no_write", b);
        run<2>("no_dpp", b);
        run<3>("no_dpp_no_write", b);
        run<4>("flow2_step_prio3", b);
        run<5>("chunk_tied_nop", b);
        run<6>("chunk_tied_nonop", b);
        run<7>("chunk_alllane_reads", b);
        run<8>("rotation", b);
    }
    return 0;
}
