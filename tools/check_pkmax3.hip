// check_pkmax3.hip -- v_pk_maximum3_f16 as an unsigned-16 max3 on gfx950 (tools only):
// for half-words in [0, 0x7BFF] (no Inf/NaN patterns, sign bit clear) the IEEE
// maximum of the f16 values is the integer maximum of the bit patterns, provided
// f16 denormals are not flushed.  Sweeps every a in [0, 0x7BFF] against random
// (b, c) and the edge values, on the GPU, and counts mismatches.
//   hipcc --offload-arch=gfx950 -O3 tools/check_pkmax3.hip -o tools/bin/check_pkmax3
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void check(unsigned long long* bad, unsigned seed) {
    const unsigned a = blockIdx.x * blockDim.x + threadIdx.x;   // 0 .. 0x7BFF (low half)
    if (a > 0x7BFFu) return;
    unsigned s = a * 2654435761u ^ seed;
    unsigned long long nbad = 0;
    for (int i = 0; i < 4096; ++i) {
        s = s * 1664525u + 1013904223u;
        unsigned b = (s >> 3) % 0x7C00u, c = (s >> 17) % 0x7C00u;
        if (i < 6) { const unsigned e[6] = {0u, 1u, 0x3FFu, 0x400u, 0x7BFEu, 0x7BFFu}; b = e[i]; c = e[(i + 3) % 6]; }
        const unsigned hi_a = (a * 7u + 13u) % 0x7C00u;
        const unsigned A = a | (hi_a << 16), B = b | (c << 16), Cw = c | (b << 16);
        unsigned d;
        asm volatile("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(A), "v"(B), "v"(Cw));
        const unsigned lo = max(max(a, b), c), hi = max(max(hi_a, c), b);
        nbad += (d != (lo | (hi << 16)));
    }
    atomicAdd(bad, nbad);
}

int main() {
    unsigned long long* bad;
    hipMalloc(&bad, 8);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(check, dim3(0x7C00 / 256), dim3(256), 0, 0, bad, 12345u);
    unsigned long long h = 0;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    printf("{\"check\": \"v_pk_maximum3_f16 as u16 max3 on [0,0x7BFF]\", \"cases\": %llu, \"mismatches\": %llu}\n",
           (unsigned long long)0x7C00 * 4096ull, h);
    return h != 0;
}
