// ubench_lanex.hip -- does a lane shift through the LDS crossbar (ds_bpermute_b32) instead of a
// DPP move free VALU issue slots in the throughput-bound ring step (tools only)?
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lanex.hip -o build/ubench_lanex
//
// Each iteration is one three-column linear-gap ring step's VALU mix (sw_flow3r3_loops.inc
// step3: 3 SDWA adds, 2 DPP, 4.5 max3, 3 clamped subtracts, 0.75 perm; written as 2 steps per
// iteration) on fixed registers, at 1 / 2 / 4 waves per SIMD, ns per step per SIMD.
//   KIND 0: as the ring loops (the conveyor v_mov_b32_dpp wave_shl and the hand-off v_add_u32_dpp
//           wave_shr)
//   KIND 1: the conveyor move as a ds_bpermute_b32 issued one step ahead (its result waited for
//           with lgkmcnt a step later)
//   KIND 2: both lane shifts as ds_bpermute_b32 (the hand-off one's result used in its own step)
//   KIND 3: the step without any lane shift (lower bound)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITERS 8192
#define CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", \
             "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45"

#define SD(d, s, b) "v_add_u32_sdwa " d ", sext(" s "), v30 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" b " src1_sel:DWORD\n"
// the step body without its lane shifts: t's, the column chain, the running max
#define BODY(b)                                                                                   \
    SD("v21", "v31", b) SD("v22", "v32", b) SD("v23", "v33", b)                                   \
    "v_max3_i32 v24, v34, v25, v21\n v_sub_u32_e64 v25, v24, 1 clamp\n"                          \
    "v_max3_i32 v26, v25, v27, v22\n v_sub_u32_e64 v27, v26, 1 clamp\n"                          \
    "v_max3_i32 v28, v27, v29, v23\n v_sub_u32_e64 v29, v28, 1 clamp\n"                          \
    "v_max3_i32 v35, v35, v21, v22\n"
#define MAXC "v_max3_i32 v35, v35, v23, v36\n"
#define PERM "v_perm_b32 v31, v37, v38, v39\n v_perm_b32 v32, v37, v38, v40\n v_perm_b32 v33, v37, v38, v41\n"
#define DPP2 "v_mov_b32_dpp v30, v34 wave_shl:1 row_mask:0xf bank_mask:0xf\n" \
             "v_add_u32_dpp v34, v28, v42 wave_shr:1 row_mask:0xf bank_mask:0xf\n"

template <int KIND>
__global__ void probe(int* out) {
    asm volatile(
        "v_mov_b32 v20, 0\n v_mov_b32 v21, 1\n v_mov_b32 v22, 2\n v_mov_b32 v23, 3\n v_mov_b32 v24, 4\n"
        "v_mov_b32 v25, 5\n v_mov_b32 v26, 6\n v_mov_b32 v27, 7\n v_mov_b32 v28, 8\n v_mov_b32 v29, 9\n"
        "v_mov_b32 v30, 10\n v_mov_b32 v31, 11\n v_mov_b32 v32, 12\n v_mov_b32 v33, 13\n v_mov_b32 v34, 14\n"
        "v_mov_b32 v35, 0\n v_mov_b32 v36, 0\n v_mov_b32 v37, 0x01020304\n v_mov_b32 v38, 0x80808080\n"
        "v_mov_b32 v39, 0x04050607\n v_mov_b32 v40, 0x05060704\n v_mov_b32 v41, 0x06070405\n v_mov_b32 v42, -1\n"
        "v_mbcnt_lo_u32_b32 v43, -1, 0\n v_mbcnt_hi_u32_b32 v43, -1, v43\n"
        "v_add_u32 v44, 1, v43\n v_lshlrev_b32 v44, 2, v44\n"       // lane l reads lane l + 1 (conveyor)
        "v_add_u32 v45, -1, v43\n v_lshlrev_b32 v45, 2, v45\n"      // lane l reads lane l - 1 (hand-off)
        ::: CLOB);
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (KIND == 0)
            asm volatile(DPP2 BODY("0") MAXC DPP2 BODY("1") PERM ::: CLOB);
        if constexpr (KIND == 1)
            asm volatile("s_waitcnt lgkmcnt(0)\n ds_bpermute_b32 v30, v44, v34\n"
                         "v_add_u32_dpp v34, v28, v42 wave_shr:1 row_mask:0xf bank_mask:0xf\n" BODY("0") MAXC
                         "s_waitcnt lgkmcnt(0)\n ds_bpermute_b32 v30, v44, v34\n"
                         "v_add_u32_dpp v34, v28, v42 wave_shr:1 row_mask:0xf bank_mask:0xf\n" BODY("1") PERM ::: CLOB);
        if constexpr (KIND == 2)
            asm volatile("ds_bpermute_b32 v30, v44, v34\n ds_bpermute_b32 v34, v45, v28\n s_waitcnt lgkmcnt(0)\n"
                         BODY("0") MAXC
                         "ds_bpermute_b32 v30, v44, v34\n ds_bpermute_b32 v34, v45, v28\n s_waitcnt lgkmcnt(0)\n"
                         BODY("1") PERM ::: CLOB);
        if constexpr (KIND == 3)
            asm volatile(BODY("0") MAXC BODY("1") PERM ::: CLOB);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int r;
    asm volatile("v_add_u32 %0, v35, v34" : "=v"(r)::CLOB);
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
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(threads), 0, 0, out);
        hipEventRecord(e1);
        if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
            printf("{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", name);
            exit(1);
        }
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    // two steps per iteration, wps waves per SIMD each running ITERS iterations
    printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"ns_per_step_per_simd\": %.3f, \"ns_per_step_per_wave\": %.3f, "
           "\"ms\": %.3f}\n", name, wps, best * 1e6 / (ITERS * 2.0 * wps), best * 1e6 / (ITERS * 2.0), best);
    fflush(stdout);
    hipFree(out);
}

int main() {
    for (int wps : {1, 2, 4}) {
        run<0>("dpp_both", wps);
        run<1>("conveyor_bpermute", wps);
        run<2>("both_bpermute", wps);
        run<3>("no_shift", wps);
    }
    return 0;
}
