// Microbenchmark: issue cost (cycles per wave-instruction per SIMD) of the VALU forms the
// fused kernel uses: plain v_fmac_f32, v_fmac_f32 with an SGPR operand, v_mov_b32_dpp
// wave_shr:1 / row_shr:1, v_mul_f32_dpp wave_shr:1.  8 waves per SIMD, 8 independent
// register chains per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, float sv, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    const float m = 0.999f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
            if (MODE == 1) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "s"(sv), "v"(a[(i + 1) & 7]));
            if (MODE == 2) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 3) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 4) asm volatile("v_mul_f32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(m));
            if (MODE == 5) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 7) asm volatile("v_dot2c_f32_f16 %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
            if (MODE == 8) asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
            if (MODE == 9) asm volatile("v_dot2c_f32_bf16 %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
            if (MODE == 10) asm volatile("v_pk_fma_f16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
            if (MODE == 11) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 5) & 7]));
            if (MODE == 12) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 13) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 14) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 15) asm volatile("v_lshlrev_b32 %0, 16, %1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 16) asm volatile("v_and_b32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 17) asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 18) asm volatile("v_fmac_f32 %0, 0.5, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
            if (MODE == 19) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*(double*)&a[(2 * i) & 7]) : "v"(*(double*)&a[(2 * i + 2) & 7]), "v"(*(double*)&a[(2 * i + 4) & 7]));
            if (MODE == 20) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]), "v"(m));
            if (MODE == 21) asm volatile("v_alignbyte_b32 %0, %1, %2, 2" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 22) asm volatile("v_lshlrev_b32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 23) asm volatile("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 24) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 25) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 26) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[(i + 4) & 7]));
            if (MODE == 27) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 28) asm volatile("v_max_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(a[(i + 2) & 7]));
            if (MODE == 29) asm volatile("v_cvt_f32_bf16 %0, %1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 30) asm volatile("v_cvt_f32_bf16_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
            if (MODE == 31) asm volatile("v_fmac_f32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(m));
            if (MODE == 32) { float t; asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(t) : "v"(a[(i + 3) & 7])); asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"(t), "v"(m)); }
            if (MODE == 6) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "s"(sv), "v"(a[(i + 1) & 7]));
        }
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int MODE>
void run(const char* name, float* o, unsigned long long* clk, int wps) {
    const int blocks = 256 * wps, iters = 2048;   // wps waves per SIMD (4 waves per block)
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, 0.5f, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, 0.5f, clk);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc(2 * blocks);
    CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
    double cy = 0, rt = 0; for (int i = 0; i < blocks; ++i) { cy += hc[2 * i]; rt += hc[2 * i + 1]; }
    const double ghz = cy / rt * 0.1;
    printf("%-30s wps %d  %.3f ms  %.2f GHz  %.2f cycles/wave-instr/SIMD\n", name, wps, ms, ghz,
           ms * 1e-3 * ghz * 1e9 / ((double)wps * 8.0 * iters));
}

int main() {
    float* o; unsigned long long* clk;
    CK(hipMalloc(&o, (size_t)1024 * 8 * 256 * 4)); CK(hipMalloc(&clk, (size_t)1024 * 8 * 16));
    for (int w : {1, 2, 3, 4, 8}) {
        run<0>("v_fmac_f32 v,v(m)", o, clk, w);
        run<12>("v_fmac_f32 v,v,v", o, clk, w);
        run<1>("v_fmac_f32 s,v", o, clk, w);
        run<2>("v_mov_b32_dpp wave_shr", o, clk, w);
        run<4>("v_mul_f32_dpp wave_shr", o, clk, w);
        run<31>("v_fmac_f32_dpp wave_shr", o, clk, w);
        run<32>("dpp mov then dependent fmac", o, clk, w);
        run<9>("v_dot2c_f32_bf16", o, clk, w);
        run<19>("v_pk_fma_f32", o, clk, w);
        run<11>("v_cvt_pk_bf16_f32", o, clk, w);
    }
    return 0;
}
