// Microbenchmark: does the VGPR bank (register index mod 4) of the three operands of
// v_fmac_f32 change its issue cost on gfx950?  8 independent accumulators per wave in fixed
// registers (inline asm with explicit register names), 1..8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 banks.hip -o banks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// accumulators v8..v15 (banks 0..3,0..3); sources v16..v63
#define INIT asm volatile( \
    "v_mov_b32 v8, 1.0\n v_mov_b32 v9, 1.0\n v_mov_b32 v10, 1.0\n v_mov_b32 v11, 1.0\n" \
    "v_mov_b32 v12, 1.0\n v_mov_b32 v13, 1.0\n v_mov_b32 v14, 1.0\n v_mov_b32 v15, 1.0\n" \
    "v_mov_b32 v16, 0.5\n v_mov_b32 v17, 0.5\n v_mov_b32 v18, 0.5\n v_mov_b32 v19, 0.5\n" \
    "v_mov_b32 v20, 0.5\n v_mov_b32 v21, 0.5\n v_mov_b32 v22, 0.5\n v_mov_b32 v23, 0.5\n" \
    "v_mov_b32 v24, 0.5\n v_mov_b32 v25, 0.5\n v_mov_b32 v26, 0.5\n v_mov_b32 v27, 0.5\n" \
    "v_mov_b32 v28, 0.5\n v_mov_b32 v29, 0.5\n v_mov_b32 v30, 0.5\n v_mov_b32 v31, 0.5\n" \
    ::: "v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21", \
        "v22","v23","v24","v25","v26","v27","v28","v29","v30","v31")
#define CLOB "v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21", \
             "v22","v23","v24","v25","v26","v27","v28","v29","v30","v31"

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    INIT;
    for (int it = 0; it < iters; ++it) {
        // dst bank d, src0 bank a, src1 bank b
        if (MODE == 0)   // all different: dst d, src0 d+1, src1 d+2
            asm volatile("v_fmac_f32 v8, v17, v18\n v_fmac_f32 v9, v18, v19\n v_fmac_f32 v10, v19, v20\n v_fmac_f32 v11, v20, v21\n"
                         "v_fmac_f32 v12, v21, v22\n v_fmac_f32 v13, v22, v23\n v_fmac_f32 v14, v23, v24\n v_fmac_f32 v15, v24, v25\n" ::: CLOB);
        if (MODE == 1)   // src0 and src1 in one bank, dst another
            asm volatile("v_fmac_f32 v8, v17, v21\n v_fmac_f32 v9, v18, v22\n v_fmac_f32 v10, v19, v23\n v_fmac_f32 v11, v20, v24\n"
                         "v_fmac_f32 v12, v21, v25\n v_fmac_f32 v13, v22, v26\n v_fmac_f32 v14, v23, v27\n v_fmac_f32 v15, v24, v28\n" ::: CLOB);
        if (MODE == 2)   // src1 and dst in one bank
            asm volatile("v_fmac_f32 v8, v17, v16\n v_fmac_f32 v9, v18, v17\n v_fmac_f32 v10, v19, v18\n v_fmac_f32 v11, v20, v19\n"
                         "v_fmac_f32 v12, v21, v20\n v_fmac_f32 v13, v22, v21\n v_fmac_f32 v14, v23, v22\n v_fmac_f32 v15, v24, v23\n" ::: CLOB);
        if (MODE == 3)   // src0 and dst in one bank
            asm volatile("v_fmac_f32 v8, v16, v17\n v_fmac_f32 v9, v17, v18\n v_fmac_f32 v10, v18, v19\n v_fmac_f32 v11, v19, v20\n"
                         "v_fmac_f32 v12, v20, v21\n v_fmac_f32 v13, v21, v22\n v_fmac_f32 v14, v22, v23\n v_fmac_f32 v15, v23, v24\n" ::: CLOB);
        if (MODE == 4)   // all three in one bank
            asm volatile("v_fmac_f32 v8, v16, v20\n v_fmac_f32 v9, v17, v21\n v_fmac_f32 v10, v18, v22\n v_fmac_f32 v11, v19, v23\n"
                         "v_fmac_f32 v12, v24, v28\n v_fmac_f32 v13, v25, v29\n v_fmac_f32 v14, v26, v30\n v_fmac_f32 v15, v27, v31\n" ::: CLOB);
        if (MODE == 5)   // one shared src0 register (a broadcast weight), src1 / dst all different banks
            asm volatile("v_fmac_f32 v8, v16, v18\n v_fmac_f32 v9, v16, v19\n v_fmac_f32 v10, v16, v21\n v_fmac_f32 v11, v16, v22\n"
                         "v_fmac_f32 v12, v16, v18\n v_fmac_f32 v13, v16, v19\n v_fmac_f32 v14, v16, v21\n v_fmac_f32 v15, v16, v22\n" ::: CLOB);
        if (MODE == 6)   // VOP3 v_fma_f32 with a distinct dst: all different banks
            asm volatile("v_fma_f32 v8, v17, v18, v8\n v_fma_f32 v9, v18, v19, v9\n v_fma_f32 v10, v19, v20, v10\n v_fma_f32 v11, v20, v21, v11\n"
                         "v_fma_f32 v12, v21, v22, v12\n v_fma_f32 v13, v22, v23, v13\n v_fma_f32 v14, v23, v24, v14\n v_fma_f32 v15, v24, v25, v15\n" ::: CLOB);
        if (MODE == 7)   // v_pk_fma_f32 on pairs, all different banks: 4 instructions = 8 FMAs
            asm volatile("v_pk_fma_f32 v[8:9], v[18:19], v[20:21], v[8:9]\n v_pk_fma_f32 v[10:11], v[20:21], v[22:23], v[10:11]\n"
                         "v_pk_fma_f32 v[12:13], v[22:23], v[24:25], v[12:13]\n v_pk_fma_f32 v[14:15], v[24:25], v[26:27], v[14:15]\n" ::: CLOB);
        if (MODE == 8)   // v_pk_fma_f32 with a broadcast src0 (op_sel_hi:[0,1,1])
            asm volatile("v_pk_fma_f32 v[8:9], v[16:17], v[20:21], v[8:9] op_sel_hi:[0,1,1]\n v_pk_fma_f32 v[10:11], v[16:17], v[22:23], v[10:11] op_sel_hi:[0,1,1]\n"
                         "v_pk_fma_f32 v[12:13], v[16:17], v[24:25], v[12:13] op_sel_hi:[0,1,1]\n v_pk_fma_f32 v[14:15], v[16:17], v[26:27], v[14:15] op_sel_hi:[0,1,1]\n" ::: CLOB);
    }
    float s;
    asm volatile("v_add_f32 %0, v8, v15" : "=v"(s) :: CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int MODE>
void run(const char* name, float* o, unsigned long long* clk, int wps, int ninstr) {
    const int blocks = 256 * wps, iters = 2048;   // wps waves per SIMD (4 waves per block)
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, clk);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc(2 * blocks);
    CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
    double cy = 0, rt = 0; for (int i = 0; i < blocks; ++i) { cy += hc[2 * i]; rt += hc[2 * i + 1]; }
    const double ghz = cy / rt * 0.1;
    printf("%-36s wps %d  %.3f ms  %.2f GHz  %.2f cycles/wave-instr/SIMD\n", name, wps, ms, ghz,
           ms * 1e-3 * ghz * 1e9 / ((double)wps * ninstr * iters));
}

int main() {
    float* o; unsigned long long* clk;
    CK(hipMalloc(&o, (size_t)1024 * 8 * 256 * 4)); CK(hipMalloc(&clk, (size_t)1024 * 8 * 16));
    for (int w : {1, 2, 3, 4, 8}) {
        run<0>("fmac banks all different", o, clk, w, 8);
        run<1>("fmac src0==src1 bank", o, clk, w, 8);
        run<2>("fmac src1==dst bank", o, clk, w, 8);
        run<3>("fmac src0==dst bank", o, clk, w, 8);
        run<4>("fmac all one bank", o, clk, w, 8);
        run<5>("fmac shared src0 reg", o, clk, w, 8);
        run<6>("v_fma_f32 (VOP3) all different", o, clk, w, 8);
        run<7>("v_pk_fma_f32 all different", o, clk, w, 4);
        run<8>("v_pk_fma_f32 broadcast src0", o, clk, w, 4);
    }
    return 0;
}
