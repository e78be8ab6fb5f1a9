// Microbenchmark (round 3): issue cost of v_pk_fma_f32 with INDEPENDENT accumulators and a
// broadcast weight (op_sel_hi), against v_fmac_f32 doing the same number of FMAs, at 1..8
// waves per SIMD; plus a correctness probe of a v_mov_b32_dpp result read by the next
// v_pk_fma_f32 as one half of its 64-bit operand (the round-2 SLP miscompile pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, unsigned long long* clk, f2 ws, float wsf) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    f2 acc[8], u[4];
    float a[16];
    for (int i = 0; i < 8; ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, 0.5f * i};
    for (int i = 0; i < 4; ++i) u[i] = f2{1.0f + i * 1e-3f, 1.0f - i * 1e-3f};
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3f + i;
    f2 w = f2{0.999f, 0.5f};
    float wf = 0.999f, uf[8];
    for (int i = 0; i < 8; ++i) uf[i] = 1.0f + i * 1e-3f;
    asm volatile("" : "+v"(w), "+v"(wf));
    int baddr = ((threadIdx.x + 63) & 63) * 4;
    if (MODE == 6) for (int i = 0; i < 8; ++i) uf[i] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // 16 FMAs per i-pair in every mode below
            if (MODE == 0) {   // pk_fma, broadcast weight, 8 independent accumulators: 2 per i
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
            }
            if (MODE == 1) {   // fmac, 16 independent accumulators: 4 per i
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[2 * i]) : "v"(wf), "v"(uf[i]));
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[2 * i + 1]) : "v"(wf), "v"(uf[(i + 1) & 7]));
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[(2 * i + 8) & 15]) : "v"(wf), "v"(uf[(i + 2) & 7]));
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[(2 * i + 9) & 15]) : "v"(wf), "v"(uf[(i + 3) & 7]));
            }
            if (MODE == 2) {   // pk_fma with a full 64-bit weight pair (no op_sel)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
            }
            if (MODE == 4) {   // pk_fma, weight pair in SGPRs (broadcast lo)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "s"(ws), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc[(i + 4) & 7]) : "s"(ws), "v"(u[(i + 1) & 3]));
            }
            if (MODE == 5) {   // VOP3 v_fma_f32 with an SGPR weight, 16 indep acc
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[2 * i]) : "s"(wsf), "v"(uf[i]));
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[2 * i + 1]) : "s"(wsf), "v"(uf[(i + 1) & 7]));
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[(2 * i + 8) & 15]) : "s"(wsf), "v"(uf[(i + 2) & 7]));
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[(2 * i + 9) & 15]) : "s"(wsf), "v"(uf[(i + 3) & 7]));
            }
            if (MODE == 6) {   // 2 pk_fma + 1 ds_bpermute (LDS pipe) per i
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
                asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(uf[i]) : "v"(baddr), "v"(a[(i + 3) & 15]));
            }
            if (MODE == 7) {   // 2 pk_fma + 1 v_mov_b32 per i
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
                asm volatile("v_mov_b32 %0, %1" : "=v"(uf[i]) : "v"(a[(i + 3) & 15]));
            }
            if (MODE == 8) {   // 2 pk_fma + 1 v_mov_b32_dpp per i
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
                asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(uf[i]) : "v"(a[(i + 3) & 15]));
            }
            if (MODE == 9) {   // pk_mul_f32 (2 per i)
                asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
            }
            if (MODE == 10) {  // 2 pk_fma + 1 v_fmac_f32_dpp (the DPP folded into an FMA) per i
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
                asm volatile("v_fmac_f32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(uf[i]) : "v"(a[(i + 3) & 15]), "v"(wf));
            }
            if (MODE == 3) {   // mix: 2 pk_fma + 1 dpp mov + 1 fmac (the shape of a rewritten step)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "v"(w), "v"(u[i & 3]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[(i + 4) & 7]) : "v"(w), "v"(u[(i + 1) & 3]));
                asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(uf[i]) : "v"(a[(i + 3) & 15]));
                asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[2 * i]) : "v"(wf), "v"(uf[(i + 5) & 7]));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y + uf[i];
    for (int i = 0; i < 16; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// DPP -> pk_fma hazard probe: pair.x = lane value shifted by one lane (wave_shr), pair.y =
// own value, then immediately acc = fma(w, pair, acc).  NOPS s_nop wait states between.
template <int NOPS>
__global__ void hz(const float* in, float* out) {
    const int l = threadIdx.x;
    float v = in[l], o = in[64 + l];
    f2 p, acc = f2{0.f, 0.f}, w = f2{2.0f, 3.0f};
    asm volatile("" : "+v"(w));
    float px;
    asm volatile(
        "v_mov_b32 %1, %3\n"
        "v_mov_b32_dpp %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        ".if %5 > 0\n s_nop %5 - 1\n .endif\n"
        : "=&v"(px), "=&v"(p.y) : "v"(v), "v"(o), "v"(0), "n"(NOPS));
    p.x = px;
    acc = __builtin_elementwise_fma(w, p, acc);
    out[2 * l] = acc.x;
    out[2 * l + 1] = acc.y;
}

template <int MODE>
void run(const char* name, float* o, unsigned long long* clk, int wps) {
    const int blocks = 256 * wps, iters = 2048;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, clk, f2{0.999f, 0.5f}, 0.999f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, iters, clk, f2{0.999f, 0.5f}, 0.999f);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc(2 * blocks);
    CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
    double cy = 0, rt = 0; for (int i = 0; i < blocks; ++i) { cy += hc[2 * i]; rt += hc[2 * i + 1]; }
    const double ghz = cy / rt * 0.1;
    const int insts = (MODE == 1 || MODE == 3 || MODE == 5) ? 4 : ((MODE >= 6 && MODE <= 8) || MODE == 10 ? 3 : 2);
    const double cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-34s wps %d  %.3f ms  %.2f GHz  %.2f cyc/wave-instr  %.1f cyc per i-unit\n", name, wps,
           ms, ghz, cyc / ((double)wps * 8.0 * insts * iters), cyc / ((double)wps * 8.0 * iters));
}

template <int NOPS>
int hz_run(float* din, float* dout) {
    hipLaunchKernelGGL(hz<NOPS>, dim3(1), dim3(64), 0, 0, din, dout);
    CK(hipDeviceSynchronize());
    std::vector<float> in(128), out(128);
    CK(hipMemcpy(in.data(), din, 512, hipMemcpyDeviceToHost));
    CK(hipMemcpy(out.data(), dout, 512, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const float px = l ? in[l - 1] : 0.f, py = in[64 + l];
        if (out[2 * l] != 2.0f * px || out[2 * l + 1] != 3.0f * py) ++bad;
    }
    printf("dpp -> pk_fma, %d s_nop wait states: %d of 64 lanes wrong\n", NOPS, bad);
    return bad;
}

int main() {
    float* o; unsigned long long* clk;
    CK(hipMalloc(&o, (size_t)1024 * 8 * 256 * 4)); CK(hipMalloc(&clk, (size_t)1024 * 8 * 16));
    float *din, *dout;
    CK(hipMalloc(&din, 512)); CK(hipMalloc(&dout, 512));
    std::vector<float> hin(128);
    for (int i = 0; i < 128; ++i) hin[i] = 1.0f + 0.25f * i;
    CK(hipMemcpy(din, hin.data(), 512, hipMemcpyHostToDevice));
    hz_run<0>(din, dout);
    hz_run<1>(din, dout);
    hz_run<2>(din, dout);
    for (int w : {2, 3, 4, 5, 6, 8}) {
        run<0>("v_pk_fma_f32 bcast w, 8 indep acc", o, clk, w);
        run<2>("v_pk_fma_f32 pair w, 8 indep acc", o, clk, w);
        run<1>("v_fmac_f32, 16 indep acc", o, clk, w);
        run<3>("2 pk_fma + dpp mov + fmac", o, clk, w);
        run<4>("v_pk_fma_f32 SGPR w, 8 indep acc", o, clk, w);
        run<5>("v_fma_f32 SGPR w, 16 indep acc", o, clk, w);
        run<6>("2 pk_fma + ds_bpermute", o, clk, w);
        run<7>("2 pk_fma + v_mov_b32", o, clk, w);
        run<8>("2 pk_fma + v_mov_b32_dpp", o, clk, w);
        run<9>("v_pk_mul_f32", o, clk, w);
        run<10>("2 pk_fma + v_fmac_f32_dpp", o, clk, w);
    }
    return 0;
}
