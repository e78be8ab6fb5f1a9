// Microbenchmark + layout probe for v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4x1, f32 in):
// the candidate engine for the 7-tap hex stencil with O <= 4 output channels (one output
// column per lane, the output channels in the 4 accumulator registers).
//   1. layout: which lane's A and which lane's B feed D[reg v] of lane l (asymmetric probe)
//   2. rates from kernel wall time: MFMA-only, VALU-only, both in one wave, and MFMA-only
//      waves beside VALU-only waves on the same SIMD
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// A is 1 in lane `la` only, B = 1 + lane: D[v](lane l) != 0 tells where A(la) lands and the
// value names the B lane.
__global__ void k_layout(float* out, int la) {
    const int l = threadIdx.x;
    const float a = (l == la) ? 1.f : 0.f, b = (float)(l + 1);
    f4 c = {0.f, 0.f, 0.f, 0.f};
    f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out[l * 4 + v] = d[v];
}

// NM MFMAs (0/1) and NF fmacs per slot, 8 slots per iteration; SPLIT: even waves run only
// the MFMAs, odd waves only the fmacs (two waves per SIMD pair up on one SIMD).
template <int NM, int NF, int SPLIT>
__global__ __launch_bounds__(256) void k_rate(float* out, int iters, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a = threadIdx.x * 1e-3f, b = 0.999f;
    asm volatile("" : "+v"(a), "+v"(b));
    f4 acc[8];
    float v[32];
    for (int i = 0; i < 8; ++i) acc[i] = f4{a, a + 1, a + 2, a + i};
    for (int i = 0; i < 32; ++i) v[i] = a + i;
    float m = 0.5f;
    asm volatile("" : "+v"(m));
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool do_m = NM > 0 && (!SPLIT || (wid & 1) == 0);
    const bool do_f = NF > 0 && (!SPLIT || (wid & 1) == 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // inline asm keeps each accumulator in place (the builtin form made hipcc rotate
            // accumulators through v_accvgpr_mov copies); an accumulator is re-read 8 MFMAs later
            if (do_m) asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
#pragma unroll
            for (int f = 0; f < NF; ++f)   // chains 8 apart: every source written >= 3 fmacs earlier
                if (do_f) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[(8 * f + i) & 31]) : "v"(v[(8 * f + i + 20) & 31]), "v"(m));
        }
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 32; ++i) s += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int NM, int NF, int SPLIT>
void run(const char* name, float* o, unsigned long long* clk, int wps) {
    const int mf = NM, vf = NF;
    const int blocks = 256 * wps, iters = 8192;   // 256 CUs x wps blocks of 4 waves
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_rate<NM, NF, SPLIT>), dim3(blocks), dim3(256), 0, 0, o, 64, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_rate<NM, NF, SPLIT>), dim3(blocks), dim3(256), 0, 0, o, iters, clk);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> hc(2 * blocks);
    CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
    double cy = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) { cy += hc[2 * i]; rt += hc[2 * i + 1]; }
    const double ghz = cy / rt * 0.1;
    const double simd_cycles = ms * 1e-3 * ghz * 1e9;            // wall cycles (every SIMD busy)
    const double per_simd_iters = (double)iters * wps;           // iterations per SIMD
    printf("%-40s wps %d  %.3f ms  %.2f GHz  per SIMD per iter(8 slots): %.1f cyc  "
           "= %.2f cyc/MFMA-slot  (%d MFMA + %d fmac per slot)\n",
           name, wps, ms, ghz, simd_cycles / per_simd_iters, simd_cycles / per_simd_iters / 8, mf, vf);
}

int main() {
    float* o; unsigned long long* clk;
    CK(hipMalloc(&o, (size_t)1024 * 8 * 256 * 4)); CK(hipMalloc(&clk, (size_t)1024 * 8 * 16));
    float* lo;
    CK(hipMalloc(&lo, 64 * 4 * 4));
    std::vector<float> h(256);
    int ok = 1;
    for (int la = 0; la < 64; ++la) {
        hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, lo, la);
        CK(hipMemcpy(h.data(), lo, 256 * 4, hipMemcpyDeviceToHost));
        for (int l = 0; l < 64; ++l)
            for (int v = 0; v < 4; ++v) {
                const float val = h[l * 4 + v];
                // hypothesis: D[v](lane l) = A(lane 4*(l/4) + v) * B(lane l)
                const bool hit = (4 * (l / 4) + v == la);
                const float want = hit ? (float)(l + 1) : 0.f;
                if (val != want) ok = 0;
                if (la == 5 && val != 0.f) printf("A lane 5 -> lane %d reg %d, B lane %d\n", l, v, (int)val - 1);
            }
    }
    printf("layout hypothesis D[v](lane l) = A(lane 4*(l/4)+v) * B(lane l): %s\n", ok ? "HOLDS" : "FAILS");
    for (int w : {1, 2, 4}) {
        run<1, 0, 0>("mfma only", o, clk, w);
        run<0, 1, 0>("fmac only, 1/slot", o, clk, w);
        run<0, 2, 0>("fmac only, 2/slot", o, clk, w);
        run<1, 1, 0>("mfma + 1 fmac, same wave", o, clk, w);
        run<1, 2, 0>("mfma + 2 fmac, same wave", o, clk, w);
        run<1, 3, 0>("mfma + 3 fmac, same wave", o, clk, w);
        run<1, 4, 0>("mfma + 4 fmac, same wave", o, clk, w);
        run<1, 2, 1>("mfma waves beside 2-fmac waves", o, clk, w);
        run<1, 4, 1>("mfma waves beside 4-fmac waves", o, clk, w);
    }
    return 0;
}
