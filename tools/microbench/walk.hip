// Microbenchmark: the fused kernel's memory structure without its arithmetic.
// One wave owns a column window of one image (3 planes) and walks a band of rows,
// loading each row of each plane PD rows ahead into a register ring and storing it
// back (a copy).  Reports GB/s for per-lane widths of 2/4/8/16 B and several PD, plus
// a plain float4 grid-stride copy as the ceiling, and VALU rates of v_fma_f32 vs
// v_pk_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, RB = 126;

template <typename T, int PD>
__global__ __launch_bounds__(256) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    constexpr int CPL = sizeof(T) / 2;              // columns per lane
    constexpr int WCOLS = 64 * CPL;
    const int nwin = W / WCOLS, nband = (H + RB - 1) / RB;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int win = wave % nwin;
    const int64_t rest = wave / nwin;
    const int band = rest % nband;
    const int64_t b = rest / nband;
    if (b >= B) return;
    const int r0 = band * RB, r1 = min(r0 + RB, H);
    const int64_t cs = (int64_t)H * W;
    const T* xb = reinterpret_cast<const T*>(x + b * C * cs + win * WCOLS) + lane;
    T* yb = reinterpret_cast<T*>(y + b * C * cs + win * WCOLS) + lane;
    const int rs = W / CPL;
    T ring[PD][C];
#pragma unroll
    for (int i = 0; i < PD; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) ring[i][c] = xb[c * (cs / CPL) + (int64_t)min(r0 + i, H - 1) * rs];
    for (int r = r0; r < r1; r += PD) {
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            if (r + i < r1) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    yb[c * (cs / CPL) + (int64_t)(r + i) * rs] = ring[i][c];
                    ring[i][c] = xb[c * (cs / CPL) + (int64_t)min(r + i + PD, H - 1) * rs];
                }
            }
        }
    }
}

__global__ void copy4(const float4* __restrict__ x, float4* __restrict__ y, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = x[i];
}

typedef float f2 __attribute__((ext_vector_type(2)));
template <bool PK>
__global__ void valu(float* out, int iters, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a[8]; f2 p[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; p[i] = f2{a[i], a[i] + 1}; }
    const float m = 0.999f; const f2 m2 = {m, m};
    for (int k = 0; k < iters; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (PK) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(p[(i + 1) & 7]), "v"(m2));
            else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(m));
        }
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += PK ? p[i].x + p[i].y : a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <typename K>
float timeit(K k, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    k(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) k();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <typename T, int PD>
void run_walk(const uint16_t* x, uint16_t* y, int B) {
    constexpr int CPL = sizeof(T) / 2;
    const int64_t waves = (int64_t)B * ((H + RB - 1) / RB) * (W / (64 * CPL));
    const int blocks = (int)((waves + 3) / 4);
    float ms = timeit([&] { hipLaunchKernelGGL((walk<T, PD>), dim3(blocks), dim3(256), 0, 0, x, y, B); }, 5);
    const double bytes = 2.0 * B * C * H * W * 2;
    printf("walk %2dB/lane PD=%d: %.3f ms  %.0f GB/s\n", (int)sizeof(T), PD, ms, bytes / ms / 1e6);
}

int main(int argc, char** argv) {
    const bool only_valu = argc > 1;
    const int B = 128;
    const size_t n = (size_t)B * C * H * W;
    uint16_t *x, *y;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&y, n * 2));
    CK(hipMemset(x, 0x3c, n * 2)); CK(hipMemset(y, 0, n * 2));
    if (!only_valu) {
    float ms = timeit([&] { hipLaunchKernelGGL(copy4, dim3(256 * 64), dim3(256), 0, 0, (const float4*)x, (float4*)y, (int64_t)(n * 2 / 16)); }, 5);
    printf("copy float4: %.3f ms  %.0f GB/s\n", ms, 2.0 * n * 2 / ms / 1e6);
    run_walk<uint16_t, 2>(x, y, B); run_walk<uint16_t, 4>(x, y, B); run_walk<uint16_t, 8>(x, y, B);
    run_walk<uint32_t, 2>(x, y, B); run_walk<uint32_t, 4>(x, y, B); run_walk<uint32_t, 8>(x, y, B);
    run_walk<uint2, 2>(x, y, B); run_walk<uint2, 4>(x, y, B); run_walk<uint2, 8>(x, y, B);
    run_walk<uint4, 2>(x, y, B); run_walk<uint4, 4>(x, y, B);
    }
    float* o; CK(hipMalloc(&o, (size_t)1024 * 8 * 256 * 4));
    const int iters = 4096;
    unsigned long long* clk; CK(hipMalloc(&clk, 1024 * 8 * 16));
    std::vector<unsigned long long> hc(1024 * 8 * 2);
    for (int pk = 0; pk < 2; ++pk) {
        float t = timeit([&] {
            if (pk) hipLaunchKernelGGL(valu<true>, dim3(1024 * 8), dim3(256), 0, 0, o, iters, clk);
            else hipLaunchKernelGGL(valu<false>, dim3(1024 * 8), dim3(256), 0, 0, o, iters, clk);
        }, 3);
        const double fl = 2.0 * 8 * iters * 1024.0 * 8 * 256 * (pk ? 2 : 1);
        CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
        double cy = 0, rt = 0; for (int i = 0; i < 1024 * 8; ++i) { cy += hc[2 * i]; rt += hc[2 * i + 1]; }
        const double ghz = cy / rt * 0.1;
        // per SIMD: 8192 blocks * 4 waves / 1024 SIMDs = 32 waves, each 8*iters instructions
        const double cyc_per_instr = t * 1e-3 * ghz * 1e9 / (32.0 * 8 * iters);
        printf("valu %s: %.3f ms  %.1f TFLOP/s  clock %.2f GHz  %.2f cycles/wave-instr/SIMD\n", pk ? "v_pk_fma_f32" : "v_fma_f32", t, fl / t / 1e9, ghz, cyc_per_instr);
    }
    return 0;
}
