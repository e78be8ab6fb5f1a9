// Microbenchmark (round 4, re-entry): the fused kernel's register-ring band walk with 4
// columns per lane (dwordx2 loads and stores, 256-column windows owning 240 + 8 + 8 halo)
// against today's 2 columns per lane (dword, 128-column windows owning 120 + 4 + 4).
// Same geometry as walk4 (4K bf16, 3 planes, B = 128, 4 windows per workgroup, XCD-swizzled
// group-fastest order): every row of every plane loaded once per window (+ 4 halo rows per
// band), the owned columns stored once.  No arithmetic.
//   CPL 2: dword per lane, OWN 120, HL 4;  CPL 4: dwordx2 per lane, OWN 240, HL 8
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3;

__device__ __forceinline__ unsigned xcd_swz(unsigned bid, unsigned nwg) {
    const unsigned q = nwg >> 3, r = nwg & 7u, x = bid & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

template <int CPL> struct Cw { using T = unsigned; };
template <> struct Cw<4> { typedef unsigned T __attribute__((ext_vector_type(2))); };

template <int CPL, int RB, int PD, int GW>
__global__ __launch_bounds__(64 * GW) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    constexpr int OWN = CPL == 2 ? 120 : 240, HL = CPL == 2 ? 4 : 8;
    constexpr int NWIN = (W + OWN - 1) / OWN, NGRP = (NWIN + GW - 1) / GW;
    constexpr int NB = (H + RB - 1) / RB;
    using T = typename Cw<CPL>::T;
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned bid = xcd_swz(blockIdx.x, gridDim.x);
    const int grp = bid % NGRP;
    const unsigned r_ = bid / NGRP;
    const int band = r_ % NB;
    const int64_t b = r_ / NB;
    if (b >= B) return;
    const int win = grp * GW + wslot;
    const int W0 = win * OWN - HL;
    const int ce = W0 + CPL * lane;
    const int s0 = band * RB, s1 = min(s0 + RB, H);
    const int64_t cs = (int64_t)H * W;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(y + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const unsigned xplane = (unsigned)(cs * 2), xrow = W * 2;
    const int lc = min(max(ce, 0), W - CPL);
    const unsigned xoff = (unsigned)lc * 2;
    const bool own = win < NWIN && lane >= HL / CPL && lane < (HL + OWN) / CPL && ce >= 0 && ce < W;
    const unsigned yoff = own ? (unsigned)ce * 2 : 0x80000000u;
    auto roff = [&](int r) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(r, 0), H - 1) * xrow)); };
    auto ld = [&](unsigned so) -> T {
        if constexpr (CPL == 2) return __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, so, 0);
        else return __builtin_amdgcn_raw_buffer_load_b64(xr, xoff, so, 0);
    };
    auto st = [&](T v, unsigned so) {
        if constexpr (CPL == 2) __builtin_amdgcn_raw_buffer_store_b32(v, yr, yoff, so, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(v, yr, yoff, so, 0);
    };
    T acc = {};
    T ring[PD + 1][C];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        const unsigned so = roff(s0 - 2 + i);
#pragma unroll
        for (int c = 0; c < C; ++c) ring[i][c] = ld(so + c * xplane);
    }
    int r = s0 - 2;
    for (; r + PD + 1 <= s1 + 2; r += PD + 1) {
#pragma unroll
        for (int i = 0; i <= PD; ++i) {
            const unsigned so = roff(r + i + PD);
#pragma unroll
            for (int c = 0; c < C; ++c) ring[(i + PD) % (PD + 1)][c] = ld(so + c * xplane);
            if (r + i >= s0 && r + i < s1) {
                const unsigned sw = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(r + i) * xrow));
#pragma unroll
                for (int c = 0; c < C; ++c) { acc += ring[i][c]; st(ring[i][c] + 1u, sw + c * xplane); }
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) acc += ring[i][c];
            }
        }
    }
    for (; r < s1 + 2; ++r) {
        const unsigned so = roff(r);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const T v = ld(so + c * xplane);
            if (r >= s0 && r < s1) st(v + 1u, (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)r * xrow)) + c * xplane);
        }
    }
    unsigned a;
    if constexpr (CPL == 2) a = acc; else a = acc.x ^ acc.y;
    if (a == 0x12345678u) y[0] = 1;   // keep the loads
}

template <typename K>
float timeit(K k, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) k();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(e0)); k(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

static const double GB = 2.0 * 128 * C * H * W * 2 / 1e9;
template <int CPL, int RB, int PD, int GW = 4>
void run(const uint16_t* x, uint16_t* y, int B) {
    constexpr int OWN = CPL == 2 ? 120 : 240;
    constexpr int NWIN = (W + OWN - 1) / OWN, NGRP = (NWIN + GW - 1) / GW;
    const int blocks = NGRP * ((H + RB - 1) / RB) * B;
    const float ms = timeit([&] { hipLaunchKernelGGL((walk<CPL, RB, PD, GW>), dim3(blocks), dim3(64 * GW), 0, 0, x, y, B); }, 9);
    printf("cols/lane %d  RB %3d  PD %d  GW %d : %.3f ms  %.3f of 8 TB/s\n", CPL, RB, PD, GW, ms, GB / ms * 1e3 / 8000);
    fflush(stdout);
}

typedef float f4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy1(const f4v* __restrict__ x, f4v* __restrict__ y, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = x[i];
}

int main() {
    const int B = 128;
    const size_t n = (size_t)B * C * H * W;
    uint16_t *x, *y;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&y, n * 2));
    CK(hipMemset(x, 0x3c, n * 2)); CK(hipMemset(y, 0, n * 2));
    const int64_t n16 = (int64_t)(n * 2 / 16);
    const float mc = timeit([&] { hipLaunchKernelGGL(copy1, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, (const f4v*)x, (f4v*)y, n16); }, 9);
    printf("%-44s %.3f ms  %.3f of 8 TB/s\n", "one-shot float4 copy (ceiling)", mc, GB / mc * 1e3 / 8000);
    for (int rep = 0; rep < 2; ++rep) {
        run<2, 42, 3>(x, y, B);
        run<4, 42, 3>(x, y, B);
        run<4, 42, 2>(x, y, B);
        run<4, 24, 3>(x, y, B);
        run<4, 18, 3>(x, y, B);
        run<4, 66, 3>(x, y, B);
        run<2, 18, 3>(x, y, B);
        run<4, 42, 3, 2>(x, y, B);
        run<4, 42, 3, 8>(x, y, B);
    }
    return 0;
}
