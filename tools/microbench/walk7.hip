// Microbenchmark (round 4): does batching a band walk's loads and stores into groups of NB rows
// (NB rows of loads issued together one block ahead, then NB rows of stores together) raise the
// HBM efficiency of the row-streaming kernels' access pattern?  Geometry of the headline
// (4K bf16, 3 planes, B = 128, 128-column windows owning 120, 4 windows per workgroup,
// XCD-swizzled group-fastest order, RB-row bands + 4 halo rows), no arithmetic.
//   NB = 1 with PD = 3 is walk4/walk6's register-ring pattern (the fused kernel's today).
//   ALT = 1: odd bands walk upwards (last row first), so a band and its upper neighbour read
//   their 2 shared halo rows together at the end / start of both walks (L2 hits?); ALT = 2:
//   every band walks upwards (control: same pattern, mirrored).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, OWN = 120, HL = 4;
constexpr int NWIN = (W + OWN - 1) / OWN, NGRP = NWIN / 4;

__device__ __forceinline__ unsigned xcd_swz(unsigned bid, unsigned nwg) {
    const unsigned q = nwg >> 3, r = nwg & 7u, x = bid & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// rows s0 - 2 .. s1 + 1 are read (the band + 4 halo rows), rows s0 .. s1 - 1 stored; blocks of NB
// rows: block k's loads are issued while block k - 1 is "processed" (stored)
template <int RB, int NB, int ALT = 0>
__global__ __launch_bounds__(256) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    constexpr int NBND = (H + RB - 1) / RB;
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned bid = xcd_swz(blockIdx.x, gridDim.x);
    const int grp = bid % NGRP;
    const unsigned r_ = bid / NGRP;
    const int band = r_ % NBND;
    const int64_t b = r_ / NBND;
    if (b >= B) return;
    const int win = grp * 4 + wslot;
    const int ce = win * OWN - HL + 2 * lane;
    const int s0 = band * RB, s1 = min(s0 + RB, H);
    const int64_t cs = (int64_t)H * W;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(y + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const unsigned xplane = (unsigned)(cs * 2), xrow = W * 2;
    const unsigned xoff = (unsigned)min(max(ce, 0), W - 2) * 2;
    const bool own = lane >= HL / 2 && lane < (HL + OWN) / 2 && ce >= 0 && ce < W;
    const unsigned yoff = own ? (unsigned)ce * 2 : 0x80000000u;
    auto roff = [&](int r) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(r, 0), H - 1) * xrow)); };
    unsigned acc = 0;
    unsigned cur[NB][C], nxt[NB][C];
    const int r0 = s0 - 2, r1 = s1 + 2;                  // rows read: r0 .. r1 - 1
    const bool up = ALT == 2 || (ALT == 1 && (band & 1));
    auto mrow = [&](int r) { return up ? r0 + r1 - 1 - r : r; };
    auto load_block = [&](int rb, unsigned (&d)[NB][C]) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const unsigned so = roff(mrow(rb + i));
#pragma unroll
            for (int c = 0; c < C; ++c) d[i][c] = __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, so + c * xplane, 0);
        }
    };
    load_block(r0, cur);
    for (int rb = r0; rb < r1; rb += NB) {
        if (rb + NB < r1) load_block(rb + NB, nxt);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int r = mrow(rb + i);
            const unsigned sw = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(r, 0), H - 1) * xrow));
            const bool st = r >= s0 && r < s1;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                acc += cur[i][c];
                __builtin_amdgcn_raw_buffer_store_b32(cur[i][c] + 1u, yr, st ? yoff : 0x80000000u, sw + c * xplane, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c) cur[i][c] = nxt[i][c];
    }
    if (acc == 0x12345678u) y[0] = 1;
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
template <int RB, int NB, int ALT = 0>
void run(const uint16_t* x, uint16_t* y, int B) {
    const int blocks = NGRP * ((H + RB - 1) / RB) * B;
    const float ms = timeit([&] { hipLaunchKernelGGL((walk<RB, NB, ALT>), dim3(blocks), dim3(256), 0, 0, x, y, B); }, 9);
    printf("RB %3d  rows per load/store batch %2d  %-12s: %.3f ms  %.3f of 8 TB/s\n", RB, NB,
           ALT == 0 ? "all down" : ALT == 1 ? "alternating" : "all up", ms, GB / ms * 1e3 / 8000);
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
        run<42, 1>(x, y, B);
        run<42, 1, 1>(x, y, B);
        run<42, 1, 2>(x, y, B);
        run<30, 1>(x, y, B);
        run<30, 1, 1>(x, y, B);
        run<18, 1>(x, y, B);
        run<18, 1, 1>(x, y, B);
        run<96, 1>(x, y, B);
        run<96, 1, 1>(x, y, B);
    }
    return 0;
}
