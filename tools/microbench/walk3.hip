// Microbenchmark: the fused kernel's band-walk memory pattern (one wave = 128-column window,
// dword per lane, 3 bf16 planes, rows PD ahead, a store per row and plane), no arithmetic,
// for band lengths RB and three block -> (window, band, image) orders, to see whether the
// set of rows the resident waves touch at one time (DRAM locality) moves the ceiling.
//   ORDER 0: window fastest, then band, then image (the fused kernel's order)
//   ORDER 1: band fastest, then window, then image
//   ORDER 2: image fastest, then window, then band
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, NWIN = W / 128;

template <int RB, int ORDER, int PD>
__global__ __launch_bounds__(256) void walk(const uint32_t* __restrict__ x, uint32_t* __restrict__ y, int B) {
    const int nband = (H + RB - 1) / RB;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    int win, band;
    int64_t b;
    if (ORDER == 0) { win = wave % NWIN; const int64_t r = wave / NWIN; band = r % nband; b = r / nband; }
    else if (ORDER == 1) { band = wave % nband; const int64_t r = wave / nband; win = r % NWIN; b = r / NWIN; }
    else { b = wave % B; const int64_t r = wave / B; win = r % NWIN; band = (int)(r / NWIN); }
    if (b >= B || band >= nband) return;
    const int r0 = band * RB, r1 = min(r0 + RB, H);
    const int64_t cs = (int64_t)H * W / 2;          // plane stride in dwords
    const uint32_t* xb = x + b * C * cs + win * 64 + lane;
    uint32_t* yb = y + b * C * cs + win * 64 + lane;
    const int rs = W / 2;
    uint32_t ring[PD][C];
#pragma unroll
    for (int i = 0; i < PD; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) ring[i][c] = xb[c * cs + (int64_t)min(r0 + i, H - 1) * rs];
    for (int r = r0; r < r1; r += PD) {
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            if (r + i < r1) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    yb[c * cs + (int64_t)(r + i) * rs] = ring[i][c];
                    ring[i][c] = xb[c * cs + (int64_t)min(r + i + PD, H - 1) * rs];
                }
            }
        }
    }
}

template <typename K>
float timeit(K k, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) k();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) k();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int RB, int ORDER>
void run(const uint32_t* x, uint32_t* y, int B) {
    const int64_t waves = (int64_t)B * ((H + RB - 1) / RB) * NWIN;
    const int blocks = (int)((waves + 3) / 4);
    const float ms = timeit([&] { hipLaunchKernelGGL((walk<RB, ORDER, 3>), dim3(blocks), dim3(256), 0, 0, x, y, B); }, 8);
    const double gb = 2.0 * B * C * H * W * 2 / 1e9;
    printf("walk RB=%3d order %d: %.3f ms  %.0f GB/s  %.3f of 8 TB/s\n", RB, ORDER, ms, gb / ms * 1e3, gb / ms * 1e3 / 8000);
}

int main() {
    const int B = 128;
    const size_t n = (size_t)B * C * H * W / 2;
    uint32_t *x, *y;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
    CK(hipMemset(x, 0x3c, n * 4)); CK(hipMemset(y, 0, n * 4));
    run<42, 0>(x, y, B); run<42, 1>(x, y, B); run<42, 2>(x, y, B);
    run<126, 0>(x, y, B); run<126, 1>(x, y, B); run<126, 2>(x, y, B);
    run<12, 0>(x, y, B); run<12, 2>(x, y, B);
    run<2160, 2>(x, y, B);
    return 0;
}
