// Microbenchmark for the next headline design: the fused kernel's bytes (128 x 3 planes of
// 2160 x 3840 bf16 in, the same out) moved by SHORT-LIVED waves that each own a tile of T
// output rows x 128 columns (120 owned, as the fused kernel's windows) and load its T + HALO
// source rows of every plane up front (dword per lane, all loads before any store), then store
// the T owned rows.  HALO = 4 is the r2h + conv row halo the fused kernel needs; the halo rows
// are re-read by the neighbouring tiles (served by L2 when the tiles run close in time).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, OWN = 120, NWIN = (W + OWN - 1) / OWN;

template <int T, int HALO>
__global__ __launch_bounds__(256) void tile(const uint32_t* __restrict__ x, uint32_t* __restrict__ y, int B) {
    constexpr int NR = T + HALO;
    const int ntile = (H + T - 1) / T;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int win = wave % NWIN;
    const int64_t rest = wave / NWIN;
    const int tl = rest % ntile;
    const int64_t b = rest / ntile;
    if (b >= B) return;
    const int r0 = tl * T;
    const int col = min(max(win * OWN - 4 + 2 * lane, 0), W - 2);   // clamped, as the kernel
    const int64_t cs = (int64_t)H * W / 2;
    const uint32_t* xb = x + b * C * cs + col / 2;
    uint32_t* yb = y + b * C * cs + col / 2;
    const bool own = lane >= 2 && lane < 62 && win * OWN - 4 + 2 * lane < W;
    uint32_t v[NR][C];
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c)
            v[i][c] = xb[c * cs + (int64_t)min(max(r0 - 2 + i, 0), H - 1) * (W / 2)];
    uint32_t acc[T][C];
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c)            // every loaded row is used (a stand-in for the stencil)
            acc[i][c] = v[i][c] ^ v[i + 1][c] ^ v[i + 2][c] ^ v[i + 3][c] ^ v[i + 4][c];
    if (own) {
#pragma unroll
        for (int i = 0; i < T; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c)
                if (r0 + i < H) yb[c * cs + (int64_t)(r0 + i) * (W / 2)] = acc[i][c];
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

template <int T>
void run(const uint32_t* x, uint32_t* y, int B) {
    const int64_t waves = (int64_t)B * ((H + T - 1) / T) * NWIN;
    const int blocks = (int)((waves + 3) / 4);
    const float ms = timeit([&] { hipLaunchKernelGGL((tile<T, 4>), dim3(blocks), dim3(256), 0, 0, x, y, B); }, 8);
    const double gb = 2.0 * B * C * H * W * 2 / 1e9;   // the fused kernel's algorithmic bytes
    printf("tile T=%2d (+4 halo rows): %.3f ms  %.0f GB/s alg  %.3f of 8 TB/s\n", T, ms, gb / ms * 1e3, gb / ms * 1e3 / 8000);
}

int main() {
    const int B = 128;
    const size_t n = (size_t)B * C * H * W / 2;
    uint32_t *x, *y;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
    CK(hipMemset(x, 0x3c, n * 4)); CK(hipMemset(y, 0, n * 4));
    run<4>(x, y, B); run<8>(x, y, B); run<12>(x, y, B); run<16>(x, y, B); run<24>(x, y, B);
    return 0;
}
