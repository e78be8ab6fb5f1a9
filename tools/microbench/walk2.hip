// Microbenchmark: the fused kernel's exact memory pattern (one wave = 128-column window of
// 3 bf16 planes, 126-row band, dword buffer loads PD rows ahead, dword buffer stores),
// no arithmetic, for several cache-policy bits on loads and stores (gfx950 aux: bit0 sc0,
// bit1 nt, bit4 sc1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, RB = 126, PD = 3;

template <int LAUX, int SAUX, int OWN, int LAL = 0, int SAL = 0, int SWZ = 0>
__global__ __launch_bounds__(256) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    const int nwin = (W + OWN - 1) / OWN, nband = (H + RB - 1) / RB;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned bid = blockIdx.x;
    if (SWZ) { const unsigned nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7u, xx = bid & 7u;
               bid = (xx < rr ? xx * (q + 1) : rr * (q + 1) + (xx - rr) * q) + (bid >> 3); }
    const int64_t wave = (int64_t)bid * 4 + wslot;
    const int lane = threadIdx.x & 63;
    const int win = wave % nwin;
    const int64_t rest = wave / nwin;
    const int band = rest % nband;
    const int64_t b = rest / nband;
    if (b >= B) return;
    const int r0 = band * RB, r1 = min(r0 + RB, H);
    const int64_t cs = (int64_t)H * W;
    const int ce = win * OWN - (128 - OWN) / 2 + 2 * lane;
    const int lc = LAL ? min(win * 128 + 2 * lane, W - 2) : min(max(ce, 0), W - 2);
    const bool own = lane >= (128 - OWN) / 4 && lane < (128 + OWN) / 4 && ce >= 0 && ce < W;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(y + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    unsigned xo[C], yo[C];
    for (int c = 0; c < C; ++c) { xo[c] = (unsigned)((c * cs + lc) * 2); yo[c] = own ? (unsigned)((c * cs + ce) * 2) : 0x80000000u;
        if (SAL) yo[c] = (win * 128 + 2 * lane < W) ? (unsigned)((c * cs + win * 128 + 2 * lane) * 2) : 0x80000000u; }
    unsigned ring[PD + 1][C];
    auto ld = [&](int slot, int r) {
        const unsigned so = __builtin_amdgcn_readfirstlane(min(r, H - 1) * W * 2);
        for (int c = 0; c < C; ++c) ring[slot][c] = __builtin_amdgcn_raw_buffer_load_b32(xr, xo[c], so, LAUX);
    };
#pragma unroll
    for (int i = 0; i < PD; ++i) ld(i, r0 + i);
    __builtin_amdgcn_s_waitcnt(0x0f70);
    int r = r0;
    for (; r + PD + 1 <= r1; r += PD + 1) {
#pragma unroll
        for (int i = 0; i <= PD; ++i) {
            ld((i + PD) % (PD + 1), r + i + PD);
            const unsigned so = __builtin_amdgcn_readfirstlane((r + i) * W * 2);
#pragma unroll
            for (int c = 0; c < C; ++c) __builtin_amdgcn_raw_buffer_store_b32(ring[i][c] + 1u, yr, yo[c], so, SAUX);
        }
    }
    for (; r < r1; ++r) {
        const unsigned so = __builtin_amdgcn_readfirstlane(r * W * 2);
        for (int c = 0; c < C; ++c) __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_raw_buffer_load_b32(xr, xo[c], so, LAUX), yr, yo[c], so, SAUX);
    }
}

template <int LAUX, int SAUX, int OWN, int LAL = 0, int SAL = 0, int SWZ = 0>
void run(const char* name, const uint16_t* x, uint16_t* y, int B) {
    const int64_t waves = (int64_t)B * ((H + RB - 1) / RB) * ((W + OWN - 1) / OWN);
    const int blocks = (int)((waves + 3) / 4);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((walk<LAUX, SAUX, OWN, LAL, SAL, SWZ>), dim3(blocks), dim3(256), 0, 0, x, y, B);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((walk<LAUX, SAUX, OWN, LAL, SAL, SWZ>), dim3(blocks), dim3(256), 0, 0, x, y, B);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    const double bytes = 2.0 * B * C * H * W * 2;
    printf("%-34s %.3f ms  %.0f GB/s\n", name, ms, bytes / ms / 1e6);
}

int main() {
    const int B = 128;
    const size_t n = (size_t)B * C * H * W;
    uint16_t *x, *y;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&y, n * 2));
    CK(hipMemset(x, 0x3c, n * 2)); CK(hipMemset(y, 0, n * 2));
    run<0, 0, 120, 0, 0, 1>("own 120 + swz", x, y, B);
    run<0, 0, 124, 0, 0, 1>("own 124 + swz", x, y, B);
    run<0, 0, 112, 0, 0, 1>("own 112 (32B-aligned) + swz", x, y, B);
    run<0, 0, 96, 0, 0, 1>("own 96 (64B-aligned) + swz", x, y, B);
    run<0, 0, 64, 0, 0, 1>("own 64 (128B-aligned) + swz", x, y, B);
    run<0, 0, 128, 0, 0, 1>("own 128 + swz", x, y, B);
    return 0;
}
