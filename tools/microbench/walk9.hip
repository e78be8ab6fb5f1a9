// Microbenchmark (round 6, the round-5 verdict's item 1c): the headline's band walk (walk8's
// REV 1 pattern: 4 windows of 256 columns per workgroup, dwordx2 row loads one row ahead, odd
// bands upwards, 30-row bands, 4K bf16 b128) with the output rows stored by a DIFFERENT wave,
// so the loading waves' vmcnt queue holds loads only:
//
//   SPLIT 0  every wave stores its own 240 owned columns (the kernel today; = walk8 REV 1);
//   SPLIT 1  the 4 loading waves write each output row (3 planes x 240 columns) into an LDS ring
//            of ROWS rows and add 1 to the slot's monotonic `ready` count (ds_add); a 5th wave per
//            workgroup waits until a slot holds all 4 contributions of its row (polling, s_sleep),
//            stores the group's 960 owned columns of each plane as 16-B lanes (whole 128-B
//            lines), and advances the slot's `freed` generation; a loading wave waits for the
//            slot's previous row to be freed before writing the next one into it.  Fences are
//            workgroup scope (LDS only).
//
// No arithmetic: the gate for porting a store wave into k_fused4 is this pattern reaching
// >= 0.72 of 8 TB/s on the headline's 12.74 GB.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3;
constexpr int OWN = 240, HL = 8, GW = 4, RB = 30;
constexpr int NWIN = (W + OWN - 1) / OWN, NGRP = (NWIN + GW - 1) / GW, NB = (H + RB - 1) / RB;

__device__ __forceinline__ unsigned xcd_swz(unsigned bid, unsigned nwg) {
    const unsigned q = nwg >> 3, r = nwg & 7u, x = bid & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// ring: ROWS slots x C planes x GW * OWN columns (bf16) + one counter per slot
template <int SPLIT, int ROWS>
__global__ __launch_bounds__(64 * (GW + SPLIT)) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    constexpr int SLOTB = C * GW * OWN * 2;                  // 5760 B
    __shared__ __attribute__((aligned(16))) unsigned char ring[SPLIT ? ROWS * SLOTB : 16];
    __shared__ int ready[SPLIT ? ROWS : 1], freed[SPLIT ? ROWS : 1];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned bid = xcd_swz(blockIdx.x, gridDim.x);
    const int grp = bid % NGRP;
    const unsigned r_ = bid / NGRP;
    const int band = r_ % NB;
    const int64_t b = r_ / NB;
    if (b >= B) return;
    const int s0 = band * RB, s1 = min(s0 + RB, H);
    const int n = s1 - s0;
    const bool up = (band & 1) && n == RB;
    auto orow = [&](int k) { return up ? s1 - 1 - k : s0 + k; };
    const int64_t cs = (int64_t)H * W;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(y + b * C * cs), (short)0, (int)(C * cs * 2), 0x00020000);
    const unsigned xplane = (unsigned)(cs * 2), xrow = W * 2;
    if (SPLIT) {
        for (int i = threadIdx.x; i < ROWS; i += blockDim.x) ready[i] = freed[i] = 0;
        __syncthreads();
    }
    if (SPLIT && wslot == GW) {
        // ---- the store wave: slot k % ROWS holds output row k once GW waves have added 1 ----
        const int gc0 = grp * GW * OWN;                      // group's first owned column
        for (int k = 0; k < n; ++k) {
            const int sl = k % ROWS, gen = k / ROWS;
            while (__atomic_load_n(&ready[sl], __ATOMIC_RELAXED) < GW * (gen + 1)) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const unsigned so = (unsigned)orow(k) * xrow;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                // 960 columns = 1920 B = 120 lanes x 16 B: two passes of 64 lanes
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const int e = p * 64 + lane;             // 16-B piece of the plane row
                    const bool ok = e < 120 && gc0 + 8 * e < W;
                    const u4 v = *reinterpret_cast<const u4*>(ring + sl * SLOTB + c * GW * OWN * 2 + 16 * (e < 120 ? e : 0));
                    __builtin_amdgcn_raw_buffer_store_b128(v, yr, ok ? (unsigned)(gc0 + 8 * e) * 2 + so + c * xplane : 0x80000000u, 0, 0);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the ring reads are done
            if (lane == 0) __atomic_store_n(&freed[sl], gen + 1, __ATOMIC_RELAXED);
        }
        return;
    }
    const int win = grp * GW + wslot;
    const int W0 = win * OWN - HL;
    const int ce = W0 + 4 * lane;
    const int lc = min(max(ce, 0), W - 4);
    const unsigned xoff = (unsigned)lc * 2;
    const bool own = win < NWIN && lane >= HL / 4 && lane < (HL + OWN) / 4 && ce >= 0 && ce < W;
    const unsigned yoff = own ? (unsigned)ce * 2 : 0x80000000u;
    const int nk = n + 4;                                    // rows s0-2 .. s1+1
    auto row = [&](int k) { return up ? s1 + 1 - k : s0 - 2 + k; };
    auto roff = [&](int r) { return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(r, 0), H - 1) * xrow)); };
    auto ld = [&](unsigned so) -> u2 { return __builtin_amdgcn_raw_buffer_load_b64(xr, xoff, so, 0); };
    u2 acc = {};
    u2 ring0[C], ring1[C];
    {
        const unsigned so = roff(row(0));
#pragma unroll
        for (int c = 0; c < C; ++c) ring0[c] = ld(so + c * xplane);
    }
    for (int k = 0; k < nk; ++k) {
        const unsigned so = roff(row(k + 1));
        const bool live = k + 1 < nk;
#pragma unroll
        for (int c = 0; c < C; ++c) ring1[c] = __builtin_amdgcn_raw_buffer_load_b64(xr, live ? xoff : 0x80000000u, so + c * xplane, 0);
        const int ok_ = k - 2;                               // output row index of this step
        if (ok_ >= 0 && ok_ < n) {
            if constexpr (SPLIT) {
                const int sl = ok_ % ROWS, gen = ok_ / ROWS;
                if (gen > 0) {                               // the slot's previous row is stored
                    while (__atomic_load_n(&freed[sl], __ATOMIC_RELAXED) < gen) __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (own) {
#pragma unroll
                    for (int c = 0; c < C; ++c)
                        *reinterpret_cast<u2*>(ring + sl * SLOTB + c * GW * OWN * 2 + (wslot * OWN + 4 * lane - HL) * 2) = ring0[c] + 1u;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __atomic_fetch_add(&ready[sl], 1, __ATOMIC_RELAXED);
            } else {
                const unsigned sw = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)orow(ok_) * xrow));
#pragma unroll
                for (int c = 0; c < C; ++c) __builtin_amdgcn_raw_buffer_store_b64(ring0[c] + 1u, yr, yoff, sw + c * xplane, 0);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) { acc += ring0[c]; ring0[c] = ring1[c]; }
    }
    if ((acc.x ^ acc.y) == 0x12345678u) y[0] = 1;            // keep the loads
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

static const int B = 128;
static const double GB = 2.0 * B * C * H * W * 2 / 1e9;
template <int SPLIT, int ROWS>
void run(const uint16_t* x, uint16_t* y, int reps) {
    const int blocks = NGRP * NB * B;
    const float ms = timeit([&] { hipLaunchKernelGGL((walk<SPLIT, ROWS>), dim3(blocks), dim3(64 * (GW + SPLIT)), 0, 0, x, y, B); }, reps);
    printf("walk9 SPLIT %d ROWS %d : %.3f ms  %.3f of 8 TB/s\n", SPLIT, ROWS, ms, GB / ms * 1e3 / 8000);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 9;
    const size_t n = (size_t)B * C * H * W;
    uint16_t *x, *y;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&y, n * 2));
    CK(hipMemset(x, 0x3c, n * 2)); CK(hipMemset(y, 0, n * 2));
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 4>(x, y, reps);
        run<1, 2>(x, y, reps);
        run<1, 4>(x, y, reps);
        run<1, 6>(x, y, reps);
    }
    // correctness of the split store path: every owned output element = input + 1 (bf16 bits)
    CK(hipMemset(y, 0, n * 2));
    run<1, 4>(x, y, 1);
    std::vector<uint16_t> hy(W * 8);
    CK(hipMemcpy(hy.data(), y + (size_t)5 * C * H * W + (size_t)1 * H * W + (size_t)37 * W, W * 2, hipMemcpyDeviceToHost));
    int bad = 0;   // (each dword + 1: even elements 0x3c3d, odd ones 0x3c3c)
    for (int i = 0; i < W; ++i) bad += hy[i] != ((i & 1) ? 0x3c3c : 0x3c3d);
    printf("split-store check: %d of %d elements wrong\n", bad, W);
    CK(hipFree(x)); CK(hipFree(y));
    return bad ? 1 : 0;
}
