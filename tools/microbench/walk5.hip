// Microbenchmark (round 4, after walk4): the fused kernel's band walk with workgroup-wide
// row pieces, by band length RB and workgroup width GW (waves = adjacent 128-column
// windows owning 120 columns each).  Geometry as the headline: 4K bf16, 3 planes, B = 128.
//   LD 0: dword buffer loads per lane into a register ring PD rows ahead (today)
//   LD 1: LDS-DMA: the workgroup's span of a plane row (GW x 240 B + halo) as 1-KiB
//         dwordx4 pieces, one piece per wave and step, a ring of NS rows, raw s_barrier
//   ST 0: dword stores of each wave's owned columns (240 B)
//   ST 1: rows staged in LDS, the workgroup's GW x 240 owned bytes stored as 16-B lanes
//         (960 B per wave-instruction), one piece per wave and step
// walk4 (profiles/r04/walk4_a.txt): RB 42 LD0/ST0 0.627, RB 12 0.705, LD1+ST1 (GW 4) 0.696,
// one-shot copy 0.779 of 8 TB/s.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int H = 2160, W = 3840, C = 3, OWN = 120, HL = 4, NWIN = W / OWN;   // 32 windows

__device__ __forceinline__ unsigned xcd_swz(unsigned bid, unsigned nwg) {
    const unsigned q = nwg >> 3, r = nwg & 7u, x = bid & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

template <int RB, int GW, int LD, int ST, int PD>
__global__ __launch_bounds__(GW * 64) void walk(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B) {
    constexpr int NB = (H + RB - 1) / RB, NGRP = NWIN / GW;
    constexpr int P = GW / 4;                      // 1-KiB pieces per plane row (LD 1 / ST 1)
    constexpr int NS = PD + 2;                     // ring rows
    constexpr int RING = LD == 1 ? NS * C * P * 1024 : 16;
    constexpr int STG = ST == 1 ? 2 * C * P * 1024 : 0;
    __shared__ __attribute__((aligned(16))) unsigned char lds[RING + STG];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned bid = xcd_swz(blockIdx.x, gridDim.x);
    const int grp = bid % NGRP;
    const unsigned r_ = bid / NGRP;
    const int band = r_ % NB;
    const int64_t b = r_ / NB;
    if (b >= B) return;
    const int win = grp * GW + wslot;
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
    // this wave's piece j = wslot (j < C * P): plane j / P, part j % P of the group's span
    const int gcol0 = grp * GW * OWN - 8;          // span starts 8 columns left (16-B aligned)
    const bool has_piece = wslot < C * P;
    const int pc_ = wslot / P, pp = wslot % P;
    const int pcol = gcol0 + pp * 512 + 8 * lane;
    const unsigned goff = (pcol >= 0 && pcol < W) ? (unsigned)pcol * 2 : 0x80000000u;
    const int scol = grp * GW * OWN + pp * 480 + 8 * lane;   // staged stores: 60 lanes x 16 B
    const unsigned sgoff = (lane < 60 && scol < W && has_piece) ? (unsigned)scol * 2 : 0x80000000u;
    unsigned* stg = reinterpret_cast<unsigned*>(lds + RING);
    unsigned acc = 0;

    auto dma = [&](int r) {
        if (!has_piece) return;
        const int slot = ((r - s0 + 2) % NS + NS) % NS;
        const unsigned so = roff(r) + pc_ * xplane;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr, (__attribute__((address_space(3))) void*)(lds + ((slot * C + pc_) * P + pp) * 1024), 16, goff,
            so, 0, 0);
    };
    auto store_row = [&](int r, const unsigned (&v)[C]) {
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)r * xrow));
        if constexpr (ST == 0) {
#pragma unroll
            for (int c = 0; c < C; ++c) __builtin_amdgcn_raw_buffer_store_b32(v[c], yr, yoff, so + c * xplane, 0);
        } else {
            const int sb = r & 1;
            if (lane >= HL / 2 && lane < (HL + OWN) / 2) {
#pragma unroll
                for (int c = 0; c < C; ++c) stg[(sb * C + c) * P * 256 + wslot * (OWN / 2) + lane - HL / 2] = v[c];
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
            if (has_piece) {
                typedef unsigned u4 __attribute__((ext_vector_type(4)));
                const u4 q = *reinterpret_cast<const u4*>(&stg[(sb * C + pc_) * P * 256 + pp * 240 + 4 * min(lane, 59)]);
                __builtin_amdgcn_raw_buffer_store_b128(q, yr, sgoff, so + pc_ * xplane, 0);
            }
        }
    };

    if constexpr (LD == 0) {
        unsigned ring[PD + 1][C];
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            const unsigned so = roff(s0 - 2 + i);
#pragma unroll
            for (int c = 0; c < C; ++c) ring[i][c] = __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, so + c * xplane, 0);
        }
        int r = s0 - 2;
        for (; r + PD + 1 <= s1 + 2; r += PD + 1) {
#pragma unroll
            for (int i = 0; i <= PD; ++i) {
                const unsigned so = roff(r + i + PD);
#pragma unroll
                for (int c = 0; c < C; ++c) ring[(i + PD) % (PD + 1)][c] = __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, so + c * xplane, 0);
                unsigned v[C];
#pragma unroll
                for (int c = 0; c < C; ++c) { v[c] = ring[i][c] + 1u; acc += ring[i][c]; }
                if (r + i >= s0 && r + i < s1) store_row(r + i, v);
            }
        }
        for (; r < s1 + 2; ++r) {
            const unsigned so = roff(r);
            unsigned v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = __builtin_amdgcn_raw_buffer_load_b32(xr, xoff, so + c * xplane, 0) + 1u;
            if (r >= s0 && r < s1) store_row(r, v);
        }
    } else {
        for (int i = 0; i < PD; ++i) dma(s0 - 2 + i);
        for (int r = s0 - 2; r < s1 + 2; ++r) {
            if (r + PD < s1 + 2) dma(r + PD);
            {   // own piece of row r landed: the ops issued after it may stay in flight
                constexpr int N = PD * (1 + (ST == 0 ? C : 1));
                static_assert(N < 64, "vmcnt");
                __builtin_amdgcn_s_waitcnt((0x0f70 & ~0xf) | (N & 0xf) | ((N >> 4) << 14));
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const int slot = ((r - s0 + 2) % NS + NS) % NS;
            unsigned v[C];
            const int cl = ce - gcol0;               // column inside the group span (>= 4)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const unsigned q = *reinterpret_cast<const unsigned*>(lds + (slot * C + c) * P * 1024 + 2 * min(max(cl, 0), P * 512 - 2));
                v[c] = q + 1u;
                acc += q;
            }
            if (r >= s0 && r < s1) store_row(r, v);
        }
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
template <int RB, int GW, int LD, int ST, int PD = 3>
void run(const uint16_t* x, uint16_t* y, int B) {
    const int blocks = (NWIN / GW) * ((H + RB - 1) / RB) * B;
    const float ms = timeit([&] { hipLaunchKernelGGL((walk<RB, GW, LD, ST, PD>), dim3(blocks), dim3(GW * 64), 0, 0, x, y, B); }, 9);
    printf("RB=%3d GW=%2d LD %d ST %d PD %d: %.3f ms  %.3f of 8 TB/s\n", RB, GW, LD, ST, PD, ms, GB / ms * 1e3 / 8000);
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
    printf("one-shot float4 copy (ceiling): %.3f ms  %.3f of 8 TB/s\n", mc, GB / mc * 1e3 / 8000);
    run<42, 4, 0, 0>(x, y, B);
    run<24, 4, 0, 0>(x, y, B);
    run<18, 4, 0, 0>(x, y, B);
    run<12, 4, 0, 0>(x, y, B);
    run<6, 4, 0, 0>(x, y, B);
    run<42, 4, 1, 1>(x, y, B);
    run<24, 4, 1, 1>(x, y, B);
    run<18, 4, 1, 1>(x, y, B);
    run<12, 4, 1, 1>(x, y, B);
    run<42, 8, 1, 1>(x, y, B);
    run<18, 8, 1, 1>(x, y, B);
    run<12, 8, 1, 1>(x, y, B);
    run<42, 16, 1, 1>(x, y, B);
    run<18, 16, 1, 1>(x, y, B);
    run<12, 16, 1, 1>(x, y, B);
    run<42, 8, 0, 0>(x, y, B);
    run<42, 16, 0, 0>(x, y, B);
    run<18, 4, 1, 1, 5>(x, y, B);
    run<42, 4, 0, 0>(x, y, B);
    return 0;
}
