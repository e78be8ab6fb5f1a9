// rt4.hip — BASELINE config 2's round trip rect -> hex -> rect (geometry_np.py:358-519 then
// :191-356, same-size lattices) with FOUR columns per lane (round 5), an opt-in alternative
// (HYGRID_RT4=1) to the two-column k_fused MD 2 (fused_kernel.h), which waits on vmcnt for ~76 %
// of its wave cycles at 3 % VALU (profiles/r04/b/pmc_rt_summary.txt).  The hypothesis was a
// latency-bound walk that needs more bytes in flight per wave (16-B accesses, 4 rows ahead, 8
// waves per SIMD); measured, it is 1.4 % slower on the config-2 launch (profiles/r05/rt4_ab.txt),
// so more bytes in flight do not move this launch and MD 2 stays the default.
//
// One wave owns a 256-column window (lane l <-> columns ce .. ce + 3, ce = W0 + 4 l; 240 owned,
// 8 + 8 halo) of one plane and walks a band of RT4_RB output rows.  Per output row a2:
//   1. rect row a2 + 1 arrives in registers, loaded RT4_PD steps earlier into a 6-slot ring
//      (16-B `dwordx4` loads per lane for fp32, 8-B for 16-bit: 1 KiB / 512 B per wave-row);
//   2. hex row a2 = the vertical r2h blend of rect rows a2 - 1 .. a2 + 1 (row weights from a
//      per-wave LDS table, geometry_np.py:440-486) and the horizontal blend of its columns
//      (per-lane weights, :441-449, 514-517; the window's outer neighbours one DPP shift away);
//   3. output row a2 = the exact same-size h2r (i_ = a2, j_ = 0.5 a2 + b + 0.25, so even rows
//      0.75 z[b] + 0.25 z[b + 1] and odd rows 0.25 z[b - 1] + 0.75 z[b], :347-354): the output
//      row depends on hex row a2 alone, so the hex image never leaves the registers.
// Every product and sum is the two-column kernel's in the same order (fmaf per column; the
// vertical blend as packed halves, each an IEEE fmaf): outputs are bit-identical to k_fused MD 2
// (tests/test_gpu_roundtrip.py), which is oracle-checked at 1e-5.
//
// Domain: fused_rt_try's (same-size near-identity lattice) with w and w1 multiples of 4 (a
// lane's four columns are all inside the raster or all outside); HG_EUNSUP otherwise.
#include <climits>
#include <cmath>
#include <cstdlib>

#include "fused_kernel.h"

namespace hg {

#ifndef RT4_RB_
#define RT4_RB_ 18                     // output rows per band (multiple of 6)
#endif
#ifndef RT4_PD
#define RT4_PD 4                       // rect rows loaded ahead of use (1..5)
#endif
#ifndef RT4_WPE
#define RT4_WPE 8                      // waves per SIMD asked of the register allocator
#endif
constexpr int RT4_GW = 4, RT4_THREADS = 256;
constexpr int RT4_HL = 8, RT4_OWN = 240;
constexpr int RT4_RB = RT4_RB_;
static_assert(RT4_RB % 6 == 0 && RT4_RB > 0, "bands are whole 6-step blocks");
static_assert(RT4_PD >= 1 && RT4_PD <= 5, "raw ring: rows a2+2 .. a2+1+PD in flight in 6 slots");

// raw row of one lane: 4 elements (16-bit: 2 dwords, fp32: 4 dwords)
template <typename T> struct Rt4Raw { typedef unsigned type __attribute__((ext_vector_type(2))); };
template <> struct Rt4Raw<float> { typedef unsigned type __attribute__((ext_vector_type(4))); };

template <typename T>
__device__ __forceinline__ typename Rt4Raw<T>::type rt4_load(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                                             unsigned soff) {
    if constexpr (sizeof(T) == 2) return __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    else return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
}

// columns ce .. ce + 3 as the pairs A = (ce, ce + 1), B = (ce + 2, ce + 3); the fp32 words are
// bit-cast as one vector (per-element casts of a buffer-load vector were miscompiled)
template <typename T>
__device__ __forceinline__ void rt4_unpack(typename Rt4Raw<T>::type r, fu_f2& a, fu_f2& b, unsigned hi16) {
    if constexpr (std::is_same<T, float>::value) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = __builtin_bit_cast(f4v, r);
        a = fu_f2{v.x, v.y};
        b = fu_f2{v.z, v.w};
    } else {
        float e, o;
        fu_unpack<T>(r.x, e, o, hi16);
        a = fu_f2{e, o};
        fu_unpack<T>(r.y, e, o, hi16);
        b = fu_f2{e, o};
    }
}

template <typename T>
__device__ __forceinline__ void rt4_store(float o0, float o1, float o2, float o3,
                                          __amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    if constexpr (std::is_same<T, float>::value) {
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        const u4v v = {__builtin_bit_cast(unsigned, o0), __builtin_bit_cast(unsigned, o1),
                       __builtin_bit_cast(unsigned, o2), __builtin_bit_cast(unsigned, o3)};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 0);
    } else {
        typedef T t2v __attribute__((ext_vector_type(2)));
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        const u2v v = {__builtin_bit_cast(unsigned, t2v{(T)o0, (T)o1}),
                       __builtin_bit_cast(unsigned, t2v{(T)o2, (T)o3})};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, soff, 0);
    }
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(RT4_THREADS) __attribute__((amdgpu_waves_per_eu(RT4_WPE)))
void k_rt4(const Tin* __restrict__ x, Tout* __restrict__ y, FusedGeom F) {
    constexpr int PD = RT4_PD, RB = RT4_RB;
    using Raw = typename Rt4Raw<Tin>::type;
    __shared__ float4 lut_all[RT4_GW][RB];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* const lut = lut_all[wslot];
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (F.nwin + RT4_GW - 1) / RT4_GW;
    const int grp = (int)(blk % ngrp);
    const int band = (int)((blk / ngrp) % F.nband);
    const int64_t p = blk / ((int64_t)ngrp * F.nband);      // plane
    if (p >= F.B) return;                                     // uniform per workgroup
    const int win = grp * RT4_GW + wslot;                     // may be >= nwin: owns nothing
    const int W0 = win * RT4_OWN - RT4_HL;
    const int ce = W0 + 4 * lane;
    const int s0 = band * RB;
    const int s1 = min(s0 + RB, F.h2);

    // ---- row table: entry e = hex row s0 + e (fp64 lattice math, geometry_np.py:440-486) ----
    for (int e = lane; e < RB; e += 64) {
        const int r = s0 + e;
        float4 t = {0.f, 0.f, 0.f, 0.f};
        if (r < F.h1) {
            const double i_ = axis_at(F.rxs, r) + (double)(F.h - 1) * 0.5;   // :440
            const int in = (int)i_;                                          // :444
            const double f = i_ - (double)(float)in;                         // :448
            const float w0 = (in >= 0 && in < F.h) ? (float)(1.0 - f) : 0.f;
            const float w1 = (in + 1 >= 0 && in + 1 < F.h) ? (float)f : 0.f;
            if (in == r - 1) { t.x = w0; t.y = w1; }
            else if (in == r) { t.y = w0; t.z = w1; }
        }
        lut[e] = t;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    int rc = 0;
    {
        bool has_a = false, has_c = false;
        for (int e = lane; e < RB; e += 64) {
            const float4 t = lut[e];
            has_a |= t.x != 0.f;
            has_c |= t.z != 0.f;
        }
        const bool any_a = __builtin_amdgcn_ballot_w64(has_a) != 0;
        const bool any_c = __builtin_amdgcn_ballot_w64(has_c) != 0;
        rc = !any_c ? 1 : (!any_a ? 2 : 0);
    }

    // ---- per-lane column weights of the two pairs (geometry_np.py:441-449, 514-517) -------
    float we[2][3], wo[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float* wr = s ? wo[k] : we[k];
            wr[0] = wr[1] = wr[2] = 0.f;
            const int q = ce + 2 * k + s;
            if (q >= 0 && q < F.w1) {
                const double j_ = axis_at(F.rys, q) + (double)(F.w - 1) * 0.5;   // :441
                const int jn = (int)j_;
                const double jf = j_ - (double)(float)jn;
#pragma unroll
                for (int kk = -1; kk <= 1; ++kk) {
                    const bool in_w = q + kk >= 0 && q + kk < F.w;
                    if (kk == jn - q && in_w) wr[kk + 1] += (float)(1.0 - jf);
                    if (kk == jn + 1 - q && in_w) wr[kk + 1] += (float)jf;
                }
            }
        }
    const bool any_l = __builtin_amdgcn_ballot_w64(we[0][0] != 0.f || wo[0][0] != 0.f ||
                                                   we[1][0] != 0.f || wo[1][0] != 0.f) != 0;
    const bool any_r = __builtin_amdgcn_ballot_w64(we[0][2] != 0.f || wo[0][2] != 0.f ||
                                                   we[1][2] != 0.f || wo[1][2] != 0.f) != 0;
    const int cd = !any_r ? 1 : (!any_l ? 2 : 0);
    const bool own = lane >= RT4_HL / 4 && lane < (RT4_HL + RT4_OWN) / 4 && ce >= 0 && ce < F.w2 &&
                     win < F.nwin;

    // ---- buffers: one plane each way --------------------------------------------------
    const int64_t cstride = (int64_t)F.h * F.w, ostride = (int64_t)F.h2 * F.w2;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + p * cstride), (short)0, (int)(cstride * (int64_t)sizeof(Tin)), 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + p * ostride), (short)0, (int)(ostride * (int64_t)sizeof(Tout)), 0x00020000);
    const int lc = min(max(ce, 0), F.w - 4);                  // clamped load column (x 0 weights)
    const unsigned xoff = (unsigned)lc * (unsigned)sizeof(Tin);
    const unsigned yoff = own ? (unsigned)ce * (unsigned)sizeof(Tout) : 0x80000000u;
    const unsigned xrow = (unsigned)F.w * (unsigned)sizeof(Tin), yrow = (unsigned)F.w2 * (unsigned)sizeof(Tout);
    auto row_off = [&](int k) -> unsigned {
        return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(k, 0), F.h - 1) * xrow));
    };
    float c75 = 0.75f, c25 = 0.25f;                           // VGPR operands, not literals
    asm volatile("" : "+v"(c75), "+v"(c25));
    // h2r neighbours outside the raster (:303-323): the lane's right neighbour (even rows) and
    // left neighbour (odd rows); the inner ones are always inside (w2 % 4 == 0)
    const float wn = (ce + 4 < F.w2) ? c25 : 0.f;
    const float wp = (ce - 1 >= 0) ? c25 : 0.f;
    unsigned hi16 = 0xffff0000u;
    asm volatile("" : "+v"(hi16));

    auto run = [&](auto CDc, auto RCc) {
        constexpr int CD = decltype(CDc)::value;
        constexpr int RC = decltype(RCc)::value;
        Raw raw[6];                         // rect rows in flight, slot (row - s0 + 1) % 6
        fu_f2 XA[3], XB[3];                 // rect rows as f32 pairs, slot (row - s0 + 1) % 3

        auto issue = [&](auto SLc, int k) {
            raw[decltype(SLc)::value] = rt4_load<Tin>(xrs, xoff, row_off(k));
        };
        // hex row a2 = s0 + PH from rect rows a2 - 1, a2, a2 + 1 (slots PH, PH + 1, PH + 2
        // mod 3), then output row a2
        auto step_row = [&](auto PHc, float4 L, int a2) {
            constexpr int PH = decltype(PHc)::value;
            constexpr int S0 = PH % 3, S1 = (PH + 1) % 3, S2 = (PH + 2) % 3;
            const fu_f2 Lxy = {L.x, L.y}, Lzw = {L.z, L.w};
            auto vblend = [&](const fu_f2 (&X)[3]) {          // = k_fused MD 2's fmaf chain
                if constexpr (RC == 1) return fu_pfma<1, false>(Lxy, X[S1], fu_pmul<0>(Lxy, X[S0]));
                else if constexpr (RC == 2) return fu_pfma<0, false>(Lzw, X[S2], fu_pmul<1>(Lxy, X[S1]));
                else return fu_pfma<0, false>(Lzw, X[S2], fu_pfma<1, false>(Lxy, X[S1], fu_pmul<0>(Lxy, X[S0])));
            };
            const fu_f2 VA = vblend(XA), VB = vblend(XB);
            float u0, u1, u2, u3;                             // hex row a2, columns ce .. ce + 3
            if constexpr (CD == 1) {                          // taps q-1, q
                u0 = fmaf(we[0][1], VA.x, we[0][0] * f_prev(VB.y));
                u1 = fmaf(wo[0][1], VA.y, wo[0][0] * VA.x);
                u2 = fmaf(we[1][1], VB.x, we[1][0] * VA.y);
                u3 = fmaf(wo[1][1], VB.y, wo[1][0] * VB.x);
            } else if constexpr (CD == 2) {                   // taps q, q+1
                u0 = fmaf(we[0][2], VA.y, we[0][1] * VA.x);
                u1 = fmaf(wo[0][2], VB.x, wo[0][1] * VA.y);
                u2 = fmaf(we[1][2], VB.y, we[1][1] * VB.x);
                u3 = fmaf(wo[1][2], f_next(VA.x), wo[1][1] * VB.y);
            } else {
                const float pl = f_prev(VB.y), nx = f_next(VA.x);
                u0 = fmaf(we[0][2], VA.y, fmaf(we[0][1], VA.x, we[0][0] * pl));
                u1 = fmaf(wo[0][2], VB.x, fmaf(wo[0][1], VA.y, wo[0][0] * VA.x));
                u2 = fmaf(we[1][2], VB.y, fmaf(we[1][1], VB.x, we[1][0] * VA.y));
                u3 = fmaf(wo[1][2], nx, fmaf(wo[1][1], VB.y, wo[1][0] * VB.x));
            }
            float o0, o1, o2, o3;
            if constexpr ((PH & 1) == 0) {                    // 0.75 z[b] + 0.25 z[b+1]
                o0 = fmaf(c25, u1, c75 * u0);
                o1 = fmaf(c25, u2, c75 * u1);
                o2 = fmaf(c25, u3, c75 * u2);
                o3 = fmaf(wn, f_next(u0), c75 * u3);
            } else {                                          // 0.25 z[b-1] + 0.75 z[b]
                o0 = fmaf(wp, f_prev(u3), c75 * u0);
                o1 = fmaf(c25, u0, c75 * u1);
                o2 = fmaf(c25, u1, c75 * u2);
                o3 = fmaf(c25, u2, c75 * u3);
            }
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a2 * yrow));
            rt4_store<Tout>(o0, o1, o2, o3, yrs, yoff, so);
        };

        // ---- prologue: rect rows s0 - 1, s0 in the X ring; rows s0 + 1 .. s0 + PD in flight
        {
            const Raw t0 = rt4_load<Tin>(xrs, xoff, row_off(s0 - 1));
            const Raw t1 = rt4_load<Tin>(xrs, xoff, row_off(s0));
            issue(IC<2>{}, s0 + 1);
            if (PD >= 2) issue(IC<3>{}, s0 + 2);
            if (PD >= 3) issue(IC<4>{}, s0 + 3);
            if (PD >= 4) issue(IC<5>{}, s0 + 4);
            if (PD >= 5) issue(IC<0>{}, s0 + 5);
            rt4_unpack<Tin>(t0, XA[0], XB[0], hi16);
            rt4_unpack<Tin>(t1, XA[1], XB[1], hi16);
        }
        __builtin_amdgcn_s_waitcnt(0x0f70);                  // vmcnt(0): see fused_kernel.h FU_DRAIN

        float4 lnext = lut[0];
        auto step = [&](auto PHc, int a2) {
            constexpr int PH = decltype(PHc)::value;
            __builtin_amdgcn_sched_barrier(0);
            rt4_unpack<Tin>(raw[(PH + 2) % 6], XA[(PH + 2) % 3], XB[(PH + 2) % 3], hi16);   // row a2+1
            issue(IC<(PH + 2 + PD) % 6>{}, a2 + 1 + PD);
            const float4 L = lnext;
            lnext = lut[min(a2 - s0 + 1, RB - 1)];
            step_row(PHc, L, a2);
        };
        auto block6 = [&](int b) {
            step(IC<0>{}, b);
            step(IC<1>{}, b + 1);
            step(IC<2>{}, b + 2);
            step(IC<3>{}, b + 3);
            step(IC<4>{}, b + 4);
            step(IC<5>{}, b + 5);
        };
        int base = s0;
        for (; base + 6 <= s1; base += 6) block6(base);
        if (base < s1) {
            step(IC<0>{}, base);
            if (base + 1 < s1) {
                step(IC<1>{}, base + 1);
                if (base + 2 < s1) {
                    step(IC<2>{}, base + 2);
                    if (base + 3 < s1) {
                        step(IC<3>{}, base + 3);
                        if (base + 4 < s1) step(IC<4>{}, base + 4);
                    }
                }
            }
        }
    };
    if (cd == 1 && rc == 1) run(IC<1>{}, IC<1>{});
    else if (cd == 1 && rc == 2) run(IC<1>{}, IC<2>{});
    else if (cd == 2 && rc == 1) run(IC<2>{}, IC<1>{});
    else if (cd == 2 && rc == 2) run(IC<2>{}, IC<2>{});
    else run(IC<0>{}, IC<0>{});
}

// The four-column round trip for a call fused_rt_try has validated (same-size near-identity
// lattice, F's axes set); HG_EUNSUP outside its narrower domain (the caller runs k_fused MD 2).
int rt4_try(const void* x, void* y, int x_dtype, int y_dtype, const FusedGeom& F0, hipStream_t st) {
    // Opt-in (HYGRID_RT4=1): measured 1.4 % SLOWER than the two-column kernel on the config-2
    // launch (0.3115 vs 0.3071 ms, 1080p fp32 b32; band 12 / 30 rows and 2 / 5 rows of prefetch
    // within +-1 % or slower: profiles/r05/rt4_ab.txt): more bytes in flight per wave did not
    // move this launch, so k_fused MD 2 stays the default.
    if (!env_is("HYGRID_RT4", "1")) return HG_EUNSUP;
    if ((F0.w % 4) || (F0.w2 % 4) || F0.w < 4) return HG_EUNSUP;
    FusedGeom F = F0;
    F.nwin = (int)((F.w2 + RT4_OWN - 1) / RT4_OWN);
    F.nband = (int)((F.h2 + RT4_RB - 1) / RT4_RB);
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + RT4_GW - 1) / RT4_GW);
    if (blocks > INT_MAX) return HG_EUNSUP;
    const dim3 grid((unsigned)blocks), blk(RT4_THREADS);
#define HG_RT4(TI, TO)                                                                         \
    hipLaunchKernelGGL((k_rt4<TI, TO>), grid, blk, 0, st, (const TI*)x, (TO*)y, F);            \
    return launch_status();
    if (x_dtype == HG_F32 && y_dtype == HG_F32) { HG_RT4(float, float) }
    if (x_dtype == HG_BF16 && y_dtype == HG_BF16) { HG_RT4(__bf16, __bf16) }
    if (x_dtype == HG_F16 && y_dtype == HG_F16) { HG_RT4(_Float16, _Float16) }
    if (x_dtype == HG_BF16 && y_dtype == HG_F32) { HG_RT4(__bf16, float) }
    if (x_dtype == HG_F16 && y_dtype == HG_F32) { HG_RT4(_Float16, float) }
#undef HG_RT4
    return HG_EUNSUP;
}

// band rows / owned columns / left halo (hg_fused_layout(7, ...): tests place edge inputs)
void rt4_layout(int* band_rows, int* win_own, int* win_halo) {
    *band_rows = RT4_RB;
    *win_own = RT4_OWN;
    *win_halo = RT4_HL;
}

}  // namespace hg
