// fused_kernel.h — the two-column streaming kernel shared by the fused pipeline
// (fused.hip: rect -> hex -> HexConv2d(r=2) -> hex -> rect) and the HexConv2d-only
// mode (fused_conv.hip).  See fused.hip for the pipeline's design notes.
#pragma once
#include <climits>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "fused.h"
#include "lattice.h"

namespace hg {

#ifndef FU_GW_
#define FU_GW_ 4
#endif
constexpr int FU_GW = FU_GW_;          // waves (adjacent windows) per workgroup
constexpr int FU_THREADS = 64 * FU_GW;
#ifndef FU_HL_
#define FU_HL_ 4
#endif
#ifndef FU_OWN_
#define FU_OWN_ 120
#endif
constexpr int FU_HL = FU_HL_;         // halo columns on the left of a window
constexpr int FU_OWN = FU_OWN_;       // owned columns per 128-column window
// Output rows per band (multiple of 6), MD 0 / MD 1.  Shorter bands than the 126 of
// round 1 measured faster (in-process A/B on 4K bf16 b128, tools/ab_fused.py /
// tools/ab_ops.py): pipeline 3.00 -> 2.83 ms at 66 (round 2), 66 -> 42 a further -1.8 %
// (round 3, profiles/r03/g); HexConv2d 3.19 -> 2.73 ms at 18.
#ifndef FU_RB_
#define FU_RB_ 42
#endif
#ifndef FU_RB_CONV_
#define FU_RB_CONV_ 18
#endif
#ifndef FU_RB_PYR_
#define FU_RB_PYR_ 60                 // MD 3 / 4: input rows per band (30 output rows)
#endif
#ifndef FU_RB_PYRS_
#define FU_RB_PYRS_ 24                // MD 5 (= MD 4 on short bands for small levels)
#endif
#ifndef FU_RB_RT_
#define FU_RB_RT_ 6                   // MD 2: rows per band (66 -> 30: 0.321 -> 0.307 ms, r03 A/B;
                                      // with the upward bands of round 6 shorter is faster: 30 /
                                      // 12 / 6 rows 0.304 / 0.297 / 0.289 ms, and the launch's
                                      // ramp + tail 42 -> 20 us at 12, profiles/r06/)
#endif
constexpr int FU_RB = FU_RB_;
constexpr int FU_RB_CONV = FU_RB_CONV_;
constexpr int FU_RB_PYR = FU_RB_PYR_;
constexpr int FU_RB_PYRS = FU_RB_PYRS_;
constexpr int FU_RB_RT = FU_RB_RT_;
constexpr int fu_max(int a, int b) { return a > b ? a : b; }
constexpr int FU_LUT =
    fu_max(fu_max(FU_RB, FU_RB_CONV), fu_max(fu_max(FU_RB_PYR, FU_RB_PYRS), FU_RB_RT)) + 2;
// the one definition of a mode's band length, used by the kernel and the host launchers
__host__ __device__ constexpr int fu_rb(int md) {
    return md == 1 ? FU_RB_CONV : md == 5 ? FU_RB_PYRS : md >= 3 ? FU_RB_PYR : md == 2 ? FU_RB_RT : FU_RB;
}
static_assert(FU_RB % 6 == 0 && FU_RB_CONV % 6 == 0 && FU_RB_PYR % 6 == 0 && FU_RB_PYRS % 6 == 0 &&
              FU_RB_RT % 6 == 0 && FU_RB > 0 && FU_RB_CONV > 0 && FU_RB_PYR > 0 && FU_RB_PYRS > 0 &&
              FU_RB_RT > 0,
              "bands are whole 6-step blocks (ring slots x row parities), even-aligned");
static_assert(FU_OWN % 2 == 0 && FU_HL % 2 == 0 && FU_HL + FU_OWN <= 128 - 2,
              "owned columns are whole lanes with a halo of >= 1 lane on each side");

// Tuning knobs (compile-time; tools/build_*variant.sh rebuild one object with other values).
#ifndef FU_PD
#define FU_PD 3                       // rect rows loaded ahead of use (1..5)
#endif
#ifndef FU_WPE
#define FU_WPE 1                      // minimum waves per SIMD asked of the register allocator
#endif
#ifndef FU_WPE_CONV
#define FU_WPE_CONV 4                 // HexConv2d mode: 129 -> 128 VGPRs buys a 4th wave per SIMD
#endif
#ifndef FU_MIN_INST
#define FU_MIN_INST 0                 // 1: build only the bf16 C3 O3 G1 kernels (variants)
#endif
#ifndef FU_WPS
#define FU_WPS 21                     // the first FU_WPS weight pairs live in SGPRs (v_pk_fma_f32
                                      // reads an SGPR operand at full rate, unlike v_fmac_f32), the
                                      // rest in VGPRs; 21 of 32 keeps both register files unspilled
#endif
#ifndef FU_REV
#define FU_REV 1                      // MD 1 / MD 2: odd full bands walk upwards (round 6, below)
#endif
// Fixed design choices of earlier rounds, each measured faster than its alternative in an
// in-process A/B: the 7-tap stencil as v_pk_fma_f32 on (even, odd) column pairs
// with the weights broadcast by op_sel (round 3); the r2h vertical blend packed the same way;
// per-band row classes and per-window column classes of the r2h taps; MD 0's h2r 0.75 folded into
// the r2h column weights and its neighbour term as v_fmac_f32_dpp; a scheduling barrier per step
// and 12-step loop bodies; the prologue's loads drained before the loop; the pyramid modes'
// triangle vertices gathered from LDS, their uniform row lattice from a per-band LDS table and
// column-interior windows without per-vertex tests.  Round 6 removed the A/B paths that lost
// (LDS-DMA row rings and staged stores, LDS-staged line stores, v_fma_mix vertical blends, the
// scalar stencil, workgroup orders, cache-policy bits) and the wrong-result diagnostics.
// (Round 3 also measured the stencil's shifted u pairs exchanged through a per-wave LDS row
// instead of DPP moves + pair copies: 6 fewer DPP and 6 fewer moves per step, but 130-136
// VGPRs (3 waves per SIMD) or scratch spills at a 128 cap, 1.6-2.2 % slower)

struct FusedGeom {
    int64_t B;
    int h, w, h1, w1, h2, w2;
    int nwin, nband;
    Axis rxs, rys;                    // r2h lattice axes (geometry_np.py:415-422)
    Axis txs, tys;                    // MD 3 / 4: hexresize lattice axes (geometry_np.py:570-582)
};

__device__ __forceinline__ float f_prev(float v) {   // result[l] = v[l-1], 0 at lane 0
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x138 /*wave_shr:1*/, 0xf, 0xf, true));
}
__device__ __forceinline__ float f_next(float v) {   // result[l] = v[l+1], 0 at lane 63
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x130 /*wave_shl:1*/, 0xf, 0xf, true));
}

// r=2 stencil taps (HexFrames.py:108-118 scatter into the dense 3x5 kernel):
// row of tap t relative to the output row (0 above, 1 centre, 2 below) and its lane
// column shift for an output row of parity `par` (type1 indexing, :417-445; derived in
// oracle/hg_oracle.c), with padding 1: shift = dk - 1.
__host__ __device__ constexpr int fu_tap_ii(int t) { return t < 2 ? 0 : (t < 5 ? 1 : 2); }
__host__ __device__ constexpr int fu_tap_col(int t) {
    return t < 2 ? 1 + 2 * t : (t < 5 ? 2 * (t - 2) : 1 + 2 * (t - 5));
}
__host__ __device__ constexpr int fu_tap_shift(int t, int par, int op) {
    return ((1 + par + fu_tap_col(t) - ((((par + fu_tap_ii(t)) & 1) + op) & 1)) >> 1) - 1;
}

template <typename T> struct RawOf { using type = unsigned; };          // 2 x 16-bit
template <> struct RawOf<float> { using type = uint2; };                // 2 x f32

template <typename T>
__device__ __forceinline__ typename RawOf<T>::type fu_load(__amdgpu_buffer_rsrc_t rs,
                                                           unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 2) {
        return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
    } else {
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        const u2v v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        return uint2{v.x, v.y};
    }
}
// hi16: 0xffff0000 held in a VGPR (a literal operand would halve the issue rate)
template <typename T>
__device__ __forceinline__ void fu_unpack(typename RawOf<T>::type r, float& e, float& o,
                                          unsigned hi16) {
    if constexpr (std::is_same<T, __bf16>::value) {
        e = __builtin_bit_cast(float, r << 16);
        o = __builtin_bit_cast(float, r & hi16);
    } else if constexpr (sizeof(T) == 2) {
        e = (float)__builtin_bit_cast(T, (unsigned short)(r & 0xffffu));
        o = (float)__builtin_bit_cast(T, (unsigned short)(r >> 16));
    } else {
        e = __builtin_bit_cast(float, r.x);
        o = __builtin_bit_cast(float, r.y);
    }
}
template <typename T>
__device__ __forceinline__ void fu_store(float e, float o, __amdgpu_buffer_rsrc_t rs,
                                         unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 2) {
        typedef T t2v __attribute__((ext_vector_type(2)));
        const t2v p = {(T)e, (T)o};
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, p), rs, voff, soff, 0);
    } else {
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(
            u2v{__builtin_bit_cast(unsigned, e), __builtin_bit_cast(unsigned, o)}, rs, voff, soff, 0);
    }
}

template <int N> using IC = std::integral_constant<int, N>;
typedef float fu_f2 __attribute__((ext_vector_type(2)));
// One packed FMA on the lane's (even, odd) column pair, each half an IEEE fmaf (so the
// result is bit-identical to two v_fmac_f32): c += w[H] * a, the weight half H of the
// opaque weight pair broadcast with op_sel.  Written as asm because the compiler, given a
// splat, materialises it as a separate VGPR pair per weight (126 VGPRs for 63 weights).
#define FU_PFMA_(SEL, WC)                                                                     \
    asm("v_pk_fma_f32 %0, %1, %2, %0 " SEL : "+v"(c) : WC(wp), "v"(a))
template <int H, bool S>
__device__ __forceinline__ fu_f2 fu_pfma(fu_f2 wp, fu_f2 a, fu_f2 c) {
    if constexpr (H && S) FU_PFMA_("op_sel:[1,0,0] op_sel_hi:[1,1,1]", "s");
    else if constexpr (H) FU_PFMA_("op_sel:[1,0,0] op_sel_hi:[1,1,1]", "v");
    else if constexpr (S) FU_PFMA_("op_sel_hi:[0,1,1]", "s");
    else FU_PFMA_("op_sel_hi:[0,1,1]", "v");
    return c;
}
#undef FU_PFMA_
// d = w[H] * a + b[HB]: the same with the bias half HB of a (VGPR) bias pair broadcast
#define FU_PFMAB_(SEL, WC)                                                                    \
    asm("v_pk_fma_f32 %0, %1, %2, %3 " SEL : "=v"(d) : WC(wp), "v"(a), "v"(bp))
template <int H, int HB, bool S>
__device__ __forceinline__ fu_f2 fu_pfma_b(fu_f2 wp, fu_f2 a, fu_f2 bp) {
    fu_f2 d;
    if constexpr (S) {
        if constexpr (H && HB) FU_PFMAB_("op_sel:[1,0,1] op_sel_hi:[1,1,1]", "s");
        else if constexpr (H) FU_PFMAB_("op_sel:[1,0,0] op_sel_hi:[1,1,0]", "s");
        else if constexpr (HB) FU_PFMAB_("op_sel:[0,0,1] op_sel_hi:[0,1,1]", "s");
        else FU_PFMAB_("op_sel_hi:[0,1,0]", "s");
    } else {
        if constexpr (H && HB) FU_PFMAB_("op_sel:[1,0,1] op_sel_hi:[1,1,1]", "v");
        else if constexpr (H) FU_PFMAB_("op_sel:[1,0,0] op_sel_hi:[1,1,0]", "v");
        else if constexpr (HB) FU_PFMAB_("op_sel:[0,0,1] op_sel_hi:[0,1,1]", "v");
        else FU_PFMAB_("op_sel_hi:[0,1,0]", "v");
    }
    return d;
}
#undef FU_PFMAB_
// d = w[H] * a (packed multiply, weight half H broadcast; VGPR weight pair)
template <int H>
__device__ __forceinline__ fu_f2 fu_pmul(fu_f2 wp, fu_f2 a) {
    fu_f2 d;
    if constexpr (H) asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(d) : "v"(wp), "v"(a));
    else asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(d) : "v"(wp), "v"(a));
    return d;
}
// The folded same-size h2r of three conv-row pairs z_o = (ze, zo) (MD 0, O = 3) as one asm
// block: the three lane-local FMAs first, then the three neighbour terms as v_fmac_f32_dpp
// (DPP on src0, 0 past the wave edge = f_next / f_prev), so every DPP source was written
// >= 3 VALU instructions earlier (a DPP read needs 2 wait states after a VALU write, and the
// hazard recognizer does not look inside an inline-asm consumer).
//   even row: oe = c13 * zo + ze,  oo = zo + next(ze) * wn
//   odd row:  oo = c13 * ze + zo,  oe = ze + prev(zo) * wp
// Bit-identical to fmaf(c13, zo, ze) / fmaf(wn, f_next(ze), zo) (products commute).
__device__ __forceinline__ void fu_h2r3_even(float& e0, float& o0, float& e1, float& o1,
                                             float& e2, float& o2, float c13, float wn) {
    float a0, a1, a2;
    asm("v_fma_f32 %0, %9, %4, %3\n\t"
        "v_fma_f32 %1, %9, %6, %5\n\t"
        "v_fma_f32 %2, %9, %8, %7\n\t"
        "v_fmac_f32_dpp %4, %3, %10 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f32_dpp %6, %5, %10 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f32_dpp %8, %7, %10 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "+v"(e0), "+v"(o0), "+v"(e1), "+v"(o1), "+v"(e2),
          "+v"(o2)
        : "v"(c13), "v"(wn));
    e0 = a0; e1 = a1; e2 = a2;
}
__device__ __forceinline__ void fu_h2r3_odd(float& e0, float& o0, float& e1, float& o1,
                                            float& e2, float& o2, float c13, float wp) {
    float a0, a1, a2;
    asm("v_fma_f32 %0, %9, %3, %4\n\t"
        "v_fma_f32 %1, %9, %5, %6\n\t"
        "v_fma_f32 %2, %9, %7, %8\n\t"
        "v_fmac_f32_dpp %3, %4, %10 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f32_dpp %5, %6, %10 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_fmac_f32_dpp %7, %8, %10 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "+v"(e0), "+v"(o0), "+v"(e1), "+v"(o1), "+v"(e2),
          "+v"(o2)
        : "v"(c13), "v"(wp));
    o0 = a0; o1 = a1; o2 = a2;
}
template <typename T>
__device__ __forceinline__ fu_f2 fu_unpack2(typename RawOf<T>::type r, unsigned hi16) {
    float e, o;
    fu_unpack<T>(r, e, o, hi16);
    return fu_f2{e, o};
}
__host__ __device__ constexpr int fu_mod(int a, int m) { return ((a % m) + m) % m; }
// compile-time loop: f(IC<B>{}), f(IC<B+1>{}), ..., f(IC<E-1>{})
template <int B, int E, typename F>
__device__ __forceinline__ void fu_sfor(F&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        fu_sfor<B + 1, E>(f);
    }
}

// MD 0: rect -> hex -> HexConv2d -> hex -> rect (the pipeline).  MD 1: HexConv2d alone
// (radius 2, stride 1, padding 1, pad value 0; HexFrames.py:96-169): the "u rows" are
// the input hex rows themselves and conv rows are stored as they complete.  MD 2: the
// round trip rect -> hex -> rect without the conv (BASELINE config 2): each u row is its
// own "conv row" (C == O, no weights) and goes straight through the h2r filter.
// MD 3 / 4: one hex-pyramid level (BASELINE config 5), the depthwise HexConv2d followed by
// hexresize to (h / 2, w / 2) (geometry_np.py:520-681) for a 2x downsample: MD 3 from the
// rect image (u rows made by r2h, as MD 0), MD 4 from a hex image (u rows = input rows, as
// MD 1; MD 5 = MD 4 on shorter bands, for levels too small to fill the chip).  Every second
// step completes the two conv rows an output row's triangles read; a window of 128 input
// columns owns 60 output columns (lane l <-> output column W0/2 + l).
//
// Band direction (MD 1 / MD 2, FU_REV, round 6; the headline's k_fused4 does the same): the
// halo rows two neighbouring bands share are read by both at the same time when the odd full
// bands walk upwards (both reach their shared boundary at their start, or both at their end,
// while they run side by side on one XCD) instead of a band's walk apart.  MD 2's u rows and
// outputs are the same either way; MD 1's conv rows sum their below taps first on an upward
// band (the same products in another order).
// A workgroup's LDS (one struct, so that a kernel running bands of several modes with the same
// PYR / O — the pyramid chain, pyramid_fused.hip — allocates it once).
constexpr int FU_ZW = 130;
constexpr int FU_NPT = FU_RB_PYR / 2 + 1;
template <bool PYR, int O>
struct FuShared {
    // per-wave u-row table {a, b, c, -}: u[r] = a*x[r-1] + b*x[r] + c*x[r+1]
    float4 lut[FU_GW][FU_LUT];
    // PYR: the two conv rows an output row reads, per wave: [row][channel][col], cols
    // 0..127 of the window + a zero at 128 (vertices outside the raster) and a pad
    float zl[PYR ? FU_GW : 1][PYR ? 2 * O * FU_ZW : 1];
    // PYR: per output row of the band {0.5 i_, i_f} and i_n (geometry_np.py:601-612)
    double ptd[PYR ? FU_GW : 1][PYR ? FU_NPT : 1][2];
    int pti[PYR ? FU_GW : 1][PYR ? FU_NPT : 1];
};

// One workgroup's work unit (image, band, group of 4 windows) = logical block `blk`.
template <typename Tin, typename Tout, int C, int O, int G, int OP, int MD>
__device__ __forceinline__ void fu_band(const Tin* __restrict__ x, const float* __restrict__ kern,
                                        const float* __restrict__ bias, Tout* __restrict__ y,
                                        const FusedGeom& F, int64_t blk,
                                        FuShared<(MD >= 3), O>& sh) {
    constexpr int CG = C / G, OG = O / G;
    constexpr int PD = FU_PD;
    constexpr bool PYR = MD >= 3;                 // hex-pyramid level (hexresize output stage)
    constexpr bool UIN = MD == 1 || MD >= 4;      // u rows = input rows (no r2h)
    constexpr bool PK = MD != 2;                  // the packed 7-tap stencil (every conv mode)
    constexpr bool VPK = PK && !UIN;              // the packed r2h vertical blend (MD 0, 3)
    constexpr bool REVOK = FU_REV && (MD == 1 || MD == 2);
    static_assert(PD >= 1 && PD <= 5, "raw ring: rows k+2 .. k+1+PD in flight in 6 slots");
    using Raw = typename RawOf<Tin>::type;

    // The 4 waves of a workgroup take 4 adjacent windows of one (image, band).
    constexpr int GW = FU_THREADS / 64;             // windows per group
    constexpr int ZW = FU_ZW;
    constexpr int NPT = FU_NPT;
    auto& lut_all = sh.lut;
    auto& zl_all = sh.zl;
    auto& ptd_all = sh.ptd;
    auto& pti_all = sh.pti;
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* const lut = lut_all[wslot];
    float* zl = zl_all[PYR ? wslot : 0];
    if constexpr (PYR) {
        if (lane < 2 * O) zl[lane * ZW + 128] = 0.f;   // the zero vertex of every row block
    }
    const int ngrp = (F.nwin + GW - 1) / GW;
    const int grp = (int)(blk % ngrp);
    const int64_t rest = blk / ngrp;
    const int band = (int)(rest % F.nband);
    const int64_t b = rest / F.nband;
    if (b >= F.B) return;                         // uniform per workgroup
    const int win = grp * GW + wslot;             // may be >= nwin: runs, owns nothing
    const int W0 = win * FU_OWN - FU_HL;
    const int ce = W0 + 2 * lane;                 // this lane's even column; odd = ce + 1
    constexpr int RB = fu_rb(MD), NLUT = RB + 2;  // rows per band, u rows band_begin-1 .. +RB
    const int s0 = band * RB;                     // first output row of the band
    const int s1 = min(s0 + RB, PYR ? F.h1 : F.h2);   // PYR: the band walks conv rows
    const bool up = REVOK && (band & 1) && s1 - s0 == RB;   // uniform

    // ---- row table (fp64 lattice math, geometry_np.py:440-486) -------------
    for (int e = lane; e < NLUT; e += 64) {
        const int r = s0 - 1 + e;                 // u row
        float4 t = {0.f, 0.f, 0.f, 0.f};
        if (UIN) {
            t.y = (r >= 0 && r < F.h) ? 1.f : 0.f;    // u row r = input row r; 0: padding row
        } else if (r >= 0 && r < F.h1) {
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
    __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0): own-wave LDS writes
    __builtin_amdgcn_wave_barrier();
    // Row class of the band (uniform): RC 1 if every u row blends rect rows r-1, r
    // (table c == 0), RC 2 if rows r, r+1 (a == 0): two terms per vertical blend instead
    // of three.  A same-size lattice switches class once, in the middle band.
    int rc = 0;
    if (!UIN) {
        bool has_a = false, has_c = false;
        for (int e = lane; e < NLUT; e += 64) {
            const float4 t = lut[e];
            has_a |= t.x != 0.f;
            has_c |= t.z != 0.f;
        }
        const bool any_a = __builtin_amdgcn_ballot_w64(has_a) != 0;
        const bool any_c = __builtin_amdgcn_ballot_w64(has_c) != 0;
        rc = !any_c ? 1 : (!any_a ? 2 : 0);
    }

    // ---- per-lane column weights --------------------------------------------
    // r2h (geometry_np.py:441-449, 514-517): u[q] = sum_k wr_k[q] v[q+k], k = -1..1
    float we[3] = {0.f, 0.f, 0.f}, wo_[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2 && !UIN; ++s) {
        const int q = ce + s;
        float* wr = s ? wo_ : we;
        if (q >= 0 && q < F.w1) {
            const double j_ = axis_at(F.rys, q) + (double)(F.w - 1) * 0.5;   // :441
            const int jn = (int)j_;
            const double jf = j_ - (double)(float)jn;
#pragma unroll
            for (int k = -1; k <= 1; ++k) {
                const bool in_w = q + k >= 0 && q + k < F.w;
                if (k == jn - q && in_w) wr[k + 1] += (float)(1.0 - jf);
                if (k == jn + 1 - q && in_w) wr[k + 1] += (float)jf;
            }
        }
    }
    // h2r neighbour weights with the raster edge folded in (outside -> 0, :303-323)
    // (w2 is even, so for an owned lane z[ce+1] and z[ce] are always inside: those two
    // weights are the constant 0.25; only the outer neighbours can fall off the raster)
    const float wn_o = (ce + 2 < F.w2) ? 0.25f : 0.f;   // even row, z[b+1], b = ce+1
    const float wp_e = (ce - 1 >= 0) ? 0.25f : 0.f;     // odd row,  z[b-1], b = ce
    const bool colin = ce >= 0 && ce < F.w;           // MD 1: input columns inside (w even)
    const int bo = W0 / 2 + lane;                     // PYR: this lane's output column
    const bool own = PYR ? (lane >= FU_HL / 2 && lane < (FU_HL + FU_OWN) / 2 && bo < F.w2 &&
                            win < F.nwin)
                         : (lane >= FU_HL / 2 && lane < (FU_HL + FU_OWN) / 2 && ce >= 0 &&
                            ce < F.w2 && win < F.nwin);
    // PYR: per-lane hexresize lattice constants (geometry_np.py:570-602) on the conv image
    // (h1, w1): j_ = 0.5 i_ + y_(b) + (w1 - 0.5) / 2 per output row
    const double t_yv = PYR ? axis_at(F.tys, min(max(bo, 0), F.w2 - 1)) : 0.0;
    // PYR: every owned lane's triangle vertices (conv columns 2b - 2 .. 2b + 2, pf_lattice_ok)
    // inside the raster: the window needs no column validity tests (uniform; round 5)
    const bool pcolint = PYR && W0 >= -2 && W0 + 124 < F.w1;
    const double t_cw = ((double)F.w1 - 0.5) * 0.5;
    const double t_ch = (double)(F.h1 - 1) * 0.5;
    if constexpr (PYR) {
        for (int e = lane; e < NPT; e += 64) {
            const int a = (s0 >> 1) + e;
            const double i_ = axis_at(F.txs, min(a, F.h2 - 1)) + t_ch;   // :601 (uniform per row)
            const int i_n = (int)i_;
            ptd_all[wslot][e][0] = 0.5 * i_;
            ptd_all[wslot][e][1] = i_ - (double)(float)i_n;
            pti_all[wslot][e] = i_n;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }

    // ---- buffers: one descriptor per image, planes by per-lane offsets ---------
    const int64_t cstride = (int64_t)F.h * F.w, ostride = (int64_t)F.h2 * F.w2;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + b * C * cstride), (short)0, (int)(C * cstride * (int64_t)sizeof(Tin)), 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + b * O * ostride), (short)0, (int)(O * ostride * (int64_t)sizeof(Tout)), 0x00020000);
    const int lc = min(max(ce, 0), F.w - 2);            // clamped even load column
    // one VGPR offset per lane; the plane of a channel is an SGPR offset
    const unsigned xoff = (unsigned)lc * (unsigned)sizeof(Tin);
    const unsigned yoff = own ? (unsigned)(PYR ? bo : ce) * (unsigned)sizeof(Tout) : 0x80000000u;
    const unsigned xplane = (unsigned)(cstride * (int64_t)sizeof(Tin));
    const unsigned yplane = (unsigned)(ostride * (int64_t)sizeof(Tout));
    const unsigned xrow = (unsigned)F.w * (unsigned)sizeof(Tin);
    const unsigned yrow = (unsigned)F.w2 * (unsigned)sizeof(Tout);
    auto row_off = [&](int k) -> unsigned {             // clamped rect row (SALU)
        return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(k, 0), F.h - 1) * xrow));
    };

    // ---- weights and bias -----------------------------------------------------------
    // A VALU instruction with an SGPR (or literal) operand issues at half rate on gfx950
    // (4.2 vs 2.3 cycles per wave-instruction, tools/microbench/issue.hip) -- except the packed
    // FMA's weight operand: the first FU_WPS weight pairs are uniform loads (SGPRs), the rest
    // vector loads behind an opaque per-lane zero offset.
    int vz = 0;
    asm volatile("" : "+v"(vz));
    // MD 0: the exact same-size h2r is 0.75 z[b] + 0.25 z[b +- 1] (geometry_np.py:347-354);
    // with z' = 0.75 z it is z'[b] + z'[b +- 1] / 3, one FMA per output column instead of two
    // (fp32-rounding level difference, well inside 1e-5): the r2h column weights (u' = 0.75 u)
    // and the bias are pre-scaled, so the conv weights stay the raw uniform loads.
    constexpr bool FOLD = MD == 0;
    if (FOLD) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            we[k] *= 0.75f;
            wo_[k] *= 0.75f;
        }
    }
    constexpr int NW = O * CG * 7;
    constexpr int NWP = (NW + 1) / 2;
    constexpr int NWS = PK ? (FU_WPS < NWP ? FU_WPS : NWP) : 0;   // weight pairs in SGPRs
    float wk[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const bool uni = i / 2 < NWS;                   // uniform load -> SGPR
        wk[i] = MD == 2 ? 0.f : kern[i + (uni ? 0 : vz)];
    }
    // the weights as (even, odd)-index pairs, a tap picks its half with op_sel: the first NWS
    // pairs are the uniform loads themselves (SGPRs), the rest opaque VGPR pairs (a splat
    // weight alone would take an aligned VGPR pair of its own)
    fu_f2 wkp[NWP];
#pragma unroll
    for (int i = 0; i < NWP; ++i) {
        wkp[i] = fu_f2{wk[2 * i], 2 * i + 1 < NW ? wk[2 * i + 1] : 0.f};
        if (PK && i >= NWS) asm volatile("" : "+v"(wkp[i]));
    }
    float bv[O];
    fu_f2 bvp[(O + 1) / 2];             // bias pairs (opaque, op_sel picks the half)
#pragma unroll
    for (int o = 0; o < O; ++o) bv[o] = (MD != 2 && bias) ? bias[o + vz] * (FOLD ? 0.75f : 1.f) : 0.f;
#pragma unroll
    for (int i = 0; i < (O + 1) / 2; ++i) {
        bvp[i] = fu_f2{bv[2 * i], 2 * i + 1 < O ? bv[2 * i + 1] : 0.f};
        if (PK) asm volatile("" : "+v"(bvp[i]));
    }
    float c75 = 0.75f, c25 = 0.25f;     // h2r weights as VGPR operands, not literals
    float c13 = 1.f / 3.f;
    asm volatile("" : "+v"(c75), "+v"(c25), "+v"(c13));
    const float wn_f = wn_o != 0.f ? c13 : 0.f, wp_f = wp_e != 0.f ? c13 : 0.f;
    unsigned hi16 = 0xffff0000u;
    asm volatile("" : "+v"(hi16));

    // Column classes of the r2h horizontal taps over this wave's lanes (uniform): CD 1 if
    // every live tap is at q-1 or q, CD 2 if at q or q+1 (one DPP shift and 2 FMAs per
    // column instead of 2 and 3), CD 0 otherwise.  Same-size round trips have one
    // window of class 0 per image row (where jn - q steps from -1 to 0).
    const bool any_l = __builtin_amdgcn_ballot_w64(we[0] != 0.f || wo_[0] != 0.f) != 0;
    const bool any_r = __builtin_amdgcn_ballot_w64(we[2] != 0.f || wo_[2] != 0.f) != 0;
    const int cd = !any_r ? 1 : (!any_l ? 2 : 0);

    // A band is walked in steps k = 0 .. s1 - s0 - 1 over rows row(k): downwards (row(k) =
    // s0 + k) or, UP, upwards (row(k) = s1 - 1 - k).  Rect row / u row / conv row row(k) lives
    // in ring slot k mod 6 / k mod 3, so slots and row parities are compile-time per step of a
    // 6-step block in both directions (s0 and, for an UP band, s1 are even).
    auto run = [&](auto CDc, auto RCc, auto UPc) {
        constexpr int CD = decltype(CDc)::value;
        constexpr int RC = decltype(RCc)::value;
        constexpr bool UP = decltype(UPc)::value;
        auto row = [&](int k) { return UP ? s1 - 1 - k : s0 + k; };
        auto lut_e = [&](int j) { return UP ? RB - j : j + 1; };   // row-table entry of u row row(j)
        // ---- state -----------------------------------------------------------------
        Raw raw[6][C];                      // rect rows in flight, slot k % 6
        fu_f2 XP[3][C];                     // rect rows as f32 (even, odd) pairs, slot k % 3
        float ZE[3][O], ZO[3][O];           // MD 2: u rows (= its conv rows), slot k % 3
        fu_f2 ZP[3][O];                     // conv rows being accumulated, (even, odd) pairs

        // live false: the loads return zeros without a memory access (an offset past the buffer)
        auto issue = [&](auto SLc, int r, bool live = true) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned so = row_off(r);
            const unsigned vo = live ? xoff : 0x80000000u;
    #pragma unroll
            for (int c = 0; c < C; ++c) raw[SL][c] = fu_load<Tin>(xrs, vo, so + c * xplane);
        };
        auto convert = [&](auto RSc, auto XSc) {
            constexpr int RS = decltype(RSc)::value, XS = decltype(XSc)::value;
    #pragma unroll
            for (int c = 0; c < C; ++c) XP[XS][c] = fu_unpack2<Tin>(raw[RS][c], hi16);
        };

        // u row r = row(PH + 1) from rect rows row(PH), row(PH + 1), row(PH + 2) (slots S0, S1,
        // S2) with table entry L, scattered into conv rows row(PH + 2) (started here with the
        // bias: slot S2), row(PH + 1) (centre: S1) and row(PH) (completed here: S0).  Downwards
        // the started row is r + 1, whose 'above' row u row r is (taps 0, 1), and the completed
        // one r - 1 (taps 5, 6); upwards the other way round.
        auto urow = [&](auto PHc, float4 L, auto CENc, auto BELc) {
            constexpr int PH = decltype(PHc)::value;
            constexpr bool CEN = decltype(CENc)::value, BEL = decltype(BELc)::value;
            constexpr int S0 = fu_mod(PH, 3), S1 = fu_mod(PH + 1, 3), S2 = fu_mod(PH + 2, 3);
            constexpr int XM = UP ? S2 : S0, XQ = UP ? S0 : S2;      // slots of rect rows r - 1, r + 1
            constexpr int PB = UP ? fu_mod(PH + 1, 2) : fu_mod(PH, 2);   // parity of conv rows r -+ 1
            constexpr int PC = 1 - PB;              // parity of conv row r
            constexpr int TN = UP ? 5 : 0, TD = UP ? 0 : 5;   // first tap of the started / completed row
            float ue[C], uo[C];
            if constexpr (UIN && RC == 1) {         // interior band and window: no padding
    #pragma unroll
                for (int c = 0; c < C; ++c) {
                    ue[c] = XP[S1][c].x;
                    uo[c] = XP[S1][c].y;
                }
            } else if constexpr (UIN) {             // u = input row, 0 outside (padding 1, value 0)
                const bool in_ = colin && L.y != 0.f;
    #pragma unroll
                for (int c = 0; c < C; ++c) {
                    ue[c] = in_ ? XP[S1][c].x : 0.f;
                    uo[c] = in_ ? XP[S1][c].y : 0.f;
                }
            } else
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                float ve, vo;
                if constexpr (VPK) {                // a x[r-1] + b x[r] + c x[r+1], packed
                    const fu_f2 Lxy = {L.x, L.y}, Lzw = {L.z, L.w};
                    fu_f2 V;
                    if constexpr (RC == 1) {
                        V = fu_pfma<1, false>(Lxy, XP[S1][c], fu_pmul<0>(Lxy, XP[XM][c]));
                    } else if constexpr (RC == 2) {
                        V = fu_pfma<0, false>(Lzw, XP[XQ][c], fu_pmul<1>(Lxy, XP[S1][c]));
                    } else {
                        V = fu_pfma<0, false>(Lzw, XP[XQ][c],
                                              fu_pfma<1, false>(Lxy, XP[S1][c], fu_pmul<0>(Lxy, XP[XM][c])));
                    }
                    ve = V.x;
                    vo = V.y;
                } else if constexpr (RC == 1) {     // rect rows r-1, r
                    ve = fmaf(L.y, XP[S1][c].x, L.x * XP[XM][c].x);
                    vo = fmaf(L.y, XP[S1][c].y, L.x * XP[XM][c].y);
                } else if constexpr (RC == 2) {     // rect rows r, r+1
                    ve = fmaf(L.z, XP[XQ][c].x, L.y * XP[S1][c].x);
                    vo = fmaf(L.z, XP[XQ][c].y, L.y * XP[S1][c].y);
                } else {
                    ve = fmaf(L.z, XP[XQ][c].x, fmaf(L.y, XP[S1][c].x, L.x * XP[XM][c].x));
                    vo = fmaf(L.z, XP[XQ][c].y, fmaf(L.y, XP[S1][c].y, L.x * XP[XM][c].y));
                }
                if constexpr (CD == 1) {            // taps q-1, q
                    ue[c] = fmaf(we[1], ve, we[0] * f_prev(vo));
                    uo[c] = fmaf(wo_[1], vo, wo_[0] * ve);
                } else if constexpr (CD == 2) {     // taps q, q+1
                    ue[c] = fmaf(we[2], vo, we[1] * ve);
                    uo[c] = fmaf(wo_[2], f_next(ve), wo_[1] * vo);
                } else {
                    const float vpo = f_prev(vo), vne = f_next(ve);
                    ue[c] = fmaf(we[2], vo, fmaf(we[1], ve, we[0] * vpo));
                    uo[c] = fmaf(wo_[2], vne, fmaf(wo_[1], vo, wo_[0] * ve));
                }
            }
            if constexpr (MD == 2) {                // z row r = u row r (no conv)
    #pragma unroll
                for (int c = 0; c < C; ++c) {
                    ZE[S1][c] = ue[c];
                    ZO[S1][c] = uo[c];
                }
                return;
            } else {
                // Packed stencil: the accumulator of conv row r' is the pair (even, odd
                // column) and every tap one v_pk_fma_f32 with the weight broadcast by op_sel;
                // its u operand is the pair at column shift s: (u[ce+s], u[ce+1+s]).
                // Channel / tap indices are compile-time (fu_sfor) so every weight's register
                // file (SGPR or VGPR pair) and half are fixed in the instruction.
                fu_sfor<0, C>([&](auto Cc) {
                    constexpr int c = decltype(Cc)::value;
                    const fu_f2 U0 = {ue[c], uo[c]};
                    // only the shifts this u row's roles use are built (the rest is dead)
                    const float ne = f_next(ue[c]);
                    const fu_f2 U1 = {uo[c], ne};
                    const fu_f2 Um = {f_prev(uo[c]), ue[c]};
                    const fu_f2 U2 = {ne, OP == 0 ? f_next(uo[c]) : 0.f};
                    auto at = [&](int s) { return s == -1 ? Um : (s == 0 ? U0 : (s == 1 ? U1 : U2)); };
                    constexpr int g = c / CG, ci = c % CG;
                    fu_sfor<0, OG>([&](auto OOc) {
                        constexpr int o = g * OG + decltype(OOc)::value;
                        constexpr int j0 = (o * CG + ci) * 7;
                        // tap t: weight j0 + t is half (j0 + t) & 1 of pair (j0 + t) / 2
                        auto tap = [&](auto Tc, fu_f2& z, int par) {
                            constexpr int j = j0 + decltype(Tc)::value;
                            constexpr bool WS = (j >> 1) < NWS;
                            const fu_f2 a = at(fu_tap_shift(decltype(Tc)::value, par, OP));
                            z = fu_pfma<j & 1, WS>(wkp[j >> 1], a, z);
                        };
                        if constexpr (ci == 0) {   // the first tap of the started row adds the bias
                            constexpr int jb = j0 + TN;
                            constexpr bool WS = (jb >> 1) < NWS;
                            ZP[S2][o] = fu_pfma_b<jb & 1, o & 1, WS>(
                                wkp[jb >> 1], at(fu_tap_shift(TN, PB, OP)), bvp[o >> 1]);
                        } else {
                            tap(IC<TN>{}, ZP[S2][o], PB);
                        }
                        tap(IC<TN + 1>{}, ZP[S2][o], PB);
                        if constexpr (CEN) {
                            tap(IC<2>{}, ZP[S1][o], PC);
                            tap(IC<3>{}, ZP[S1][o], PC);
                            tap(IC<4>{}, ZP[S1][o], PC);
                        }
                        if constexpr (BEL) {
                            tap(IC<TD>{}, ZP[S0][o], PB);
                            tap(IC<TD + 1>{}, ZP[S0][o], PB);
                        }
                    });
                });
            }
        };

        // PYR: output row a of hexresize (geometry_np.py:601-678) from conv rows R0 = i_n(a)
        // and R1 = R0 + 1: R0 = 2a and R1 = 2a + 1 (Z1), or, for the one row with
        // i_n(a) = 2a + 1 (the last, host-checked: R1 is then outside the raster), R0 = Z1.
        // The triangle (:612-648): p1 = (R0, c0), p2 = (R1, c1) if i_f > j_f else
        // (R0, c0 + 1), p3 = (R1, c1 + 1), c0 = j_n - (i_n + 1) // 2, c1 = j_n - (i_n + 2) // 2;
        // c0 - 2b in {-1, 0, 1} and c1 - 2b in {-2 .. 1} (host-checked).  The vertices are read
        // from the wave's two conv rows in LDS (three ds_read_b32 per channel at per-lane
        // addresses, a zero slot for vertices outside the raster, :636-648).  Weights: the
        // barycentric coordinates in the lattice's (i, j) index frame (an affine image of the
        // reference's Cartesian frame, :651-678): (1 - i_f, i_f - j_f, j_f) if i_f > j_f, else
        // (1 - j_f, j_f - i_f, i_f).  The uniform row terms come from the band's LDS table.
        auto pyr_out = [&](const fu_f2 (&Z1)[O], int a) {
            const int e = a - (s0 >> 1);
            const double hi = ptd_all[wslot][e][0];
            const double i_f = ptd_all[wslot][e][1];
            const int i_n = __builtin_amdgcn_readfirstlane(pti_all[wslot][e]);
            const bool e1 = i_n != 2 * a;                                // uniform
            const double j_ = hi + t_yv + t_cw;                          // = 0.5 * i_ + y_ + cw (:602)
            const int j_n = (int)j_;
            const double j_f = j_ - (double)(float)j_n;
            const bool flag = i_f > j_f;
            // the same values as (flag ? 1 - i_f : 1 - j_f) and (flag ? i_f - j_f : j_f - i_f):
            // select first, subtract once (IEEE subtraction is sign-symmetric)
            const double d_ = i_f - j_f;
            const float wa = (float)(1.0 - (flag ? i_f : j_f));
            const float wb = (float)(flag ? d_ : -d_);
            const float wg = (float)(flag ? j_f : i_f);
            const int c0 = j_n - (i_n + 1) / 2, c1 = j_n - (i_n + 2) / 2;
            const bool r1in = i_n + 1 < F.h1;
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a * yrow));
            // conv row 2a + 1 next to row 2a (written at the previous step); per-lane vertex
            // addresses (window-local columns, clamped: halo lanes only), the zero vertex
            // outside the raster
            asm volatile("" ::: "memory");
    #pragma unroll
            for (int o = 0; o < O; ++o)
                *reinterpret_cast<fu_f2*>(&zl[(O + o) * ZW + 2 * lane]) = Z1[o];
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int r0b = e1 ? O * ZW : 0;
            int a1, a2, a3;
            if (pcolint) {
                // owned lanes' vertices are inside; halo lanes (outputs dropped) may read
                // past their window's row (other LDS data or zeros beyond the allocation)
                a1 = r0b + c0 - W0;
                a2 = flag ? (r1in ? O * ZW + c1 - W0 : 128) : r0b + c0 + 1 - W0;
                a3 = r1in ? O * ZW + c1 + 1 - W0 : 128;
            } else {
                // vertex validity (bitwise, no short-circuit branches)
                const bool v1 = (c0 >= 0) & (c0 < F.w1);
                const bool v2 = flag ? (r1in & (c1 >= 0) & (c1 < F.w1)) : ((c0 + 1 >= 0) & (c0 + 1 < F.w1));
                const bool v3 = r1in & (c1 + 1 >= 0) & (c1 + 1 < F.w1);
                auto col = [&](int c) { return min(max(c - W0, 0), 127); };
                a1 = v1 ? r0b + col(c0) : 128;
                a2 = v2 ? (flag ? O * ZW + col(c1) : r0b + col(c0 + 1)) : 128;
                a3 = v3 ? O * ZW + col(c1 + 1) : 128;
            }
    #pragma unroll
            for (int o = 0; o < O; ++o) {
                const float q1 = zl[a1 + o * ZW], q2 = zl[a2 + o * ZW], q3 = zl[a3 + o * ZW];
                const float z = fmaf(wg, q3, fmaf(wb, q2, wa * q1));
                if constexpr (sizeof(Tout) == 2)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (Tout)z),
                                                          yrs, yoff, so + o * yplane, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, z), yrs, yoff,
                                                          so + o * yplane, 0);
            }
        };

        // conv row row(k) (slot PH % 3) -> output row row(k) (exact same-size h2r; PYR: every
        // second conv row completes an output row of the hexresize)
        auto out_row = [&](auto PHc, int k) {
            constexpr int PH = decltype(PHc)::value;
            constexpr int S0 = PH % 3;
            constexpr int PAR = UP ? (PH + 1) & 1 : PH & 1;   // parity of output row row(k)
            if constexpr (PYR) {                    // (PYR bands walk downwards: row(k) = s0 + k)
                if constexpr ((PH & 1) == 0) {      // conv row 2a: kept in LDS for the next step
                    asm volatile("" ::: "memory");   // after the previous row's reads
    #pragma unroll
                    for (int o = 0; o < O; ++o)
                        *reinterpret_cast<fu_f2*>(&zl[o * ZW + 2 * lane]) = ZP[S0][o];
                } else {                            // conv row 2a + 1: output row a
                    pyr_out(ZP[S0], row(k) >> 1);
                }
                return;
            }
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)row(k) * yrow));
            if constexpr (FOLD && O == 3) {
                float e0 = ZP[S0][0].x, o0 = ZP[S0][0].y, e1 = ZP[S0][1].x, o1 = ZP[S0][1].y;
                float e2 = ZP[S0][2].x, o2 = ZP[S0][2].y;
                if constexpr (PAR == 0) fu_h2r3_even(e0, o0, e1, o1, e2, o2, c13, wn_f);
                else fu_h2r3_odd(e0, o0, e1, o1, e2, o2, c13, wp_f);
                fu_store<Tout>(e0, o0, yrs, yoff, so);
                fu_store<Tout>(e1, o1, yrs, yoff, so + yplane);
                fu_store<Tout>(e2, o2, yrs, yoff, so + 2 * yplane);
                return;
            }
    #pragma unroll
            for (int o = 0; o < O; ++o) {
                const float ze = PK ? ZP[S0][o].x : ZE[S0][o], zo = PK ? ZP[S0][o].y : ZO[S0][o];
                float oe, oo;
                if constexpr (MD == 1) {            // HexConv2d output row as is
                    oe = ze;
                    oo = zo;
                } else if constexpr (FOLD && PAR == 0) {   // z' = 0.75 z
                    oe = fmaf(c13, zo, ze);
                    oo = fmaf(wn_f, f_next(ze), zo);
                } else if constexpr (FOLD) {
                    oe = fmaf(wp_f, f_prev(zo), ze);
                    oo = fmaf(c13, ze, zo);
                } else if constexpr (PAR == 0) {    // 0.75 z[b] + 0.25 z[b+1]
                    oe = fmaf(c25, zo, c75 * ze);
                    oo = fmaf(wn_o, f_next(ze), c75 * zo);
                } else {                            // 0.25 z[b-1] + 0.75 z[b]
                    oe = fmaf(wp_e, f_prev(zo), c75 * ze);
                    oo = fmaf(c25, ze, c75 * zo);
                }
                fu_store<Tout>(oe, oo, yrs, yoff, so + o * yplane);
            }
        };

        // ---- prologue: u rows row(-1) and row(0) ---------------------------------------
        {
            Raw t0[C], t1[C], t2[C];
            const unsigned o0 = row_off(row(-2)), o1 = row_off(row(-1)), o2 = row_off(row(0));
            // MD 2 outputs u rows row(0) .. row(n-1) only: u row(-1) is not made, so rect row
            // row(-2) is not needed (an out-of-range load: no memory access)
            const unsigned xo0 = MD == 2 ? 0x80000000u : xoff;
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                t0[c] = fu_load<Tin>(xrs, xo0, o0 + c * xplane);
                t1[c] = fu_load<Tin>(xrs, xoff, o1 + c * xplane);
                t2[c] = fu_load<Tin>(xrs, xoff, o2 + c * xplane);
            }
            issue(IC<1>{}, row(1));
    #pragma unroll
            for (int i = 0; i < PD; ++i) {          // ring: rect rows row(2) .. row(1 + PD)
                if (i == 0) issue(IC<2>{}, row(2));
                if (i == 1) issue(IC<3>{}, row(3));
                if (i == 2) issue(IC<4>{}, row(4));
                if (i == 3) issue(IC<5>{}, row(5));
                if (i == 4) issue(IC<0>{}, row(6));
            }
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                XP[1][c] = fu_unpack2<Tin>(t0[c], hi16);   // row(-2) -> slot 1
                XP[2][c] = fu_unpack2<Tin>(t1[c], hi16);   // row(-1) -> slot 2
                XP[0][c] = fu_unpack2<Tin>(t2[c], hi16);   // row(0)  -> slot 0
            }
        }
        if constexpr (MD != 2)
            urow(IC<-2>{}, lut[lut_e(-1)], std::false_type{}, std::false_type{});   // u row(-1): start only
        convert(IC<1>{}, IC<1>{});                                              // row(1) -> slot 1
        urow(IC<-1>{}, lut[lut_e(0)], std::true_type{}, std::false_type{});     // u row(0): start, centre
        // Drain the prologue's loads: the compiler's wait counts at the loop header merge the
        // entry path with the back edge, and a ring load issued late on the entry path would
        // otherwise put a near-zero vmcnt wait into every iteration.
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)

        // ---- main loop ---------------------------------------------------------------
        const int n = s1 - s0;
        float4 lnext = lut[lut_e(1)];
        auto step = [&](auto PHc, int k) {
            constexpr int PH = decltype(PHc)::value;
            // keep each step's instructions inside the step: across a 12-step body the
            // scheduler otherwise hoists loads many steps ahead (266 VGPRs, 1 wave / SIMD)
            __builtin_amdgcn_sched_barrier(0);
            convert(IC<(PH + 2) % 6>{}, IC<(PH + 2) % 3>{});            // rect row row(k+2)
            // rows past the band's last halo row (row(n+1)) are never read: their loads go out
            // of range (no memory access) instead of fetching PD rows per band from HBM
            // (round 6; repeating row(n+1) instead, an L2 hit, measured slower)
            issue(IC<(PH + 2 + PD) % 6>{}, row(min(k + 2 + PD, n + 1)), k + 2 + PD <= n + 1);
            const float4 L = lnext;
            lnext = lut[min(max(lut_e(k + 2), 0), NLUT - 1)];
            urow(PHc, L, std::true_type{}, std::true_type{});           // u row row(k+1)
            out_row(PHc, k);
        };
        // Full blocks of six unconditional steps: an exit or a conditional store between
        // steps would let the compiler sink each rect-row load (and the last FMAs of a conv
        // row) into the rarer block that consumes them, which removes the prefetch distance
        // and serialises the accumulation.  The band's last n % 6 rows run as a tail (a
        // downward band only: upward bands are whole).  Two blocks per loop trip.
        auto block6 = [&](int base) {
            step(IC<0>{}, base);
            step(IC<1>{}, base + 1);
            step(IC<2>{}, base + 2);
            step(IC<3>{}, base + 3);
            step(IC<4>{}, base + 4);
            step(IC<5>{}, base + 5);
        };
        auto tail = [&](int base) {
            if (base >= n) return;
            step(IC<0>{}, base);
            if (base + 1 < n) {
                step(IC<1>{}, base + 1);
                if (base + 2 < n) {
                    step(IC<2>{}, base + 2);
                    if (base + 3 < n) {
                        step(IC<3>{}, base + 3);
                        if (base + 4 < n) step(IC<4>{}, base + 4);
                    }
                }
            }
        };
        int base = 0;
        for (; base + 12 <= n; base += 12) {
            block6(base);
            block6(base + 6);
        }
        if (base + 6 <= n) {
            block6(base);
            base += 6;
        }
        if constexpr (!UP) tail(base);
    };
    auto dir = [&](auto CDc, auto RCc) {
        if (REVOK && up) run(CDc, RCc, std::true_type{});
        else run(CDc, RCc, std::false_type{});
    };
    if constexpr (UIN) {
        (void)cd; (void)rc;
        // every u row of the band (s0 - 1 .. s1) and every lane's columns inside the input:
        // the padding selects drop out (RC 1 marks that loop for the u = input modes)
        const bool inner = s0 >= 1 && s1 + 1 <= F.h && __builtin_amdgcn_ballot_w64(!colin) == 0;
        if (inner) dir(IC<0>{}, IC<1>{});
        else dir(IC<0>{}, IC<0>{});
    } else {
        // the common classes get their own loop; mixed windows / bands run the generic one
        if (cd == 1 && rc == 1) dir(IC<1>{}, IC<1>{});
        else if (cd == 1 && rc == 2) dir(IC<1>{}, IC<2>{});
        else if (cd == 2 && rc == 1) dir(IC<2>{}, IC<1>{});
        else if (cd == 2 && rc == 2) dir(IC<2>{}, IC<2>{});
        else dir(IC<0>{}, IC<0>{});
    }
}

// MD 1 with 16-bit input and output fits 128 VGPRs (4 waves per SIMD); an fp32 raw ring or
// fp32 stores need more, and capping those at 128 spills to scratch inside the row loop.
template <typename Tin, typename Tout, int C, int O, int G, int OP, int MD = 0>
__global__ __launch_bounds__(FU_THREADS) __attribute__((amdgpu_waves_per_eu(
    (MD == 1 && sizeof(Tin) == 2 && sizeof(Tout) == 2) ? FU_WPE_CONV : FU_WPE)))
void k_fused(const Tin* __restrict__ x, const float* __restrict__ kern,
             const float* __restrict__ bias, Tout* __restrict__ y, FusedGeom F) {
    __shared__ FuShared<(MD >= 3), O> sh;
    fu_band<Tin, Tout, C, O, G, OP, MD>(x, kern, bias, y, F,
                                        (int64_t)xcd_swizzle(blockIdx.x, gridDim.x), sh);
}

}  // namespace hg
