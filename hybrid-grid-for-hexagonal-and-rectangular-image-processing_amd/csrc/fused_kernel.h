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
#define FU_RB_RT_ 30                  // MD 2: rows per band (66 -> 30: 0.321 -> 0.307 ms, r03 A/B)
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

// Tuning knobs (compile-time; tools/build_fvariant.sh builds variants of this file).
#ifndef FU_PD
#define FU_PD 3                       // rect rows loaded ahead of use (1..4)
#endif
#ifndef FU_WPE
#define FU_WPE 1                      // minimum waves per SIMD asked of the register allocator
#endif
#ifndef FU_WPE_CONV
#define FU_WPE_CONV 4                 // HexConv2d mode: 129 -> 128 VGPRs buys a 4th wave per SIMD
#endif
#ifndef FU_NOMEM
#define FU_NOMEM 0                    // diagnostic: every row load / store hits row 0 (cache-resident)
#endif
#ifndef FU_WSGPR
#define FU_WSGPR 0                    // 1: conv weights in SGPRs (uniform loads) instead of VGPRs
#endif
#ifndef FU_STAGE
#define FU_STAGE 0                    // 16-bit outputs: stage rows in LDS, store whole 128-B lines
#endif
#ifndef FU_SCHED
#define FU_SCHED 1                    // scheduling barrier between steps (bounds register use: with
                                      // the packed stencil 126 -> 120 VGPRs, 2.92 -> 2.76 ms A/B)
#endif
#ifndef FU_CD
#define FU_CD 1                       // per-wave column-class specialisation of the r2h taps
#endif
#ifndef FU_L12
#define FU_L12 1                      // 12-step loop body (two 6-step blocks per trip)
#endif
#ifndef FU_MIN_INST
#define FU_MIN_INST 0                 // 1: build only the bf16 C3 O3 G1 kernels (variants)
#endif
#ifndef FU_DRAIN
#define FU_DRAIN 1                    // drain the prologue's loads before the row loop
#endif
#ifndef FU_RC
#define FU_RC 1                       // per-band row-class specialisation of the r2h rows
#endif
#ifndef FU_FOLD
#define FU_FOLD 1                     // MD 0: the h2r 0.75 folded into the conv weights
#endif
#ifndef FU_PK
#define FU_PK 1                       // 7-tap stencil as v_pk_fma_f32 on (even, odd) column pairs
#endif
#ifndef FU_WPS
#define FU_WPS 21                     // PK: the first FU_WPS weight pairs live in SGPRs (v_pk_fma_f32
                                      // reads an SGPR operand at full rate, unlike v_fmac_f32), the
                                      // rest in VGPRs; 21 of 32 keeps both register files unspilled
#endif
#ifndef FU_BIAS_INIT
#define FU_BIAS_INIT 0                // debugging: bias as the accumulator's start value
#endif
#ifndef FU_ONE_CLASS
#define FU_ONE_CLASS 0                // ISA inspection: instantiate only the (CD 1, RC 1) loop
#endif
#ifndef FU_VPK
#define FU_VPK 1                      // PK: the r2h vertical blend as v_pk_mul/fma_f32 on the
                                      // (even, odd) rect pair, row weights broadcast by op_sel
#endif
#ifndef FU_PLDS
#define FU_PLDS 1                     // MD 3 / 4: the triangle vertices read from the wave's two
                                      // conv rows in LDS (3 ds_read_b32 per channel at per-lane
                                      // addresses) instead of 5 DPP moves + 9 selects per channel
#endif
#ifndef FU_PTAB
#define FU_PTAB 1                     // MD 3 / 4 / 5: the output rows' uniform lattice terms (0.5 i_,
                                      // i_f, i_n) from a per-band LDS table instead of fp64 VALU per
                                      // output row; weights selected before subtracting (round 5)
#endif
#ifndef FU_FMIX
#define FU_FMIX 0                     // MD 3, fp16 input: the r2h vertical blend as v_fma_mix_f32 on the
                                      // raw f16 rows (no conversion pass; the same products and sums):
                                      // 118 -> 96 VGPRs, 5 waves per SIMD, but level 0 within 0.7 %
                                      // (profiles/r05/pyramid_fmix_ab.txt): off
#endif
#ifndef FU_WPE_FMIX
#define FU_WPE_FMIX 5                 // MD 3 with FMIX: the raw f16 ring leaves room for a 5th wave
#endif
#ifndef FU_PCOLINT
#define FU_PCOLINT 1                  // MD 3 / 4 / 5: windows whose owned vertices are all inside the
                                      // raster skip the per-vertex column tests (round 5)
#endif
#ifndef FU_DMA
#define FU_DMA 0                      // MD 0, 16-bit input: rect rows arrive by LDS-DMA as
                                      // workgroup-wide 1-KiB row pieces (one per plane, issued by
                                      // waves 0..C-1), a ring of rows in LDS, one s_barrier per step
#endif
#ifndef FU_DMA_ST
#define FU_DMA_ST 1                   // with FU_DMA and 16-bit outputs: output rows staged in LDS
                                      // and stored as the workgroup's 960-B row pieces (16-B lanes)
#endif
#ifndef FU_DPD
#define FU_DPD 3                      // with FU_DMA: rect rows in flight ahead of the one read
#endif
#ifndef FU_ORDER
#define FU_ORDER 0                    // workgroup -> (window group, band, image) order (A/B
                                      // variants; 0: group fastest, then band, then image)
#endif
#ifndef FU_LAUX
#define FU_LAUX 0                     // cache-policy bits of the row loads / stores (A/B variants)
#endif
#ifndef FU_SAUX
#define FU_SAUX 0
#endif
#ifndef FU_ODPP
#define FU_ODPP 1                     // MD 0: the h2r neighbour term as one v_fmac_f32_dpp
#endif
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
        return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, FU_LAUX);
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
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, p), rs, voff, soff, FU_SAUX);
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
// d = a * f16(half HI of b) + c in fp32 (v_fma_mix_f32: the f16 operand converts exactly, one
// rounding: the same value as fmaf(a, (float)h, c))
template <int HI>
__device__ __forceinline__ float fu_fmix(float a, unsigned b, float c) {
    float d;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
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
// MD 1; MD 5 = MD 4 on shorter bands, for levels too small to fill the chip).  Every second step completes the two conv rows an output row's triangles read; a
// window of 128 input columns owns 60 output columns (lane l <-> output column W0/2 + l).
template <typename Tin, typename Tout, int C, int O, int G, int OP, int MD = 0>
// MD 1 with 16-bit input and output fits 128 VGPRs (4 waves per SIMD); an fp32 raw ring or
// fp32 stores need more, and capping those at 128 spills to scratch inside the row loop.
__global__ __launch_bounds__(FU_THREADS) __attribute__((amdgpu_waves_per_eu(
    (MD == 1 && sizeof(Tin) == 2 && sizeof(Tout) == 2) ? FU_WPE_CONV
    : (MD == 3 && FU_FMIX && std::is_same<Tin, _Float16>::value) ? FU_WPE_FMIX : FU_WPE)))
void k_fused(const Tin* __restrict__ x,
                                                      const float* __restrict__ kern,
                                                      const float* __restrict__ bias,
                                                      Tout* __restrict__ y, FusedGeom F) {
    constexpr int CG = C / G, OG = O / G;
    constexpr int PD = FU_PD;
    constexpr bool PYR = MD >= 3;                 // hex-pyramid level (hexresize output stage)
    constexpr bool UIN = MD == 1 || MD >= 4;      // u rows = input rows (no r2h)
    constexpr bool VPK = FU_VPK && FU_PK && MD != 2 && !UIN;
    static_assert(PD >= 1 && PD <= 5, "raw ring: rows a2+2 .. a2+1+PD in flight in 6 slots");
    using Raw = typename RawOf<Tin>::type;

    // The 4 waves of a workgroup take 4 adjacent windows of one (image, band): a group
    // of FU_GRP owned columns.  With STAGE, output rows go through LDS and the group
    // stores them as aligned 128-B lines (a window's 240 owned bytes are not line
    // aligned; partial-line stores cost ~20 % of HBM throughput, tools/microbench/walk2).
    constexpr bool STAGE = FU_STAGE && sizeof(Tout) == 2;
    constexpr int GW = FU_THREADS / 64;             // windows per group
    constexpr int GDW = GW * FU_OWN / 2;            // dwords of one output row of a group
    // DMA: ring of NSR rect rows, each C planes x the group's 1-KiB span (columns
    // grp * GW * FU_OWN - 8 .. + 511); DST: two output rows, O planes x 256 dwords.  With DMA
    // the row tables, the ring and the staged rows share ONE __shared__ array: LDS accesses
    // to a second __shared__ object make hipcc wait vmcnt(0) for every LDS-DMA in flight.
    // P: 1-KiB pieces per plane row of the group (GW windows of FU_OWN columns + halo)
    constexpr int DP = (GW * FU_OWN + 16 + 511) / 512;
    // (MD 0 and the pyramid levels MD 3 / 4 / 5; FU_DMA = 2: the pyramid levels only)
    constexpr bool DMA = (FU_DMA == 1 ? (MD == 0 || MD >= 3) : FU_DMA == 2 ? MD >= 3 : false) &&
                         sizeof(Tin) == 2 && GW >= C * DP;
    constexpr bool DST = DMA && MD == 0 && FU_DMA_ST && sizeof(Tout) == 2 && GW >= O * DP;
    constexpr int DPD = FU_DPD, NSR = DPD + 6;
    static_assert(!(DMA && (FU_STAGE || FU_NOMEM)), "FU_DMA replaces FU_STAGE / FU_NOMEM");
    constexpr int DLUT = GW * FU_LUT * 16, DRING = NSR * C * DP * 1024, DSTGB = DST ? 2 * O * DP * 1024 : 0;
    __shared__ __attribute__((aligned(16))) unsigned char dsm[DMA ? DLUT + DRING + DSTGB : 16];
    unsigned char* const dring = dsm + DLUT;
    // the ring's LDS byte address (the M0 base of an LDS-DMA), from the array itself
    const unsigned dring_lds =
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)dsm + (unsigned)DLUT;
    unsigned* const dstg = reinterpret_cast<unsigned*>(dsm + DLUT + DRING);
    // per-wave u-row table {a, b, c, -}: u[r] = a*x[r-1] + b*x[r] + c*x[r+1]
    __shared__ float4 lut_all[DMA ? 1 : GW][FU_LUT];
    __shared__ unsigned stg[STAGE ? 2 : 1][STAGE ? 6 : 1][STAGE ? O : 1][STAGE ? GDW + 4 : 1];
    // PLDS: the two conv rows an output row reads, per wave: [row][channel][col], cols
    // 0..127 of the window + a zero at 128 (vertices outside the raster) and a pad
    constexpr bool PLDS = FU_PLDS && PYR;
    constexpr int ZW = 130;
    __shared__ float zl_all[PLDS ? GW : 1][PLDS ? 2 * O * ZW : 1];
    // PTAB: per output row of the band {0.5 i_, i_f} and i_n (geometry_np.py:601-612)
    constexpr bool PTAB = FU_PTAB && PYR;
    constexpr int NPT = FU_RB_PYR / 2 + 1;
    __shared__ double ptd_all[PTAB ? GW : 1][PTAB ? NPT : 1][2];
    __shared__ int pti_all[PTAB ? GW : 1][PTAB ? NPT : 1];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* lut = DMA ? reinterpret_cast<float4*>(dsm) + wslot * FU_LUT : lut_all[DMA ? 0 : wslot];
    float* zl = zl_all[PLDS ? wslot : 0];
    if constexpr (PLDS) {
        if (lane < 2 * O) zl[lane * ZW + 128] = 0.f;   // the zero vertex of every row block
    }
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (F.nwin + GW - 1) / GW;
    const int grp = (int)(blk % ngrp);
    int64_t rest = blk / ngrp;
    if (FU_ORDER == 3) {   // scrambled (band, image) index (40503 is prime to 52 x 128)
        const int64_t n = (int64_t)F.nband * F.B;
        rest = (rest * 40503 + 12345) % n;
    }
    const int band = (int)(FU_ORDER == 4 ? rest / F.B : rest % F.nband);
    const int64_t b = FU_ORDER == 4 ? rest % F.B : rest / F.nband;
    if (b >= F.B) return;                         // uniform per workgroup
    const int win = grp * GW + wslot;             // may be >= nwin: runs, owns nothing
    const int W0 = win * FU_OWN - FU_HL;
    const int ce = W0 + 2 * lane;                 // this lane's even column; odd = ce + 1
    constexpr int RB = fu_rb(MD), NLUT = RB + 2;  // rows per band, u rows band_begin-1 .. +RB
    const int s0 = band * RB;                     // first output row of the band
    const int s1 = min(s0 + RB, PYR ? F.h1 : F.h2);   // PYR: the band walks conv rows

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
    if (!UIN && FU_RC) {
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
    const bool pcolint = PYR && FU_PCOLINT && W0 >= -2 && W0 + 124 < F.w1;
    const double t_cw = ((double)F.w1 - 0.5) * 0.5;
    const double t_ch = (double)(F.h1 - 1) * 0.5;
    if constexpr (PTAB) {
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
    // staging slot of this lane's two output columns (non-owned lanes write a pad dword)
    const int sidx = (lane >= FU_HL / 2 && lane < (FU_HL + FU_OWN) / 2)
                         ? wslot * (FU_OWN / 2) + lane - FU_HL / 2 : GDW + (lane & 3);

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
        if (FU_NOMEM) return 0u;
        return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(k, 0), F.h - 1) * xrow));
    };
    // DMA: the group's span of a rect row starts 8 columns left of the group (16-B aligned)
    // and is DP 1-KiB pieces; wave j < C * DP moves piece j % DP of plane j / DP, lane l 8
    // columns (16 B) of it; columns outside the raster read as zeros
    const int dcol0 = grp * GW * FU_OWN - 8;
    const int dpl = wslot / DP, dpp = wslot % DP;      // this wave's plane / piece
    const int dgc = dcol0 + dpp * 512 + 8 * lane;
    const unsigned dvoff = (dgc >= 0 && dgc < F.w) ? (unsigned)dgc * 2u : 0x80000000u;
    const int dlcol = 2 * (ce - dcol0);                 // this lane's column pair in the span
    // DST: wave j < O * DP stores part j % DP (960 owned bytes, 16 B per lane) of plane j / DP
    // of the group's output row
    const int dscol = grp * GW * FU_OWN + dpp * 480 + 8 * lane;
    const unsigned dsoff = (lane < 60 && dscol < F.w2) ? (unsigned)dscol * 2u : 0x80000000u;
    // a part whose last 16-B piece crosses the raster's right edge (w2 % 8 != 0) stores as dwords
    const bool dedge = (F.w2 & 7) != 0 && grp * GW * FU_OWN + dpp * 480 < F.w2 &&
                       grp * GW * FU_OWN + dpp * 480 + 480 > F.w2;
    // this lane's dword in a staged output row (pad dwords past the owned ones otherwise)
    const int dsidx = (lane >= FU_HL / 2 && lane < (FU_HL + FU_OWN) / 2)
                          ? wslot * (FU_OWN / 2) + lane - FU_HL / 2 : GW * (FU_OWN / 2) + (lane & 3);

    // ---- weights and bias in VGPRs -------------------------------------------------
    // A VALU instruction with an SGPR (or literal) operand issues at half rate on gfx950
    // (4.2 vs 2.3 cycles per wave-instruction, tools/microbench/issue.hip), so every
    // FMA operand is a VGPR: an opaque per-lane zero offset makes these vector loads.
    int vz = 0;
    asm volatile("" : "+v"(vz));
    // MD 0 with FU_FOLD: the exact same-size h2r is 0.75 z[b] + 0.25 z[b +- 1]
    // (geometry_np.py:347-354); with z' = 0.75 z it is z'[b] + z'[b +- 1] / 3, one FMA per
    // output column instead of two (fp32-rounding level difference, well inside 1e-5).  The
    // scalar stencil pre-scales the conv weights and the bias; the packed one scales the r2h
    // column weights (u' = 0.75 u) and the bias, so its conv weights stay the raw uniform
    // loads that live in SGPRs.
    constexpr bool FOLD = FU_FOLD && MD == 0;
    constexpr bool PKW = FU_PK && MD != 2;
    const float ws_ = (FOLD && !PKW) ? 0.75f : 1.f;
    if (FOLD && PKW) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            we[k] *= 0.75f;
            wo_[k] *= 0.75f;
        }
    }
    constexpr int NW = O * CG * 7;
    constexpr int NWP = (NW + 1) / 2;
    constexpr int NWS = PKW ? (FU_WPS < NWP ? FU_WPS : NWP) : 0;   // PK: weight pairs in SGPRs
    float wk[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const bool uni = FU_WSGPR || i / 2 < NWS;          // uniform load -> SGPR
        wk[i] = MD == 2 ? 0.f : kern[i + (uni ? 0 : vz)] * ws_;
    }
    // PK: the weights as (even, odd)-index pairs, a tap picks its half with op_sel: the
    // first NWS pairs are the uniform loads themselves (SGPRs), the rest opaque VGPR pairs
    // (a splat weight alone would take an aligned VGPR pair of its own)
    fu_f2 wkp[NWP];
#pragma unroll
    for (int i = 0; i < NWP; ++i) {
        wkp[i] = fu_f2{wk[2 * i], 2 * i + 1 < NW ? wk[2 * i + 1] : 0.f};
        if (PKW && i >= NWS) asm volatile("" : "+v"(wkp[i]));
    }
    float bv[O];
    fu_f2 bvp[(O + 1) / 2];             // PK: bias pairs (opaque, op_sel picks the half)
#pragma unroll
    for (int o = 0; o < O; ++o) bv[o] = (MD != 2 && bias) ? bias[o + vz] * (FOLD ? 0.75f : 1.f) : 0.f;
#pragma unroll
    for (int i = 0; i < (O + 1) / 2; ++i) {
        bvp[i] = fu_f2{bv[2 * i], 2 * i + 1 < O ? bv[2 * i + 1] : 0.f};
        if (PKW) asm volatile("" : "+v"(bvp[i]));
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
    const int cd = !FU_CD ? 0 : (!any_r ? 1 : (!any_l ? 2 : 0));

    auto run = [&](auto CDc, auto RCc) {
        constexpr int CD = decltype(CDc)::value;
        constexpr int RC = decltype(RCc)::value;
        // ---- state -----------------------------------------------------------------
        Raw raw[6][C];                      // rect rows in flight, slot (row - s0) % 6
        Raw rawn[C];                        // DMA: the next rect row, read from the LDS ring
        fu_f2 XP[3][C];                     // rect rows as f32 (even, odd) pairs, slot (row - s0) % 3
        // FMIX: the rect rows stay raw (two f16 per lane) and the vertical blend reads them with
        // v_fma_mix_f32 (MD 3 from an fp16 rect image, register ring only)
        constexpr bool FMIX = FU_FMIX && MD == 3 && !DMA && std::is_same<Tin, _Float16>::value;
        Raw XR[3][C];
        auto xset = [&](auto XSc, int c, Raw r) {
            constexpr int XS = decltype(XSc)::value;
            if constexpr (FMIX) XR[XS][c] = r;
            else XP[XS][c] = fu_unpack2<Tin>(r, hi16);
        };
        float ZE[3][O], ZO[3][O];           // conv rows being accumulated, slot (row - s0) % 3
        constexpr bool PK = FU_PK && MD != 2;
        static_assert(PK || !PYR, "the pyramid modes use the packed stencil");
        fu_f2 ZP[3][O];                     // PK: the same rows as (even, odd) pairs
        fu_f2 ZK[PYR ? O : 1];              // PYR: conv row 2a, kept for output row a

        auto issue = [&](auto SLc, int k) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned so = row_off(k);
    #pragma unroll
            for (int c = 0; c < C; ++c) raw[SL][c] = fu_load<Tin>(xrs, xoff, so + c * xplane);
        };
        auto convert = [&](auto RSc, auto XSc) {
            constexpr int RS = decltype(RSc)::value, XS = decltype(XSc)::value;
    #pragma unroll
            for (int c = 0; c < C; ++c) xset(IC<XS>{}, c, raw[RS][c]);
        };
        // DMA: rect row R lives in ring slot (R - s0 + 2) % NSR; waves 0 .. C-1 each move one
        // plane's 1-KiB piece of it (uniform branch), every wave reads its column pair
        auto dslot = [&](int R) { return (R - s0 + 2) % NSR; };
        // (inline asm: hipcc does not see these loads, so it inserts no vmcnt(0) before the
        // kernel's other LDS accesses; the waits are counted by hand below)
        auto dma_row = [&](int R) {
            if (wslot < C * DP) {
                const unsigned so = row_off(R) + (unsigned)dpl * xplane;
                const unsigned lda = dring_lds + (unsigned)(((dslot(R) * C + dpl) * DP + dpp) * 1024);
                unsigned keep;
                const unsigned vo = dvoff;          // (asm operands: locals of this lambda)
                const __amdgpu_buffer_rsrc_t rs = xrs;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                             "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(vo), "s"(rs), "s"(lda), "s"(so) : "memory");
            }
        };
        auto read_row = [&](int R, Raw (&r)[C]) {
            const unsigned char* const src = dring + dslot(R) * C * DP * 1024 + dlcol;
    #pragma unroll
            for (int c = 0; c < C; ++c) r[c] = *reinterpret_cast<const Raw*>(src + c * DP * 1024);
        };
        // DST: output row R (staged at the previous step, buffer R & 1) as the group's 960-B
        // pieces, wave o storing plane o; `valid` false: a dropped store (keeps the wait count)
        auto dst_store = [&](int R, bool valid) {
            if (wslot < O * DP) {
                const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)max(R, 0) * yrow)) +
                                    (unsigned)dpl * yplane;
                const unsigned* const src =
                    dstg + ((R & 1) * O + dpl) * DP * 256 + dpp * 240 + 4 * min(lane, 59);
                if (!dedge) {
                    const hg_u4v q = *reinterpret_cast<const hg_u4v*>(src);
                    hg_store_b128(q, yrs, valid ? dsoff : 0x80000000u, so);
                } else {   // the row end crosses a 16-B piece: dword stores, column-checked
    #pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const bool in_ = valid && lane < 60 && dscol + 2 * i < F.w2;
                        __builtin_amdgcn_raw_buffer_store_b32(src[i], yrs,
                                                              in_ ? (unsigned)(dscol + 2 * i) * 2u : 0x80000000u,
                                                              so, 0);
                    }
                }
            }
        };

        // u row r (= s0 + PH + 1) from rect rows r-1, r, r+1 (ring slots PH, PH+1, PH+2
        // mod 3) with table entry L, scattered into conv rows r+1 (above role; slot
        // PH+2, started with the bias), r (centre; slot PH+1) and r-1 (below; slot PH).
        auto urow = [&](auto PHc, float4 L, auto CENc, auto BELc) {
            constexpr int PH = decltype(PHc)::value;
            constexpr bool CEN = decltype(CENc)::value, BEL = decltype(BELc)::value;
            constexpr int S0 = fu_mod(PH, 3), S1 = fu_mod(PH + 1, 3), S2 = fu_mod(PH + 2, 3);
            constexpr int PB = fu_mod(PH, 2);       // parity of conv row r-1 (and r+1)
            constexpr int PC = 1 - PB;              // parity of conv row r
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
                if constexpr (FMIX) {               // the same products and sums on the raw f16 rows
                    float m0 = -0.f;                // x * y + (-0) = x * y exactly (signed zeros too)
                    asm volatile("" : "+v"(m0));
                    const Raw r0 = XR[S0][c], r1 = XR[S1][c], r2 = XR[S2][c];
                    if constexpr (RC == 1) {
                        ve = fu_fmix<0>(L.y, r1, fu_fmix<0>(L.x, r0, m0));
                        vo = fu_fmix<1>(L.y, r1, fu_fmix<1>(L.x, r0, m0));
                    } else if constexpr (RC == 2) {
                        ve = fu_fmix<0>(L.z, r2, fu_fmix<0>(L.y, r1, m0));
                        vo = fu_fmix<1>(L.z, r2, fu_fmix<1>(L.y, r1, m0));
                    } else {
                        ve = fu_fmix<0>(L.z, r2, fu_fmix<0>(L.y, r1, fu_fmix<0>(L.x, r0, m0)));
                        vo = fu_fmix<1>(L.z, r2, fu_fmix<1>(L.y, r1, fu_fmix<1>(L.x, r0, m0)));
                    }
                } else if constexpr (VPK) {         // the same products and sums, packed
                    const fu_f2 Lxy = {L.x, L.y}, Lzw = {L.z, L.w};
                    fu_f2 V;
                    if constexpr (RC == 1) {
                        V = fu_pfma<1, false>(Lxy, XP[S1][c], fu_pmul<0>(Lxy, XP[S0][c]));
                    } else if constexpr (RC == 2) {
                        V = fu_pfma<0, false>(Lzw, XP[S2][c], fu_pmul<1>(Lxy, XP[S1][c]));
                    } else {
                        V = fu_pfma<0, false>(Lzw, XP[S2][c],
                                              fu_pfma<1, false>(Lxy, XP[S1][c], fu_pmul<0>(Lxy, XP[S0][c])));
                    }
                    ve = V.x;
                    vo = V.y;
                } else if constexpr (RC == 1) {     // rect rows r-1, r
                    ve = fmaf(L.y, XP[S1][c].x, L.x * XP[S0][c].x);
                    vo = fmaf(L.y, XP[S1][c].y, L.x * XP[S0][c].y);
                } else if constexpr (RC == 2) {     // rect rows r, r+1
                    ve = fmaf(L.z, XP[S2][c].x, L.y * XP[S1][c].x);
                    vo = fmaf(L.z, XP[S2][c].y, L.y * XP[S1][c].y);
                } else {
                    ve = fmaf(L.z, XP[S2][c].x, fmaf(L.y, XP[S1][c].x, L.x * XP[S0][c].x));
                    vo = fmaf(L.z, XP[S2][c].y, fmaf(L.y, XP[S1][c].y, L.x * XP[S0][c].y));
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
            }
            if constexpr (PK) {
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
                        if constexpr (ci == 0 && FU_BIAS_INIT) {   // accumulator starts at the bias
                            ZP[S2][o] = fu_f2{bv[o], bv[o]};
                            tap(IC<0>{}, ZP[S2][o], PB);
                        } else if constexpr (ci == 0) {   // the first tap of conv row r+1 adds the bias
                            constexpr bool WS = (j0 >> 1) < NWS;
                            ZP[S2][o] = fu_pfma_b<j0 & 1, o & 1, WS>(
                                wkp[j0 >> 1], at(fu_tap_shift(0, PB, OP)), bvp[o >> 1]);
                        } else {
                            tap(IC<0>{}, ZP[S2][o], PB);
                        }
                        tap(IC<1>{}, ZP[S2][o], PB);
                        if constexpr (CEN) {
                            tap(IC<2>{}, ZP[S1][o], PC);
                            tap(IC<3>{}, ZP[S1][o], PC);
                            tap(IC<4>{}, ZP[S1][o], PC);
                        }
                        if constexpr (BEL) {
                            tap(IC<5>{}, ZP[S0][o], PB);
                            tap(IC<6>{}, ZP[S0][o], PB);
                        }
                    });
                });
                return;
            }
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                // u at column offsets -1 .. 2 of each of the lane's two columns
                const float pe = f_prev(uo[c]);     // even col - 1
                const float ne = f_next(ue[c]);     // odd col + 1 (= even col + 2)
                const float no = OP == 0 ? f_next(uo[c]) : 0.f;   // odd col + 2
                auto at_e = [&](int s) { return s == -1 ? pe : (s == 0 ? ue[c] : (s == 1 ? uo[c] : ne)); };
                auto at_o = [&](int s) { return s == -1 ? ue[c] : (s == 0 ? uo[c] : (s == 1 ? ne : no)); };
                const int g = c / CG, ci = c % CG;
    #pragma unroll
                for (int oo = 0; oo < OG; ++oo) {
                    const int o = g * OG + oo;
                    const float* w = &wk[(o * CG + ci) * 7];
                    // above role (taps with ii == 0) of conv row r+1, parity PB
    #pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int s = fu_tap_shift(t, PB, OP);
                        if (ci == 0 && t == 0) {
                            ZE[S2][o] = fmaf(w[t], at_e(s), bv[o]);
                            ZO[S2][o] = fmaf(w[t], at_o(s), bv[o]);
                        } else {
                            ZE[S2][o] = fmaf(w[t], at_e(s), ZE[S2][o]);
                            ZO[S2][o] = fmaf(w[t], at_o(s), ZO[S2][o]);
                        }
                    }
                    if constexpr (CEN) {
    #pragma unroll
                        for (int t = 2; t < 5; ++t) {
                            const int s = fu_tap_shift(t, PC, OP);
                            ZE[S1][o] = fmaf(w[t], at_e(s), ZE[S1][o]);
                            ZO[S1][o] = fmaf(w[t], at_o(s), ZO[S1][o]);
                        }
                    }
                    if constexpr (BEL) {
    #pragma unroll
                        for (int t = 5; t < 7; ++t) {
                            const int s = fu_tap_shift(t, PB, OP);
                            ZE[S0][o] = fmaf(w[t], at_e(s), ZE[S0][o]);
                            ZO[S0][o] = fmaf(w[t], at_o(s), ZO[S0][o]);
                        }
                    }
                }
            }
        };

        // PYR: output row a of hexresize (geometry_np.py:601-678) from conv rows R0 = i_n(a)
        // and R1 = R0 + 1: R0 = 2a (ZK) and R1 = 2a + 1 (Z1), or, for the one row with
        // i_n(a) = 2a + 1 (the last, host-checked: R1 is then outside the raster), R0 = Z1.
        // The triangle (:612-648): p1 = (R0, c0), p2 = (R1, c1) if i_f > j_f else
        // (R0, c0 + 1), p3 = (R1, c1 + 1), c0 = j_n - (i_n + 1) // 2, c1 = j_n - (i_n + 2) // 2;
        // c0 - 2b in {-1, 0, 1} and c1 - 2b in {-2 .. 1} (host-checked), so each vertex is
        // the lane's own conv value or a neighbour lane's, picked with selects; vertices
        // outside the raster read 0 (:636-648).  Weights: the barycentric coordinates in the
        // lattice's (i, j) index frame (an affine image of the reference's Cartesian frame,
        // :651-678): (1 - i_f, i_f - j_f, j_f) if i_f > j_f, else (1 - j_f, j_f - i_f, i_f).
        auto pyr_out = [&](const fu_f2 (&Z1)[O], int a) {
            double hi, i_f;
            int i_n;
            if constexpr (PTAB) {                                       // the band's table (uniform)
                const int e = a - (s0 >> 1);
                hi = ptd_all[wslot][e][0];
                i_f = ptd_all[wslot][e][1];
                i_n = __builtin_amdgcn_readfirstlane(pti_all[wslot][e]);
            } else {
                const double i_ = axis_at(F.txs, a) + t_ch;              // uniform
                i_n = __builtin_amdgcn_readfirstlane((int)i_);
                i_f = i_ - (double)(float)i_n;
                hi = 0.5 * i_;
            }
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
            const int d0 = c0 - 2 * bo, d1 = c1 - 2 * bo;
            const bool r1in = i_n + 1 < F.h1;
            // vertex validity (bitwise, no short-circuit branches; only the clamped-column
            // paths below need it)
            auto vflags = [&](bool& v1, bool& v2, bool& v3) {
                v1 = (c0 >= 0) & (c0 < F.w1);
                v2 = flag ? (r1in & (c1 >= 0) & (c1 < F.w1)) : ((c0 + 1 >= 0) & (c0 + 1 < F.w1));
                v3 = r1in & (c1 + 1 >= 0) & (c1 + 1 < F.w1);
            };
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a * yrow));
            if constexpr (PLDS) {
                // conv row 2a + 1 next to row 2a (written at the previous step); per-lane
                // vertex addresses (window-local columns, clamped: halo lanes only), the
                // zero vertex outside the raster; the same arithmetic as below
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
                    bool v1, v2, v3;
                    vflags(v1, v2, v3);
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
                return;
            }
            bool v1, v2, v3;
            vflags(v1, v2, v3);
    #pragma unroll
            for (int o = 0; o < O; ++o) {
                const fu_f2 z0 = e1 ? Z1[o] : ZK[o], z1 = Z1[o];
                const float y0pm = f_prev(z0.y), y0ne = f_next(z0.x);
                const float y1pe = f_prev(z1.x), y1po = f_prev(z1.y), y1ne = f_next(z1.x);
                const float p1 = d0 < 0 ? y0pm : (d0 == 0 ? z0.x : z0.y);
                const float p2a = d0 < 0 ? z0.x : (d0 == 0 ? z0.y : y0ne);
                const float p2b = d1 < -1 ? y1pe : (d1 == -1 ? y1po : (d1 == 0 ? z1.x : z1.y));
                const float p3 = d1 < -1 ? y1po : (d1 == -1 ? z1.x : (d1 == 0 ? z1.y : y1ne));
                const float q1 = v1 ? p1 : 0.f;
                const float q2 = v2 ? (flag ? p2b : p2a) : 0.f;
                const float q3 = v3 ? p3 : 0.f;
                const float z = fmaf(wg, q3, fmaf(wb, q2, wa * q1));
                if constexpr (sizeof(Tout) == 2)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (Tout)z),
                                                          yrs, yoff, so + o * yplane, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, z), yrs, yoff,
                                                          so + o * yplane, 0);
            }
        };

        // conv row a2 (slot PH % 3, parity PH % 2) -> output row a2 (exact same-size h2r)
        auto out_row = [&](auto PHc, auto SBc, int a2) {
            constexpr int PH = decltype(PHc)::value;
            constexpr int SB = STAGE ? decltype(SBc)::value : 0;
            constexpr int S0 = PH % 3;
            if constexpr (PYR) {
                if constexpr ((PH & 1) == 0) {      // conv row 2a: kept for the next step
                    if constexpr (PLDS) {
                        asm volatile("" ::: "memory");   // after the previous row's reads
    #pragma unroll
                        for (int o = 0; o < O; ++o)
                            *reinterpret_cast<fu_f2*>(&zl[o * ZW + 2 * lane]) = ZP[S0][o];
                    } else {
    #pragma unroll
                        for (int o = 0; o < O; ++o) ZK[o] = ZP[S0][o];
                    }
                } else {                            // conv row 2a + 1: output row a
                    pyr_out(ZP[S0], a2 >> 1);
                }
                return;
            }
            const unsigned so = FU_NOMEM ? 0u : (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a2 * yrow));
            if constexpr (FU_ODPP && FOLD && PK && O == 3 && !STAGE) {
                float e0 = ZP[S0][0].x, o0 = ZP[S0][0].y, e1 = ZP[S0][1].x, o1 = ZP[S0][1].y;
                float e2 = ZP[S0][2].x, o2 = ZP[S0][2].y;
                if constexpr ((PH & 1) == 0) fu_h2r3_even(e0, o0, e1, o1, e2, o2, c13, wn_f);
                else fu_h2r3_odd(e0, o0, e1, o1, e2, o2, c13, wp_f);
                if constexpr (DST) {                // staged: stored at the next step
                    typedef Tout t2v __attribute__((ext_vector_type(2)));
                    unsigned* const d = dstg + (a2 & 1) * O * DP * 256 + dsidx;
                    d[0] = __builtin_bit_cast(unsigned, t2v{(Tout)e0, (Tout)o0});
                    d[DP * 256] = __builtin_bit_cast(unsigned, t2v{(Tout)e1, (Tout)o1});
                    d[2 * DP * 256] = __builtin_bit_cast(unsigned, t2v{(Tout)e2, (Tout)o2});
                    return;
                }
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
                } else if constexpr (FOLD && (PH & 1) == 0) {   // z' = 0.75 z
                    oe = fmaf(c13, zo, ze);
                    oo = fmaf(wn_f, f_next(ze), zo);
                } else if constexpr (FOLD) {
                    oe = fmaf(wp_f, f_prev(zo), ze);
                    oo = fmaf(c13, ze, zo);
                } else if constexpr ((PH & 1) == 0) {      // 0.75 z[b] + 0.25 z[b+1]
                    oe = fmaf(c25, zo, c75 * ze);
                    oo = fmaf(wn_o, f_next(ze), c75 * zo);
                } else {                            // 0.25 z[b-1] + 0.75 z[b]
                    oe = fmaf(wp_e, f_prev(zo), c75 * ze);
                    oo = fmaf(c25, ze, c75 * zo);
                }
                    if constexpr (DST) {
                    typedef Tout t2v __attribute__((ext_vector_type(2)));
                    dstg[((a2 & 1) * O + o) * DP * 256 + dsidx] = __builtin_bit_cast(unsigned, t2v{(Tout)oe, (Tout)oo});
                } else if constexpr (STAGE) {
                    typedef Tout t2v __attribute__((ext_vector_type(2)));
                    const t2v pk = {(Tout)oe, (Tout)oo};
                    stg[SB][PH][o][sidx] = __builtin_bit_cast(unsigned, pk);
                } else {
                    fu_store<Tout>(oe, oo, yrs, yoff, so + o * yplane);
                }
            }
        };

        // Store rows base .. base+nr-1 of the group from staging buffer SB: per (row, o) the
        // group's segment of GDW dwords, as 4 line-aligned 256-B pieces (one dword per lane;
        // lanes outside the segment store past the buffer range).  Rows are spread over
        // the group's waves.
        const int gcol0 = grp * GW * FU_OWN;                          // first column of the group
        const int gdw = max(0, min(GDW, (F.w2 - gcol0) / 2));         // valid dwords per row
        auto flush = [&](auto SBc, int base, int nr) {
            constexpr int SB = decltype(SBc)::value;
            __builtin_amdgcn_s_waitcnt(0xc07f);                       // lgkmcnt(0): our writes
            __builtin_amdgcn_s_barrier();
            // fixed trip count (the wait counts of the following steps stay exact): pairs
            // past nr * O store nothing
    #pragma unroll
            for (int i = 0; i < (6 * O + GW - 1) / GW; ++i) {
                const int p = wslot + GW * i;
                const bool pv = p < nr * O;
                const int row = pv ? p / O : 0, o = pv ? p - row * O : 0;
                const unsigned S = (unsigned)((((int64_t)o * F.h2 + base + row) * F.w2 + gcol0) *
                                              (int64_t)sizeof(Tout));
                const unsigned A = S & ~127u;
    #pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned gb = A + 256u * k + 4u * lane;
                    const int d = (int)(gb - S) / 4;
                    const bool ok = pv && gb >= S && d < gdw;
                    const unsigned v = stg[SB][row][o][ok ? d : 0];
                    __builtin_amdgcn_raw_buffer_store_b32(v, yrs, ok ? gb : 0x80000000u, 0, 0);
                }
            }
        };

        // ---- prologue: u rows s0-1 and s0 -------------------------------------------
        if constexpr (DMA) {
            // rect rows s0-2 .. s0+2+DPD into the ring, drained and published to the group
            for (int R = s0 - 2; R <= s0 + 2 + DPD; ++R) dma_row(R);
            __builtin_amdgcn_s_waitcnt(0x0f70);                     // vmcnt(0)
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            Raw t0[C], t1[C], t2[C];
            read_row(s0 - 2, t0);
            read_row(s0 - 1, t1);
            read_row(s0, t2);
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                XP[1][c] = fu_unpack2<Tin>(t0[c], hi16);   // row s0-2 -> slot 1
                XP[2][c] = fu_unpack2<Tin>(t1[c], hi16);   // row s0-1 -> slot 2
                XP[0][c] = fu_unpack2<Tin>(t2[c], hi16);   // row s0   -> slot 0
            }
            urow(IC<-2>{}, lut[0], std::false_type{}, std::false_type{});   // u row s0-1: above only
            read_row(s0 + 1, t0);
    #pragma unroll
            for (int c = 0; c < C; ++c) XP[1][c] = fu_unpack2<Tin>(t0[c], hi16);   // row s0+1
            urow(IC<-1>{}, lut[1], std::true_type{}, std::false_type{});    // u row s0: above, centre
            read_row(s0 + 2, rawn);
        } else {
        {
            Raw t0[C], t1[C], t2[C];
            const unsigned o0 = row_off(s0 - 2), o1 = row_off(s0 - 1), o2 = row_off(s0);
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                t0[c] = fu_load<Tin>(xrs, xoff, o0 + c * xplane);
                t1[c] = fu_load<Tin>(xrs, xoff, o1 + c * xplane);
                t2[c] = fu_load<Tin>(xrs, xoff, o2 + c * xplane);
            }
            issue(IC<1>{}, s0 + 1);
    #pragma unroll
            for (int i = 0; i < PD; ++i) {          // ring: rect rows s0+2 .. s0+1+PD
                if (i == 0) issue(IC<2>{}, s0 + 2);
                if (i == 1) issue(IC<3>{}, s0 + 3);
                if (i == 2) issue(IC<4>{}, s0 + 4);
                if (i == 3) issue(IC<5>{}, s0 + 5);
                if (i == 4) issue(IC<0>{}, s0 + 6);
            }
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                xset(IC<1>{}, c, t0[c]);   // row s0-2 -> slot 1
                xset(IC<2>{}, c, t1[c]);   // row s0-1 -> slot 2
                xset(IC<0>{}, c, t2[c]);   // row s0   -> slot 0
            }
        }
        urow(IC<-2>{}, lut[0], std::false_type{}, std::false_type{});   // u row s0-1: above only
        convert(IC<1>{}, IC<1>{});                                      // row s0+1 -> slot 1
        urow(IC<-1>{}, lut[1], std::true_type{}, std::false_type{});    // u row s0: above, centre
        // Drain the prologue's loads: the compiler's wait counts at the loop header merge the
        // entry path with the back edge, and a ring load issued late on the entry path would
        // otherwise put a near-zero vmcnt wait into every iteration.
        if (FU_DRAIN) __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        }

        // ---- main loop ---------------------------------------------------------------
        float4 lnext = lut[2];
        auto step = [&](auto PHc, auto SBc, int a2) {
            constexpr int PH = decltype(PHc)::value;
            // keep each step's instructions inside the step: across a 12-step body the
            // scheduler otherwise hoists loads many steps ahead (266 VGPRs, 1 wave / SIMD)
            if (FU_SCHED) __builtin_amdgcn_sched_barrier(0);
            if constexpr (DMA) {
                dma_row(a2 + 3 + DPD);
                // this wave's piece of row a2+3 landed once at most the operations issued after
                // it are outstanding: DPD steps of (1 piece + the step's stores) (vmcnt counts
                // loads, stores and LDS-DMA together, in issue order); then the group's barrier
                // publishes every piece of the row (and orders the staged row's reads)
                // (the pyramid levels store O samples every second step: DPD even keeps the
                // count exact, the waits otherwise over-count, which is safe)
                constexpr int N = PYR ? DPD + (DPD / 2) * O : DPD * (1 + (DST ? 1 : O));
                static_assert(N < 64, "vmcnt");
                // + lgkmcnt(0): this wave's staged row (LDS writes of the previous step) is in
                // LDS before the barrier lets the storing waves read it
                __builtin_amdgcn_s_waitcnt(0x0070 | (N & 0xf) | ((N >> 4) << 14));
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
    #pragma unroll
                for (int c = 0; c < C; ++c) XP[(PH + 2) % 3][c] = fu_unpack2<Tin>(rawn[c], hi16);   // row a2+2
                read_row(a2 + 3, rawn);
                if constexpr (DST) dst_store(a2 - 1, a2 > s0);
            } else {
            convert(IC<(PH + 2) % 6>{}, IC<(PH + 2) % 3>{});            // rect row a2+2
            issue(IC<(PH + 2 + PD) % 6>{}, a2 + 2 + PD);
            }
            const float4 L = lnext;
            lnext = lut[min(a2 - s0 + 3, NLUT - 1)];
            urow(PHc, L, std::true_type{}, std::true_type{});           // u row a2+1
            out_row(PHc, SBc, a2);
        };
        // Full blocks of six unconditional steps: an exit or a conditional store between
        // steps would let the compiler sink each rect-row load (and the last FMAs of a conv
        // row) into the rarer block that consumes them, which removes the prefetch distance
        // and serialises the accumulation.  The band's last h2 % 6 rows run as a tail.
        // Two iterations per trip so the staging buffer index is a constant.
        auto block6 = [&](auto SBc, int base) {
            step(IC<0>{}, SBc, base);
            step(IC<1>{}, SBc, base + 1);
            step(IC<2>{}, SBc, base + 2);
            step(IC<3>{}, SBc, base + 3);
            step(IC<4>{}, SBc, base + 4);
            step(IC<5>{}, SBc, base + 5);
            if constexpr (STAGE) flush(SBc, base, 6);
        };
        auto tail = [&](auto SBc, int base) {
            if (base >= s1) return;
            step(IC<0>{}, SBc, base);
            if (base + 1 < s1) {
                step(IC<1>{}, SBc, base + 1);
                if (base + 2 < s1) {
                    step(IC<2>{}, SBc, base + 2);
                    if (base + 3 < s1) {
                        step(IC<3>{}, SBc, base + 3);
                        if (base + 4 < s1) step(IC<4>{}, SBc, base + 4);
                    }
                }
            }
            if constexpr (STAGE) flush(SBc, base, s1 - base);
        };
        int base = s0;
        if constexpr (STAGE || FU_L12) {   // two blocks per trip (constant staging index)
            for (; base + 12 <= s1; base += 12) {
                block6(IC<0>{}, base);
                block6(IC<1>{}, base + 6);
            }
        } else {
            for (; base + 12 <= s1; base += 6) block6(IC<0>{}, base);
        }
        if (base + 6 <= s1) {
            block6(IC<0>{}, base);
            tail(IC<1>{}, base + 6);
        } else {
            tail(IC<0>{}, base);
        }
        if constexpr (DST) {                        // the band's last output row
            __builtin_amdgcn_s_waitcnt(0xc07f);     // lgkmcnt(0): this wave's staged row
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            dst_store(s1 - 1, true);
        }
    };
    if constexpr (UIN) {
        (void)cd; (void)rc;
        // every u row of the band (s0 - 1 .. s1) and every lane's columns inside the input:
        // the padding selects drop out (RC 1 marks that loop for the u = input modes)
        const bool inner = s0 >= 1 && s1 + 1 <= F.h && __builtin_amdgcn_ballot_w64(!colin) == 0;
        if (inner) run(IC<0>{}, IC<1>{});
        else run(IC<0>{}, IC<0>{});
    } else {
        // the common classes get their own loop; mixed windows / bands run the generic one
        if (FU_ONE_CLASS) run(IC<1>{}, IC<1>{});
        else if (FU_CD && cd == 1 && rc == 1) run(IC<1>{}, IC<1>{});
        else if (FU_CD && cd == 1 && rc == 2) run(IC<1>{}, IC<2>{});
        else if (FU_CD && cd == 2 && rc == 1) run(IC<2>{}, IC<1>{});
        else if (FU_CD && cd == 2 && rc == 2) run(IC<2>{}, IC<2>{});
        else run(IC<0>{}, IC<0>{});
    }
}

}  // namespace hg
