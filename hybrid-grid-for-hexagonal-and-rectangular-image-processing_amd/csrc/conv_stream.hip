// conv_stream.hip — HexConv2d fast path: radius 2, stride 1, dilation 1,
// constant padding, up to 3 channels (the hot configurations: 3->3 dense,
// 3->3 depthwise, 1->1).
//
// Same execution model as the fused pipeline (pipeline.hip): a wavefront owns a
// 64-lane column window of one image and walks a band of output rows.  Lane l
// holds input column W0+l; the stencil's column taps are DPP wave shifts; the
// padded rows P[y] (y = input row + p) live in a 3-slot register ring keyed by
// y % 3 with the row loop unrolled x6 (3 slots x 2 parities), so slots and tap
// offsets are compile-time.  Input rows are raw buffer loads issued two rows ahead
// into phase-keyed register sets (no branch around a load, so they stay in flight).
// Tap geometry (HexFrames.py:108-162 restated): output (ro, q) tap t reads
// P[ro + ii_t][q + dk_t(ro & 1)], dk in [0, 3]; P col >= W' is the type1 raster's
// structural zero, other padding cells hold padding_value.
#include <algorithm>
#include <climits>
#include <type_traits>

#include "common.h"
#include "fused.h"

namespace hg {

struct ConvStreamGeom {
    int64_t B;
    int h, w, ho, wo, p;
    float padv;
    int HL, nown, nwin, nband, RB;
    Epilogue epi;
};

typedef float float2v_cs __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float cs_next(float v) {   // result[l] = v[l+1]
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ float cs_prev(float v) {   // result[l] = v[l-1]
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
__host__ __device__ constexpr int cs_tap_ii(int t) { return t < 2 ? 0 : (t < 5 ? 1 : 2); }
__host__ __device__ constexpr int cs_tap_col(int t) {
    return t < 2 ? 1 + 2 * t : (t < 5 ? 2 * (t - 2) : 1 + 2 * (t - 5));
}
__host__ __device__ constexpr int cs_tap_dk(int t, int par, int op) {
    return (1 + par + cs_tap_col(t) - ((((par + cs_tap_ii(t)) & 1) + op) & 1)) >> 1;
}

template <typename T>
__device__ __forceinline__ T cs_load(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 1) {
        return __builtin_bit_cast(T, (unsigned char)__builtin_amdgcn_raw_buffer_load_b8(rs, voff, soff, 0));
    } else if constexpr (sizeof(T) == 2) {
        return __builtin_bit_cast(T, (unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0));
    } else if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    } else {
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
    }
}
template <typename T>
__device__ __forceinline__ void cs_store(T v, __amdgpu_buffer_rsrc_t rs, unsigned voff,
                                         unsigned soff) {
    if constexpr (sizeof(T) == 2) {
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), rs, voff, soff, 0);
    } else if constexpr (sizeof(T) == 4) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, voff, soff, 0);
    } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, voff, soff, 0);
    }
}

// P: padding (0..2).  Lane offsets of the taps: dk - P in [-P, DKMAX - P].
template <typename Tin, typename Tout, int C, int O, int G, int OP, int P>
__global__ __launch_bounds__(256) void k_hexconv_stream(const Tin* __restrict__ x,
                                                        const float* __restrict__ kern,
                                                        const float* __restrict__ bias,
                                                        Tout* __restrict__ y, ConvStreamGeom F) {
    constexpr int CG = C / G, OG = O / G;
    constexpr int DKMAX = OP ? 2 : 3;
    constexpr int NS = DKMAX + 1;        // shifts d = dk - P + P = dk, lane offset dk - P
    constexpr int PD = 2, NSET = 3;
    constexpr bool PK = C == 3 && O == 3 && G == 1;
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int win = (int)(wave % F.nwin);
    const int64_t rest = wave / F.nwin;
    const int band = (int)(rest % F.nband);
    const int64_t b = rest / F.nband;
    if (b >= F.B) return;
    const int W0 = win * F.nown - F.HL;
    const int col = W0 + lane;                       // input column = output column
    const int r0 = band * F.RB;                      // F.RB % 6 == 0
    const int r1 = min(r0 + F.RB, F.ho);
    const bool col_in_w = col >= 0 && col < F.w;
    // P col = col + P; structural zero when P col >= W' = w + 2P
    const float colpad = (col + P >= F.w + 2 * P) ? 0.f : F.padv;
    const bool own = lane >= F.HL && lane < F.HL + F.nown && col >= 0 && col < F.wo;
    const unsigned lbyte = (unsigned)min(max(col, 0), F.w - 1) * (unsigned)sizeof(Tin);
    const unsigned obytecol = (unsigned)max(col, 0) * (unsigned)sizeof(Tout);
    const int64_t cst = (int64_t)F.h * F.w, ost = (int64_t)F.ho * F.wo;
    const Tin* xb = x + b * C * cst;
    Tout* yb = y + b * O * ost;
    __amdgpu_buffer_rsrc_t xrs[C], yrs[O];
#pragma unroll
    for (int c = 0; c < C; ++c)
        xrs[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(xb + c * cst), (short)0,
                                                   (int)(cst * (int64_t)sizeof(Tin)), 0x00020000);
#pragma unroll
    for (int o = 0; o < O; ++o)
        yrs[o] = __builtin_amdgcn_make_buffer_rsrc((void*)(yb + o * ost), (short)0,
                                                   (int)(ost * (int64_t)sizeof(Tout)), 0x00020000);

    // weights in VGPRs (opaque per-lane zero keeps them out of SGPRs)
    int vz = 0;
    asm volatile("" : "+v"(vz));
    const float* kv = kern + vz;
    float2v_cs wp2[PK ? O * 7 : 1];
    float wk[PK ? O * 7 : O * CG * 7], bs[O];
    if constexpr (PK) {
#pragma unroll
        for (int o = 0; o < O; ++o)
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                wp2[o * 7 + t] = float2v_cs{kv[(o * 3 + 0) * 7 + t], kv[(o * 3 + 1) * 7 + t]};
                wk[o * 7 + t] = kv[(o * 3 + 2) * 7 + t];
            }
    } else {
#pragma unroll
        for (int i = 0; i < O * CG * 7; ++i) wk[i] = kv[i];
    }
#pragma unroll
    for (int o = 0; o < O; ++o) bs[o] = bias ? bias[o + vz] : 0.f;

    // input rows in flight: set k holds P row y with y % 3 == k
    Tin X[NSET][C];
    int XOK[NSET];
#pragma unroll
    for (int k = 0; k < NSET; ++k) XOK[k] = 0;
    auto issue = [&](auto SETc, int yrow) {          // P row yrow = input row yrow - P
        constexpr int SET = decltype(SETc)::value;
        const int r = yrow - P;
        const unsigned rb = (unsigned)(min(max(r, 0), F.h - 1) * F.w) * (unsigned)sizeof(Tin);
#pragma unroll
        for (int c = 0; c < C; ++c) X[SET][c] = cs_load<Tin>(xrs[c], lbyte, rb);
        XOK[SET] = (r >= 0 && r < F.h) ? 1 : 0;
    };

    constexpr int CS = PK ? 1 : C;
    float2v_cs UP[3][NS];
    float U[3][NS][CS];
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
        for (int d = 0; d < NS; ++d) {
            UP[s3][d] = float2v_cs{0.f, 0.f};
#pragma unroll
            for (int c = 0; c < CS; ++c) U[s3][d][c] = 0.f;
        }
    // P row from set SET into slot SL, at lane shifts dk - P for dk = 0 .. DKMAX
    auto fill = [&](auto SLc, auto SETc) {
        constexpr int SL = decltype(SLc)::value;
        constexpr int SET = decltype(SETc)::value;
        const bool ok = XOK[SET] && col_in_w;
        float sh[NS][C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float v = XOK[SET] ? (col_in_w ? to_acc<float>(X[SET][c]) : colpad) : colpad;
            (void)ok;
            // shifts: sh[d] = v[lane + d - P]
            float t = v;
            sh[P][c] = v;
#pragma unroll
            for (int d = P + 1; d < NS; ++d) { t = cs_next(t); sh[d][c] = t; }
            t = v;
#pragma unroll
            for (int d = P - 1; d >= 0; --d) { t = cs_prev(t); sh[d][c] = t; }
        }
#pragma unroll
        for (int d = 0; d < NS; ++d) {
            if constexpr (PK) {
                UP[SL][d] = float2v_cs{sh[d][0], sh[d][1]};
                U[SL][d][0] = sh[d][2];
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) U[SL][d][c] = sh[d][c];
            }
        }
    };

    auto step = [&](auto PHc, int ro) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int PAR = PH & 1;
        constexpr int SLT[3] = {PH % 3, (PH + 1) % 3, (PH + 2) % 3};   // P rows ro, ro+1, ro+2
        issue(std::integral_constant<int, (PH + 2 + PD) % NSET>{}, ro + 2 + PD);
        fill(std::integral_constant<int, (PH + 2) % 3>{}, std::integral_constant<int, (PH + 2) % NSET>{});
        const unsigned ob = (unsigned)__builtin_amdgcn_readfirstlane(ro * F.wo) * (unsigned)sizeof(Tout);
        if constexpr (PK) {
#pragma unroll
            for (int o = 0; o < 3; ++o) {
                float2v_cs ap = {bs[o], 0.f};
                float as = 0.f;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int sl = SLT[cs_tap_ii(t)];
                    const int dk = cs_tap_dk(t, PAR, OP);
                    ap = __builtin_elementwise_fma(wp2[o * 7 + t], UP[sl][dk], ap);
                    as = fmaf(wk[o * 7 + t], U[sl][dk][0], as);
                }
                float v = (ap.x + ap.y) + as;
                if (F.epi.on) v = epi_apply(v, o, F.epi);
                if (own) cs_store<Tout>(from_acc<Tout>(v), yrs[o], obytecol, ob);
            }
        } else {
#pragma unroll
            for (int o = 0; o < O; ++o) {
                float acc = bs[o];
#pragma unroll
                for (int ci = 0; ci < CG; ++ci) {
                    const int c = (o / OG) * CG + ci;
#pragma unroll
                    for (int t = 0; t < 7; ++t)
                        acc = fmaf(wk[(o * CG + ci) * 7 + t],
                                   U[SLT[cs_tap_ii(t)]][cs_tap_dk(t, PAR, OP)][c], acc);
                }
                if (F.epi.on) acc = epi_apply(acc, o, F.epi);
                if (own) cs_store<Tout>(from_acc<Tout>(acc), yrs[o], obytecol, ob);
            }
        }
    };

    // prologue: P rows r0 (slot/set 0), r0+1 (1); loads for r0+2 .. r0+1+PD in flight
    issue(std::integral_constant<int, 0>{}, r0);
    issue(std::integral_constant<int, 1>{}, r0 + 1);
    fill(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    issue(std::integral_constant<int, 2>{}, r0 + 2);
    fill(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    issue(std::integral_constant<int, 0>{}, r0 + 3);
    for (int base = r0; base < r1; base += 6) {
        step(std::integral_constant<int, 0>{}, base);
        if (base + 1 >= r1) break;
        step(std::integral_constant<int, 1>{}, base + 1);
        if (base + 2 >= r1) break;
        step(std::integral_constant<int, 2>{}, base + 2);
        if (base + 3 >= r1) break;
        step(std::integral_constant<int, 3>{}, base + 3);
        if (base + 4 >= r1) break;
        step(std::integral_constant<int, 4>{}, base + 4);
        if (base + 5 >= r1) break;
        step(std::integral_constant<int, 5>{}, base + 5);
    }
}

template <typename Tin, typename Tout, int C, int O, int G>
static int launch_cs(const void* x, const float* k, const float* b, void* y,
                     const ConvStreamGeom& F, int op, hipStream_t st) {
    const int64_t waves = F.B * (int64_t)F.nband * F.nwin;
    const dim3 grid((unsigned)((waves + 3) / 4)), blk(256);
#define HG_CS(OPV, PV) hipLaunchKernelGGL((k_hexconv_stream<Tin, Tout, C, O, G, OPV, PV>), grid, \
                                          blk, 0, st, (const Tin*)x, k, b, (Tout*)y, F)
    switch (F.p * 2 + op) {
    case 0: HG_CS(0, 0); break;
    case 1: HG_CS(1, 0); break;
    case 2: HG_CS(0, 1); break;
    case 3: HG_CS(1, 1); break;
    case 4: HG_CS(0, 2); break;
    case 5: HG_CS(1, 2); break;
    default: return HG_EUNSUP;
    }
#undef HG_CS
    return launch_status();
}

template <typename Tin, typename Tout>
static int cs_channels(const void* x, const float* k, const float* b, void* y,
                       const ConvStreamGeom& F, int C, int O, int G, int op, hipStream_t st) {
    if (C == 3 && O == 3 && G == 1) return launch_cs<Tin, Tout, 3, 3, 1>(x, k, b, y, F, op, st);
    if (C == 3 && O == 3 && G == 3) return launch_cs<Tin, Tout, 3, 3, 3>(x, k, b, y, F, op, st);
    if (C == 1 && O == 1 && G == 1) return launch_cs<Tin, Tout, 1, 1, 1>(x, k, b, y, F, op, st);
    return HG_EUNSUP;
}

// Returns HG_EUNSUP when the configuration is not covered (the caller then runs the
// generic LDS-tiled kernel).  Preconditions checked by hg_hexconv2d: radius 2,
// stride 1, dilation 1, constant padding, float32 weights.
int launch_conv_stream(const void* x, const float* k, const float* b, void* y, int x_dtype,
                       int y_dtype, int64_t B, int C, int O, int64_t h, int64_t w, int p,
                       int groups, int off, double pad_value, const Epilogue& epi,
                       hipStream_t st) {
    if (p < 0 || p > 2 || h > INT_MAX / 4 || w > INT_MAX / 4) return HG_EUNSUP;
    {   // two-column streaming kernel (fused_conv.hip) where it applies
        const int rc = fused_conv_try(x, k, b, y, x_dtype, y_dtype, B, C, O, groups, h, w, p, off,
                                      pad_value, epi.on != 0, st);
        if (rc != HG_EUNSUP) return rc;
    }
    if (h * w * 8 >= INT_MAX) return HG_EUNSUP;   // 32-bit buffer offsets
    ConvStreamGeom F;
    F.B = B; F.h = (int)h; F.w = (int)w; F.p = p; F.padv = (float)pad_value;
    F.epi = epi;
    F.ho = F.h + 2 * p - 2;
    F.wo = F.w + 2 * p - 2;
    if (F.ho < 1 || F.wo < 1) return HG_EUNSUP;
    const int op = (off + p) & 1;
    const int dkmax = op ? 2 : 3;
    // lanes read offsets [-p, dkmax - p]
    F.HL = std::max(0, p);
    const int hr = std::max(0, dkmax - p);
    F.nown = 64 - F.HL - hr;
    F.nwin = (F.wo + F.nown - 1) / F.nown;
    F.RB = 126;
    F.nband = (F.ho + F.RB - 1) / F.RB;
    switch (x_dtype) {
    case HG_BF16:
        if (y_dtype == HG_BF16) return cs_channels<__bf16, __bf16>(x, k, b, y, F, C, O, groups, op, st);
        if (y_dtype == HG_F32) return cs_channels<__bf16, float>(x, k, b, y, F, C, O, groups, op, st);
        return HG_EUNSUP;
    case HG_F16:
        if (y_dtype == HG_F16) return cs_channels<_Float16, _Float16>(x, k, b, y, F, C, O, groups, op, st);
        if (y_dtype == HG_F32) return cs_channels<_Float16, float>(x, k, b, y, F, C, O, groups, op, st);
        return HG_EUNSUP;
    case HG_F32:
        if (y_dtype == HG_F32) return cs_channels<float, float>(x, k, b, y, F, C, O, groups, op, st);
        if (y_dtype == HG_BF16) return cs_channels<float, __bf16>(x, k, b, y, F, C, O, groups, op, st);
        return HG_EUNSUP;
    default:
        return HG_EUNSUP;
    }
}

}  // namespace hg
