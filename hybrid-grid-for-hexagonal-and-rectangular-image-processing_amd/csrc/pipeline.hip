// pipeline.hip — the fused rect -> hex -> HexConv2d -> hex -> rect pass.
//
// The reference chains three host round trips: rect_to_hex_resample
// (geometry_np.py:358-519) -> HexConv2d (HexFrames.py:96-169) ->
// hex_to_rect_resample (geometry_np.py:191-356).  Unfused on the GPU that is
// 3 kernels x (read + write) = 36 B/px in bf16; fused, the rect input is read
// once and the rect output written once: 12 B/px.
//
// Execution model: one wavefront owns a 64-lane column window (lane l <->
// column W0+l in every stage's own column space) of one image, and walks a
// band of output rows top to bottom.  All intermediate rows live in registers:
//   x rows (rect input, 2 rows)  --vertical bilinear (row maps uniform)-->  v
//   v --cross-lane gather (per-lane column map)-->  u  (hex row, r2h output)
//   u (3 rows, 3 lane shifts each) --7-tap hex stencil, weights in SGPRs--> z
//   z (2 rows) --cross-lane gather + triangle weights--> output row
// Cross-lane traffic stays inside the wave, so the outermost lanes of each stage
// are halo; the host sizes the halo from the lattice maps (near-identity
// geometries only — e.g. same-size round trips; others use the 3-kernel chain).
// No LDS, no barriers.  Intermediates are fp32 (the reference's are fp64/fp32),
// so the fused path is at least as close to the reference as the unfused bf16 one.
#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>

#include "common.h"
#include "fused.h"
#include "lattice.h"

namespace hg {

constexpr int PL_THREADS = 256;   // 4 independent waves per workgroup
constexpr int PL_KMAX = 3 * 3 * 7;

struct PipeGeom {
    int64_t B;
    int h, w, h1, w1, ho, wo, h2, w2;
    int p, op;             // conv padding, (even_odd_offset + p) & 1
    float padv;
    Geom r2h, h2r;         // lattice geometries of the two resamplers
    int HL, nown;          // halo lanes on the left, owned lanes per wave
    int nwin, nband, RB;   // column windows, row bands, rows per band
};

// Column offset (in P / u columns, relative to the output column) of tap t of the
// r=2 stencil on an output row of parity `par` (see hexconv.hip / hg_oracle.c).
__host__ __device__ constexpr int tap_ii(int t) { return t < 2 ? 0 : (t < 5 ? 1 : 2); }
__host__ __device__ constexpr int tap_col(int t) {
    return t < 2 ? 1 + 2 * t : (t < 5 ? 2 * (t - 2) : 1 + 2 * (t - 5));
}
__host__ __device__ constexpr int tap_dk(int t, int par, int op) {
    return (1 + par + tap_col(t) - ((((par + tap_ii(t)) & 1) + op) & 1)) >> 1;
}

// ---- cross-lane movement --------------------------------------------------
// Generic: ds_bpermute (any source lane).  DPP mode: wave-wide shifts by one lane
// (GFX9 DPP wave_shl:1 / wave_shr:1, full VALU rate, no LDS round trip) build a
// small window of shifted copies, and each lane selects its offset from it.
__device__ __forceinline__ float lane_get(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ float dpp_next(float v) {   // result[l] = v[l+1], 0 past lane 63
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x130 /*wave_shl:1*/, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_prev(float v) {   // result[l] = v[l-1], 0 before lane 0
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x138 /*wave_shr:1*/, 0xf, 0xf, true));
}
// s[k - LO] = v[l + k] for k in [LO, HI]
template <int LO, int HI>
__device__ __forceinline__ void window(float v, float* s) {
    s[-LO] = v;
    float t = v;
#pragma unroll
    for (int i = 1; i <= HI; ++i) { t = dpp_next(t); s[-LO + i] = t; }
    t = v;
#pragma unroll
    for (int i = 1; i <= -LO; ++i) { t = dpp_prev(t); s[-LO - i] = t; }
}
template <int LO, int HI>
__device__ __forceinline__ float pick(const float* s, int k) {   // k in [LO, HI] per lane
    float r = s[0];
#pragma unroll
    for (int i = 1; i <= HI - LO; ++i) r = (k - LO == i) ? s[i] : r;
    return r;
}

// DPP-mode windows (lane offsets relative to the own column), checked by the host.
constexpr int PL_RLO = -1, PL_RHI = 2;    // r2h: v at jn, jn+1
constexpr int PL_ZALO = -1, PL_ZAHI = 2;  // h2r: z row i2n at c1, c1+1
constexpr int PL_ZBLO = -2, PL_ZBHI = 2;  // h2r: z row i2n+1 at c1-e, c1-e+1
constexpr int PL_PF = 4;                  // rect rows prefetched ahead (latency cover)

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// HZ: every h2r sample row lies exactly on a hex row (i_f == 0 for all rows, e.g. a
// same-size round trip): gamma == |i_f| == 0 and p2 == p2a, so row i2n+1 is never read.
template <typename Tin, typename Tout, int C, int O, int G, int OP, bool DPP, bool HZ>
__global__ __launch_bounds__(PL_THREADS) void k_pipeline(const Tin* __restrict__ x,
                                                         const float* __restrict__ kern,
                                                         const float* __restrict__ bias,
                                                         Tout* __restrict__ y, PipeGeom F) {
    constexpr int CG = C / G, OG = O / G;
    constexpr int DKMAX = OP ? 2 : 3;   // stencil column shifts dk in [0, DKMAX]
    constexpr int NS = DKMAX + 1;
    constexpr int NW = (O * CG * 7 + 3) & ~3;
    // kernel weights [O][C/G][7] and bias, staged once per workgroup in LDS and
    // read back as wave-uniform broadcasts (no SGPR pressure, no per-step spills)
    __shared__ __attribute__((aligned(16))) float wsh[NW + 4];
    for (int i = threadIdx.x; i < NW + 4; i += PL_THREADS) {
        float v = 0.f;
        if (i < O * CG * 7) v = kern[i];
        else if (i >= NW && i - NW < O && bias) v = bias[i - NW];
        wsh[i] = v;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    // wave index made provably wave-uniform: everything derived from it (image, band,
    // window, row bounds, base pointers, buffer descriptors) then lives in SGPRs
    const int64_t wave = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (PL_THREADS / 64) +
                         __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int win = (int)(wave % F.nwin);
    const int64_t rest = wave / F.nwin;
    const int band = (int)(rest % F.nband);
    const int64_t b = rest / F.nband;
    if (b >= F.B) return;
    const int W0 = win * F.nown - F.HL;
    const int col = W0 + lane;
    const int a2_begin = band * F.RB;
    const int a2_end = min(a2_begin + F.RB, F.h2);
    const int p = DPP ? 1 : F.p;

    // ---- per-lane column maps (fp64, once) --------------------------------
    int src_l = lane, src_r = lane;     // r2h: lanes holding v at rect cols jn, jn+1
    float fj = 0.f, gj = 0.f;
    if (col >= 0 && col < F.w1) {
        const double y_ = axis_at(F.r2h.ys, col);
        const double j_ = y_ + (double)(F.w - 1) * 0.5;            // geometry_np.py:441
        const int64_t jn = (int64_t)j_;
        const double jf = j_ - (double)(float)jn;
        fj = (float)jf;
        gj = (float)(1.0 - jf);
        src_l = (int)(jn - W0);
        src_r = (int)(jn + 1 - W0);
    }
    const double y2 = (col >= 0 && col < F.w2) ? axis_at(F.h2r.ys, col) : 0.0;
    const double cj2 = ((double)F.wo - 0.5) * 0.5;                 // :277
    const bool col_in_w = col >= 0 && col < F.w;
    const bool col_in_w1 = col >= 0 && col < F.w1;
    const bool col_struct0 = col >= F.w1 + p;                      // type1 structural zero
    const bool col_in_wo = col >= 0 && col < F.wo;
    const bool own = lane >= F.HL && lane < F.HL + F.nown && col >= 0 && col < F.w2;

    const Tin* xb = x + b * (int64_t)C * F.h * F.w + (col_in_w ? col : 0);
    Tout* yb = y + b * (int64_t)O * F.h2 * F.w2;
    const int64_t cstride = (int64_t)F.h * F.w;

    // ---- pipeline state ----------------------------------------------------
    float x0[C], x1[C];                 // rect rows xr-1, xr at column col
    Tin pf[PL_PF][C];                   // rect rows xr+1 .. xr+PL_PF (loads in flight)
    float us[3][NS][C];                 // u rows ur-2..ur at lane shifts dk - p
    float z0[O], z1[O];                 // conv rows zr-1, zr
#pragma unroll
    for (int c = 0; c < C; ++c) {
        x0[c] = x1[c] = 0.f;
#pragma unroll
        for (int i = 0; i < PL_PF; ++i) pf[i][c] = (Tin)0;
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int d = 0; d < NS; ++d) us[s][d][c] = 0.f;
    }
#pragma unroll
    for (int o = 0; o < O; ++o) z0[o] = z1[o] = 0.f;

    auto h2r_row = [&](int a2, double& i2_, int64_t& i2n) {
        const double xx = axis_at(F.h2r.xs, a2);
        i2_ = xx + (double)(F.ho - 1) * 0.5;                         // :276
        i2n = uniform((int)i2_);
    };
    auto r2h_row = [&](int a1, int64_t& in, float& fi, float& gi) {
        const double xx = axis_at(F.r2h.xs, a1);
        const double i_ = xx + (double)(F.h - 1) * 0.5;              // :440
        in = uniform((int)i_);
        const double f = i_ - (double)(float)in;
        fi = (float)f;
        gi = (float)(1.0 - f);
    };
    auto fetch = [&](int r, Tin* dst) {
        const bool ok = r >= 0 && r < F.h && col_in_w;
#pragma unroll
        for (int c = 0; c < C; ++c) dst[c] = ok ? xb[c * cstride + (int64_t)r * F.w] : (Tin)0;
    };

    double i2_0;
    int64_t i2n0;
    h2r_row(a2_begin, i2_0, i2n0);
    int zr = (int)i2n0 - 1;             // z1 holds row zr
    int ur = zr + 1 - p + 2 - 3;        // us slot 2 holds row ur
    int xr = INT_MIN;                   // x1 holds rect row xr (INT_MIN: none)

    auto restart_x = [&](int in) {      // x0 = row in, x1 = row in+1, pf = in+2 ..
        Tin t0[C], t1[C];
        fetch(in, t0);
        fetch(in + 1, t1);
#pragma unroll
        for (int i = 0; i < PL_PF; ++i) fetch(in + 2 + i, pf[i]);
#pragma unroll
        for (int c = 0; c < C; ++c) { x0[c] = to_acc<float>(t0[c]); x1[c] = to_acc<float>(t1[c]); }
        xr = in + 1;
    };
    auto advance_x = [&]() {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            x0[c] = x1[c];
            x1[c] = to_acc<float>(pf[0][c]);
#pragma unroll
            for (int i = 0; i + 1 < PL_PF; ++i) pf[i][c] = pf[i + 1][c];
        }
        ++xr;
        fetch(xr + PL_PF, pf[PL_PF - 1]);
    };
    auto advance_u = [&]() {
        ++ur;
        const bool row_in = ur >= 0 && ur < F.h1;
        float uv[C];
        if (row_in) {
            int64_t in; float fi, gi;
            r2h_row(ur, in, fi, gi);
            if (xr < (int)in) restart_x((int)in);   // first use, or a jump of >= 2 rows
            while (xr < (int)in + 1) advance_x();   // x0 = row in, x1 = row in+1
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float v = fi * x1[c] + gi * x0[c];         // t = fi*p3 + (1-fi)*p1
                float vl, vr;
                if constexpr (DPP) {
                    float sw[PL_RHI - PL_RLO + 1];
                    window<PL_RLO, PL_RHI>(v, sw);
                    vl = pick<PL_RLO, PL_RHI>(sw, src_l - lane);
                    vr = pick<PL_RLO, PL_RHI>(sw, src_r - lane);
                } else {
                    vl = lane_get(v, src_l);
                    vr = lane_get(v, src_r);
                }
                const float u = fj * vr + gj * vl;               // :517
                uv[c] = col_in_w1 ? u : (col_struct0 ? 0.f : F.padv);
            }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) uv[c] = col_struct0 ? 0.f : F.padv;   // pad rows
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
#pragma unroll
            for (int d = 0; d < NS; ++d) {
                us[0][d][c] = us[1][d][c];
                us[1][d][c] = us[2][d][c];
            }
            if constexpr (DPP) {
                float sw[NS];
                window<-1, DKMAX - 1>(uv[c], sw);   // p == 1: lane offsets dk - 1
#pragma unroll
                for (int d = 0; d < NS; ++d) us[2][d][c] = sw[d];
            } else {
#pragma unroll
                for (int d = 0; d < NS; ++d) us[2][d][c] = lane_get(uv[c], lane + d - p);
            }
        }
    };
    auto advance_z = [&]() {
        ++zr;
        while (ur < zr - p + 2) advance_u();
        float acc[O];
        float wk[NW], bs[4];
        // an opaque zero offset keeps the compiler from hoisting the weight reads out of
        // the row loop into 63 long-lived VGPRs: they are re-read per row (16 x b128)
        int wo0 = 0;
        asm volatile("" : "+v"(wo0));
#pragma unroll
        for (int i = 0; i < NW; i += 4) {
            const float4 w4 = *reinterpret_cast<const float4*>(&wsh[wo0 + i]);
            wk[i] = w4.x; wk[i + 1] = w4.y; wk[i + 2] = w4.z; wk[i + 3] = w4.w;
        }
        {
            const float4 b4 = *reinterpret_cast<const float4*>(&wsh[wo0 + NW]);
            bs[0] = b4.x; bs[1] = b4.y; bs[2] = b4.z; bs[3] = b4.w;
        }
#pragma unroll
        for (int o = 0; o < O; ++o) acc[o] = bs[o];
        if ((zr & 1) == 0) {
#pragma unroll
            for (int o = 0; o < O; ++o)
#pragma unroll
                for (int ci = 0; ci < CG; ++ci) {
                    const int c = (o / OG) * CG + ci;
#pragma unroll
                    for (int t = 0; t < 7; ++t)
                        acc[o] += wk[(o * CG + ci) * 7 + t] * us[tap_ii(t)][tap_dk(t, 0, OP)][c];
                }
        } else {
#pragma unroll
            for (int o = 0; o < O; ++o)
#pragma unroll
                for (int ci = 0; ci < CG; ++ci) {
                    const int c = (o / OG) * CG + ci;
#pragma unroll
                    for (int t = 0; t < 7; ++t)
                        acc[o] += wk[(o * CG + ci) * 7 + t] * us[tap_ii(t)][tap_dk(t, 1, OP)][c];
                }
        }
        const bool ok = zr >= 0 && zr < F.ho && col_in_wo;
#pragma unroll
        for (int o = 0; o < O; ++o) {
            z0[o] = z1[o];
            z1[o] = ok ? acc[o] : 0.f;
        }
    };

    for (int a2 = a2_begin; a2 < a2_end; ++a2) {
        double i2_;
        int64_t i2n;
        h2r_row(a2, i2_, i2n);
        if constexpr (HZ) {
            while (zr < (int)i2n) advance_z();          // z1 = row i2n
        } else {
            while (zr < (int)i2n + 1) advance_z();      // z0 = row i2n, z1 = row i2n+1
        }
        // per-sample triangle (geometry_np.py:277-298) and closed-form barycentric weights
        const double j_ = 0.5 * i2_ + y2 + cj2;
        const int64_t jn = (int64_t)j_;
        const double i_f = i2_ - (double)(float)i2n;
        const double j_f = j_ - (double)(float)jn;
        const bool flag = i_f > j_f;
        const int64_t s1 = (int64_t)((double)(i2n + 1) / 2.0);
        const int64_t s2 = (int64_t)((double)(i2n + 2) / 2.0);
        const int k1 = (int)(jn - s1) - col;            // offset of p1 (row i2n)
        const int k2 = (int)(jn - s2) - col;            // offset of (row i2n+1, col j - s2)
        const float u = (float)i_f, v = (float)j_f;
        const float wa = fabsf(1.f - (flag ? u : v));
        const float wb = fabsf(v - u);
        const float wg = fabsf(flag ? v : u);
        const float rs = 1.f / (wa + wb + wg);
        if constexpr (HZ) {   // u == 0: flag false, gamma 0, p2 = (i2n, c1+1)
#pragma unroll
            for (int o = 0; o < O; ++o) {
                float p1, p2;
                if constexpr (DPP) {
                    float sa[PL_ZAHI - PL_ZALO + 1];
                    window<PL_ZALO, PL_ZAHI>(z1[o], sa);
                    p1 = pick<PL_ZALO, PL_ZAHI>(sa, k1);
                    p2 = pick<PL_ZALO, PL_ZAHI>(sa, k1 + 1);
                } else {
                    p1 = lane_get(z1[o], lane + k1);
                    p2 = lane_get(z1[o], lane + k1 + 1);
                }
                const float out = (wa * p1 + wb * p2) * rs;
                if (own) yb[((int64_t)o * F.h2 + a2) * F.w2 + col] = from_acc<Tout>(out);
            }
            continue;
        }
#pragma unroll
        for (int o = 0; o < O; ++o) {
            float p1, p2a, p2b, p3;
            if constexpr (DPP) {
                float sa[PL_ZAHI - PL_ZALO + 1], sb[PL_ZBHI - PL_ZBLO + 1];
                window<PL_ZALO, PL_ZAHI>(z0[o], sa);
                window<PL_ZBLO, PL_ZBHI>(z1[o], sb);
                p1 = pick<PL_ZALO, PL_ZAHI>(sa, k1);
                p2a = pick<PL_ZALO, PL_ZAHI>(sa, k1 + 1);
                p2b = pick<PL_ZBLO, PL_ZBHI>(sb, k2);
                p3 = pick<PL_ZBLO, PL_ZBHI>(sb, k2 + 1);
            } else {
                p1 = lane_get(z0[o], lane + k1);
                p2a = lane_get(z0[o], lane + k1 + 1);
                p2b = lane_get(z1[o], lane + k2);
                p3 = lane_get(z1[o], lane + k2 + 1);
            }
            const float p2 = flag ? p2b : p2a;
            const float out = (wa * p1 + wb * p2 + wg * p3) * rs;
            if (own) yb[((int64_t)o * F.h2 + a2) * F.w2 + col] = from_acc<Tout>(out);
        }
    }
}

// ---------------------------------------------------------------------------
// Same-size fast path (mode 3): h2 == ho, w2 == wo, padding 1.  Then the h2r
// lattice is exact in fp64: x_ = a - (ho-1)/2 and y_ = b - wo/2 + 0.5
// (linspace steps are exactly 1), so i_ = a, j_ = 0.5a + b + 0.25, i_f = 0 and
// (geometry_np.py:276-298) p1 = z[a][b + k1], p2 = z[a][b + k1 + 1] with
// (k1, j_f) = (0, 0.25) on even rows and (-1, 0.75) on odd rows: a fixed 2-tap
// horizontal filter (alpha = 1 - j_f, beta = j_f, gamma = 0).  The r2h column
// maps stay per lane (weights over a 4-lane DPP window).  The row loop is unrolled
// by 6 = lcm(3 u slots, 2 parities): u row r lives in slot r % 3; the rect input
// rows live in a 6-slot ring keyed by the step phase and prefetched 5 rows ahead.
// No register is shuffled between steps; fp32 math is FMA / packed FMA.
// ---------------------------------------------------------------------------
typedef float float2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float2v pk_fma(float2v a, float2v b, float2v c) {
    return __builtin_elementwise_fma(a, b, c);
}

template <typename T>
__device__ __forceinline__ void buf_store(T v, __amdgpu_buffer_rsrc_t rs, unsigned voff,
                                          unsigned soff) {
    if constexpr (sizeof(T) == 2)
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), rs, voff, soff, 0);
    else if constexpr (sizeof(T) == 4)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, voff, soff, 0);
    else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, voff, soff, 0);
    }
}

// Raw buffer load of one element: SGPR descriptor + VGPR byte offset + SGPR byte
// offset, so a row fetch costs no per-lane address arithmetic.
template <typename T>
__device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    if constexpr (sizeof(T) == 1) {
        const unsigned char v = __builtin_amdgcn_raw_buffer_load_b8(rs, voff, soff, 0);
        return __builtin_bit_cast(T, v);
    } else if constexpr (sizeof(T) == 2) {
        const unsigned short v = __builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0);
        return __builtin_bit_cast(T, v);
    } else {
        const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
        return __builtin_bit_cast(T, v);
    }
}

// Tuning knobs of the static kernel (compile-time; tools/build_variant.sh sweeps them).
#ifndef PL_S_PD
#define PL_S_PD 2            // u rows whose rect rows are loaded ahead
#endif
#ifndef PL_S_OOBST
#define PL_S_OOBST 0         // 1: non-owned lanes store out of range instead of branching
#endif
#ifndef PL_S_FIV
#define PL_S_FIV 1           // 1: row weights as broadcast VGPR operands, 0: SGPRs
#endif
#ifndef PL_S_WPE
#define PL_S_WPE 0           // min waves per SIMD requested from the register allocator
#endif
// Rows of the per-wave r2h row table: u rows [a2_begin - 1, a2_begin + RB + PD].
constexpr int PL_LUT = 136;

// R3: every live r2h tap lies in the lane window [-1, 1] (jn - q in {-1, 0} wherever
// a tap is in range, e.g. same-size resamples); otherwise the window is [-1, 2].
template <typename Tin, typename Tout, int C, int O, int G, int OP, bool R3>
__global__ __launch_bounds__(PL_THREADS) __attribute__((amdgpu_waves_per_eu(PL_S_WPE ? PL_S_WPE : 1)))
void k_pipeline_s(const Tin* __restrict__ x, const float* __restrict__ kern,
                  const float* __restrict__ bias, Tout* __restrict__ y, PipeGeom F) {
    constexpr int CG = C / G, OG = O / G;
    constexpr int DKMAX = OP ? 2 : 3;          // stencil shifts dk in [0, DKMAX], lanes dk-1
    constexpr int NS = DKMAX + 1;
    // per-wave r2h row table: {byte offset of row in, of row in+1, fi, 1-fi} with the
    // weight of an out-of-range rect row folded to 0 (geometry_np.py:465-486)
    __shared__ uint4 lut_all[PL_THREADS / 64][PL_LUT];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4* lut = lut_all[wslot];
    // wave index made provably wave-uniform: everything derived from it (image, band,
    // window, row bounds, base pointers, buffer descriptors) then lives in SGPRs
    const int64_t wave = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (PL_THREADS / 64) + wslot;
    const int win = (int)(wave % F.nwin);
    const int64_t rest = wave / F.nwin;
    const int band = (int)(rest % F.nband);
    const int64_t b = rest / F.nband;
    if (b >= F.B) return;
    const int W0 = win * F.nown - F.HL;
    const int col = W0 + lane;
    const int a2_begin = band * F.RB;                 // F.RB % 6 == 0
    const int a2_end = min(a2_begin + F.RB, F.h2);
    const int ubase = a2_begin - 1;                   // u row of lut[0]

    // row table: lane l fills entries l, l+64, l+128 (fp64 lattice math, :440-449)
    for (int e = lane; e < PL_LUT; e += 64) {
        const int r = min(max(ubase + e, 0), F.h1 - 1);
        const double i_ = axis_at(F.r2h.xs, r) + (double)(F.h - 1) * 0.5;   // :440
        const int in = (int)i_;
        const double f = i_ - (double)(float)in;
        const bool ok0 = in >= 0 && in < F.h, ok1 = in + 1 >= 0 && in + 1 < F.h;
        uint4 t;
        t.x = (unsigned)(min(max(in, 0), F.h - 1) * F.w) * (unsigned)sizeof(Tin);
        t.y = (unsigned)(min(max(in + 1, 0), F.h - 1) * F.w) * (unsigned)sizeof(Tin);
        t.z = __builtin_bit_cast(unsigned, ok1 ? (float)f : 0.f);
        t.w = __builtin_bit_cast(unsigned, ok0 ? (float)(1.0 - f) : 0.f);
        lut[e] = t;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): own-wave LDS writes visible
    __builtin_amdgcn_wave_barrier();

    // r2h column weights over the lane window [-1, NR-2]: u = sum_k wr[k+1] * v[lane+k].
    // A tap on a rect column outside [0, w) reads 0 in the reference: its weight is 0
    // here, so v may hold anything finite there (the loads are column-clamped).
    constexpr int NR = R3 ? 3 : 4;
    float wr[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) wr[k] = 0.f;
    if (col >= 0 && col < F.w1) {
        const double j_ = axis_at(F.r2h.ys, col) + (double)(F.w - 1) * 0.5;   // :441
        const int64_t jn = (int64_t)j_;
        const double jf = j_ - (double)(float)jn;
        const int kl = (int)(jn - col);
#pragma unroll
        for (int k = -1; k <= NR - 2; ++k) {
            const bool in_w = col + k >= 0 && col + k < F.w;
            if (k == kl && in_w) wr[k + 1] = (float)(1.0 - jf);   // weight of t1 = v[jn]
            if (k == kl + 1 && in_w) wr[k + 1] = (float)jf;       // weight of t2 = v[jn+1]
        }
    }
    const bool col_in_w1 = col >= 0 && col < F.w1;
    // padding cells hold padv; u columns >= w1 + 1 are the type1 raster's structural
    // zeros, read only by OP == 0 outputs (for OP == 1 they reach only z columns >= wo,
    // which are zeroed), so for OP == 1 colpad stays wave-uniform
    const float colpad = (OP == 0 && col >= F.w1 + 1) ? 0.f : F.padv;
    const bool col_in_wo = col >= 0 && col < F.wo;
    const bool own = lane >= F.HL && lane < F.HL + F.nown && col >= 0 && col < F.w2;
    const unsigned lcol = (unsigned)min(max(col, 0), F.w - 1);   // clamped lane offset
    const unsigned ocol = col >= 0 ? (unsigned)col : 0u;

    const Tin* xb = x + b * (int64_t)C * F.h * F.w;                // wave-uniform bases
    Tout* yb = y + b * (int64_t)O * F.h2 * F.w2;
    const int64_t cstride = (int64_t)F.h * F.w;
    const int64_t ostride = (int64_t)F.h2 * F.w2;

    // Input path, branch-free: the rect rows (in, in+1) of u row r are loaded PD steps
    // before use into register set (r - a2_begin) mod NSET; row offsets and weights
    // come from the table.
    constexpr int PD = PL_S_PD;         // u rows loaded ahead
    static_assert(PD >= 2 && PD <= 4, "row table holds RB + 2 + PD <= PL_LUT rows");
    constexpr int NSET = PD + 1 <= 3 ? 3 : 6;   // register sets keyed by row % NSET (NSET | 6)
    // [set][channel] rows (in, in+1); 16-bit types share one VGPR (d16 / d16_hi loads)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr bool X16 = sizeof(Tin) == 2;
    using XT = typename std::conditional<X16, u16x2, Tin[2]>::type;
    XT X[NSET][C];
    float FI[NSET], GI[NSET];           // row weights of the set's u row (uniform)
    __amdgpu_buffer_rsrc_t xrs[C];      // one buffer descriptor per input channel plane
#pragma unroll
    for (int c = 0; c < C; ++c)
        xrs[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(xb + c * cstride), (short)0,
                                                   (int)(cstride * (int64_t)sizeof(Tin)),
                                                   0x00020000);
    const unsigned lbyte = lcol * (unsigned)sizeof(Tin);
    __amdgpu_buffer_rsrc_t yrs[O];      // one buffer descriptor per output channel plane
#pragma unroll
    for (int o = 0; o < O; ++o)
        yrs[o] = __builtin_amdgcn_make_buffer_rsrc((void*)(yb + o * ostride), (short)0,
                                                   (int)(ostride * (int64_t)sizeof(Tout)),
                                                   0x00020000);
    // PL_S_OOBST: lanes that do not own their column store to a byte offset past the
    // plane (the buffer range check drops the write) instead of branching around it
    const unsigned obytecol = (!PL_S_OOBST || own) ? ocol * (unsigned)sizeof(Tout) : 0x80000000u;
#pragma unroll
    for (int k = 0; k < NSET; ++k) FI[k] = GI[k] = 0.f;

    auto issue = [&](auto SETc, uint4 t) {     // loads for the u row of table entry t
        constexpr int SET = decltype(SETc)::value;
        const unsigned r0 = uniform((int)t.x), r1 = uniform((int)t.y);
        if (PL_S_FIV) {
            FI[SET] = __builtin_bit_cast(float, t.z);      // broadcast VGPR operands
            GI[SET] = __builtin_bit_cast(float, t.w);
        } else {
            FI[SET] = __builtin_bit_cast(float, uniform((int)t.z));
            GI[SET] = __builtin_bit_cast(float, uniform((int)t.w));
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if constexpr (X16) {
                X[SET][c] = u16x2{buf_load<unsigned short>(xrs[c], lbyte, r0),
                                  buf_load<unsigned short>(xrs[c], lbyte, r1)};
            } else {
                X[SET][c][0] = buf_load<Tin>(xrs[c], lbyte, r0);
                X[SET][c][1] = buf_load<Tin>(xrs[c], lbyte, r1);
            }
        }
    };

    // u row r in slot r % 3 at lane shifts -1 .. DKMAX-1.  For three channels the
    // values are held as a (c0, c1) pair + c2, the operand shape of the packed conv.
    constexpr bool PK = C == 3 && O == 3 && G == 1;
    constexpr int CS = PK ? 1 : C;      // scalar channels kept in U
    float2v UP[3][NS];                  // (c0, c1)         (PK only)
    float U[3][NS][CS];                 // c2 (PK) or all channels
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
        for (int d = 0; d < NS; ++d) {
            UP[s3][d] = float2v{0.f, 0.f};
#pragma unroll
            for (int c = 0; c < CS; ++c) U[s3][d][c] = 0.f;
        }

    // u row r from register set SET into slot SL
    auto compute_u = [&](auto SLc, auto SETc, int r) {
        constexpr int SL = decltype(SLc)::value;
        constexpr int SET = decltype(SETc)::value;
        const bool uok = (r >= 0 && r < F.h1) && col_in_w1;
        float uv[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            float x0, x1;
            if constexpr (X16) {
                x0 = to_acc<float>(__builtin_bit_cast(Tin, (unsigned short)X[SET][c].x));
                x1 = to_acc<float>(__builtin_bit_cast(Tin, (unsigned short)X[SET][c].y));
            } else {
                x0 = to_acc<float>(X[SET][c][0]);
                x1 = to_acc<float>(X[SET][c][1]);
            }
            const float v = fmaf(FI[SET], x1, GI[SET] * x0);         // t = fi*p3 + (1-fi)*p1
            const float vp = dpp_next(v);
            float u;
            if constexpr (R3)
                u = fmaf(wr[0], dpp_prev(v), fmaf(wr[1], v, wr[2] * vp));
            else
                u = fmaf(wr[0], dpp_prev(v), fmaf(wr[1], v, fmaf(wr[2], vp, wr[3] * dpp_next(vp))));
            uv[c] = uok ? u : colpad;                                 // pad rows / cols
        }
        float sh[NS][C];                // lane shifts -1 .. DKMAX-1 of every channel
#pragma unroll
        for (int c = 0; c < C; ++c) {
            sh[1][c] = uv[c];
            sh[0][c] = dpp_prev(uv[c]);
            sh[2][c] = dpp_next(uv[c]);
            if constexpr (NS == 4) sh[3][c] = dpp_next(sh[2][c]);
        }
#pragma unroll
        for (int d = 0; d < NS; ++d) {
            if constexpr (PK) {
                UP[SL][d] = float2v{sh[d][0], sh[d][1]};
                U[SL][d][0] = sh[d][2];
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) U[SL][d][c] = sh[d][c];
            }
        }
    };

    // kernel weights, loaded once into VGPRs.  For C = O = 3, groups 1: per output o
    // and tap t the pair (w[o][0][t], w[o][1][t]) for the packed (c0, c1) FMA, and
    // w[o][2][t] for c2.  An opaque per-lane zero makes these vector loads (the
    // SGPRs are needed for the row / descriptor state).
    int vz = 0;
    asm volatile("" : "+v"(vz));
    const float* kv = kern + vz;
    float2v wp2[PK ? O * 7 : 1];
    float wk[PK ? O * 7 : O * CG * 7], bs[O];
    if constexpr (PK) {
#pragma unroll
        for (int o = 0; o < O; ++o)
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                wp2[o * 7 + t] = float2v{kv[(o * 3 + 0) * 7 + t], kv[(o * 3 + 1) * 7 + t]};
                wk[o * 7 + t] = kv[(o * 3 + 2) * 7 + t];
            }
    } else {
#pragma unroll
        for (int i = 0; i < O * CG * 7; ++i) wk[i] = kv[i];
    }
#pragma unroll
    for (int o = 0; o < O; ++o) bs[o] = bias ? bias[o] : 0.f;     // scalar loads: SGPRs

    // HexConv2d row a2 from the u slots
    auto conv_row = [&](auto PHc, int a2, float* z) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int PAR = PH & 1;
        constexpr int SLT[3] = {(PH + 2) % 3, PH % 3, (PH + 1) % 3};   // rows a2-1, a2, a2+1
        const bool zok = a2 < F.ho && col_in_wo;
        if constexpr (PK) {
            // per output: packed FMA over the (c0, c1) pair + scalar FMA for c2
#pragma unroll
            for (int o = 0; o < 3; ++o) {
                float2v ap = {bs[o], 0.f};
                float as = 0.f;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int sl = SLT[tap_ii(t)];
                    const int dk = tap_dk(t, PAR, OP);
                    ap = pk_fma(wp2[o * 7 + t], UP[sl][dk], ap);
                    as = fmaf(wk[o * 7 + t], U[sl][dk][0], as);
                }
                z[o] = zok ? (ap.x + ap.y) + as : 0.f;
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
                                   U[SLT[tap_ii(t)]][tap_dk(t, PAR, OP)][c], acc);
                }
                z[o] = zok ? acc : 0.f;
            }
        }
    };

    // one output row a2 (phase PH = a2 % 6): u row a2+1 lives in set (PH + 1) % NSET.
    // The table entry of the row issued at a step is read from LDS one step earlier.
    uint4 tl[2];
    auto step = [&](auto PHc, int a2) {
        constexpr int PH = decltype(PHc)::value;
        issue(std::integral_constant<int, (PH + 1 + PD) % NSET>{}, tl[PH & 1]);
        tl[(PH + 1) & 1] = lut[a2 + 2 + PD - ubase];
        compute_u(std::integral_constant<int, (PH + 1) % 3>{},
                  std::integral_constant<int, (PH + 1) % NSET>{}, a2 + 1);
        float z[O];
        conv_row(PHc, a2, z);
        const unsigned obyte = (unsigned)uniform(a2 * F.w2) * (unsigned)sizeof(Tout);
#pragma unroll
        for (int o = 0; o < O; ++o) {
            float out;
            if constexpr ((PH & 1) == 0)   // even row: 0.75 z[b] + 0.25 z[b+1]
                out = fmaf(0.75f, z[o], 0.25f * dpp_next(z[o]));
            else                           // odd row: 0.25 z[b-1] + 0.75 z[b]
                out = fmaf(0.25f, dpp_prev(z[o]), 0.75f * z[o]);
            if (PL_S_OOBST || own) buf_store<Tout>(from_acc<Tout>(out), yrs[o], obytecol, obyte);
        }
    };

    // prologue: u rows a2_begin-1 (slot 2) and a2_begin (slot 0), rect rows of u rows up
    // to a2_begin + PD in flight (u row r uses set (r - a2_begin) mod NSET)
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, 2>;
    issue(std::integral_constant<int, NSET - 1>{}, lut[0]);
    issue(I0{}, lut[1]);
    issue(std::integral_constant<int, 1>{}, lut[2]);
    if constexpr (NSET == 3) {          // PD == 2: set 2 is reused by u row a2_begin + 2
        compute_u(I2{}, I2{}, a2_begin - 1);
        issue(I2{}, lut[3]);
    } else {
        issue(I2{}, lut[3]);
        if constexpr (PD >= 3) issue(std::integral_constant<int, 3>{}, lut[4]);
        if constexpr (PD >= 4) issue(std::integral_constant<int, 4>{}, lut[5]);
        compute_u(I2{}, std::integral_constant<int, NSET - 1>{}, a2_begin - 1);
    }
    compute_u(I0{}, I0{}, a2_begin);
    tl[0] = lut[PD + 2];                // u row a2_begin + 1 + PD
    for (int base = a2_begin; base < a2_end; base += 6) {
        step(std::integral_constant<int, 0>{}, base);
        if (base + 1 >= a2_end) break;
        step(std::integral_constant<int, 1>{}, base + 1);
        if (base + 2 >= a2_end) break;
        step(std::integral_constant<int, 2>{}, base + 2);
        if (base + 3 >= a2_end) break;
        step(std::integral_constant<int, 3>{}, base + 3);
        if (base + 4 >= a2_end) break;
        step(std::integral_constant<int, 4>{}, base + 4);
        if (base + 5 >= a2_end) break;
        step(std::integral_constant<int, 5>{}, base + 5);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

// Exact range of jn(q) - q over the hex columns q (r2h reads v at jn, jn+1).
static void r2h_offsets(const Geom& g, int* lo, int* hi) {
    int mn = INT_MAX, mx = INT_MIN;
    for (int64_t q = 0; q < g.w1; ++q) {
        const double j_ = axis_at(g.ys, q) + (double)(g.w - 1) * 0.5;
        const int64_t jn = (int64_t)j_;
        mn = (int)std::min<int64_t>(mn, jn - q);
        mx = (int)std::max<int64_t>(mx, jn - q);
    }
    *lo = mn; *hi = mx;
}

// The same over the columns with at least one r2h tap (jn or jn+1) inside [0, w): a
// column with none reads zeros whatever the window (used by the static kernel).
static void r2h_offsets_live(const Geom& g, int* lo, int* hi) {
    int mn = INT_MAX, mx = INT_MIN;
    for (int64_t q = 0; q < g.w1; ++q) {
        const double j_ = axis_at(g.ys, q) + (double)(g.w - 1) * 0.5;
        const int64_t jn = (int64_t)j_;
        if (!((jn >= 0 && jn < g.w) || (jn + 1 >= 0 && jn + 1 < g.w))) continue;
        mn = (int)std::min<int64_t>(mn, jn - q);
        mx = (int)std::max<int64_t>(mx, jn - q);
    }
    *lo = mn; *hi = mx;
}

// h2r: c1 - b = trunc(j_) - s1 - b with j_ - s1 - b = r(a) + D(b), r(a) = 0.5*i_ - s1,
// D(b) = y_(b) + cj - b; trunc(j_) lies in (j_ - 1, j_ + 1), so c1 - b is an integer
// in the open interval (min(r)+min(D) - 1, max(r)+max(D) + 1).  O(h2 + w2) on the host.
static void h2r_offsets(const Geom& g, int* lo, int* hi, bool* on_rows, bool* identity_rows) {
    double dmin = 1e300, dmax = -1e300, rmin = 1e300, rmax = -1e300;
    *on_rows = true;
    *identity_rows = true;
    const double cj = ((double)g.w - 0.5) * 0.5;
    for (int64_t bb = 0; bb < g.w1; ++bb) {
        const double d = axis_at(g.ys, bb) + cj - (double)bb;
        dmin = std::min(dmin, d); dmax = std::max(dmax, d);
    }
    for (int64_t a = 0; a < g.h1; ++a) {
        const double i_ = axis_at(g.xs, a) + (double)(g.h - 1) * 0.5;
        const int64_t in = (int64_t)i_;
        const double r = 0.5 * i_ - (double)(int64_t)((double)(in + 1) / 2.0);
        if (i_ - (double)(float)in != 0.0) *on_rows = false;
        if (i_ != (double)a) *identity_rows = false;
        rmin = std::min(rmin, r); rmax = std::max(rmax, r);
    }
    *lo = (int)std::floor(dmin + rmin - 1.0 - 1e-9) + 1;
    *hi = (int)std::ceil(dmax + rmax + 1.0 + 1e-9) - 1;
}

template <typename Tin, typename Tout, int C, int O, int G>
static int launch_pipeline(const void* x, const float* k, const float* bias, void* y,
                           PipeGeom F, int mode, hipStream_t st) {
    const int64_t waves = F.B * (int64_t)F.nband * F.nwin;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(PL_THREADS);
    const Tin* xp = (const Tin*)x;
    Tout* yp = (Tout*)y;
#define HG_PL(OPV, DPPV, HZV) \
    hipLaunchKernelGGL((k_pipeline<Tin, Tout, C, O, G, OPV, DPPV, HZV>), grid, blk, 0, st, xp, \
                       k, bias, yp, F)
    // mode: 0 generic (bpermute), 1 DPP windows, 2 DPP windows + rows on hex rows,
    // 3 same-size static pipeline
    if (mode == 3 || mode == 4) {       // 4: static with the 3-tap r2h window
#define HG_PLS(OPV, R3V) hipLaunchKernelGGL((k_pipeline_s<Tin, Tout, C, O, G, OPV, R3V>), grid, \
                                            blk, 0, st, xp, k, bias, yp, F)
        if (mode == 4) { if (F.op) HG_PLS(1, true); else HG_PLS(0, true); }
        else { if (F.op) HG_PLS(1, false); else HG_PLS(0, false); }
#undef HG_PLS
    } else if (mode == 2) { if (F.op) HG_PL(1, true, true); else HG_PL(0, true, true); }
    else if (mode == 1) { if (F.op) HG_PL(1, true, false); else HG_PL(0, true, false); }
    else { if (F.op) HG_PL(1, false, false); else HG_PL(0, false, false); }
#undef HG_PL
    return launch_status();
}

template <typename Tin, typename Tout>
static int pipeline_channels(const void* x, const float* k, const float* b, void* y,
                             const PipeGeom& F, int C, int O, int G, int dpp, hipStream_t st) {
    if (C == 3 && O == 3 && G == 1) return launch_pipeline<Tin, Tout, 3, 3, 1>(x, k, b, y, F, dpp, st);
    if (C == 3 && O == 3 && G == 3) return launch_pipeline<Tin, Tout, 3, 3, 3>(x, k, b, y, F, dpp, st);
    if (C == 1 && O == 1 && G == 1) return launch_pipeline<Tin, Tout, 1, 1, 1>(x, k, b, y, F, dpp, st);
    return HG_EUNSUP;
}

}  // namespace hg

extern "C" int hg_pipeline_r2h_conv_h2r(const void* x, const float* kernel, const float* bias,
                                        void* y, int x_dtype, int y_dtype, int64_t batch,
                                        int64_t channels, int64_t out_channels, int64_t h,
                                        int64_t w, int64_t h1, int64_t w1, int64_t h2,
                                        int64_t w2, int padding, int groups,
                                        int even_odd_offset, double pad_value, void* stream) {
    using namespace hg;
    if (batch < 0 || h < 1 || w < 1 || h1 < 1 || w1 < 1 || h2 < 0 || w2 < 0 || padding < 0)
        return HG_EINVAL;
    if (groups < 1 || channels % groups || out_channels % groups) return HG_EINVAL;
    if (!kernel) return HG_EINVAL;
    if (h > INT_MAX / 4 || w > INT_MAX / 4 || h1 > INT_MAX / 4 || w1 > INT_MAX / 4 ||
        h2 > INT_MAX / 4 || w2 > INT_MAX / 4)
        return HG_ESHAPE;
    PipeGeom F;
    F.B = batch;
    F.h = (int)h; F.w = (int)w; F.h1 = (int)h1; F.w1 = (int)w1; F.h2 = (int)h2; F.w2 = (int)w2;
    F.p = padding;
    F.op = (even_odd_offset + padding) & 1;
    F.padv = (float)pad_value;
    // conv output size, radius 2, stride 1, dilation 1 (HexFrames.py:127-169)
    F.ho = F.h1 + 2 * padding - 2;
    F.wo = F.w1 + 2 * padding - 2;
    if (F.ho < 1 || 2 * (F.w1 + 2 * padding) - 1 < 5) return HG_ESHAPE;
    F.r2h = make_r2h(h, w, h1, w1);
    F.h2r = make_tri(F.ho, F.wo, h2, w2, 0.75);
    if (batch == 0 || h2 == 0 || w2 == 0) return HG_OK;
    if (!x || !y) return HG_EINVAL;
    const int C = (int)channels, O = (int)out_channels, G = groups;
    if (O * (C / G) * 7 > PL_KMAX || O > 3 || C > 3) return HG_EUNSUP;
    {   // the two-column streaming kernel (fused.hip) where its geometry holds
        const int rc = fused_try(x, kernel, bias, y, x_dtype, y_dtype, batch, C, O, G, h, w, h1,
                                 w1, h2, w2, padding, F.op, pad_value,
                                 reinterpret_cast<hipStream_t>(stream));
        if (rc != HG_EUNSUP) return rc;
    }
    // lane halo from the lattice maps
    int jlo, jhi, clo, chi;
    bool on_rows, identity_rows;
    r2h_offsets(F.r2h, &jlo, &jhi);          // jn - q
    h2r_offsets(F.h2r, &clo, &chi, &on_rows, &identity_rows); // c1 - b
    const int dkmax = F.op ? 2 : 3;
    const bool dpp = padding == 1 && jlo >= PL_RLO && jhi + 1 <= PL_RHI &&
                     clo >= PL_ZALO && chi + 1 <= PL_ZAHI &&
                     clo - 1 >= PL_ZBLO && chi + 1 <= PL_ZBHI;
    int rlo = jlo, rhi = jhi + 1;                       // v lanes read by u
    int zlo_off = -padding, zhi_off = dkmax - padding;  // u lanes read by z
    int olo = clo - 1, ohi = chi + 1;                   // z lanes read by the output
    if (dpp) {   // the DPP windows read their whole (compile-time) range
        rlo = PL_RLO; rhi = PL_RHI; zlo_off = -1; zhi_off = dkmax - 1;
        olo = PL_ZBLO; ohi = PL_ZAHI;
    }
    // mode 3: exactly same-size h2r (closed-form 2-tap rows), padding 1, DPP r2h window
    // (32-bit buffer offsets: planes below 2 GiB; a dropped store's offset is 2^31)
    const bool stat = dpp && identity_rows && h2 == F.ho && w2 == F.wo &&
                      h * w * 8 < ((int64_t)1 << 31) && h2 * w2 * 8 < ((int64_t)1 << 31);
    bool r3 = false;
    if (stat) {
        int llo, lhi;
        r2h_offsets_live(F.r2h, &llo, &lhi);
        r3 = llo >= -1 && lhi + 1 <= 1;
        if (r3) rhi = 1;
        olo = -1; ohi = 1;                   // 0.75 / 0.25 taps at b-1 .. b+1
    }
    const int u_lo = std::max(0, -rlo), u_hi = std::min(63, 63 - rhi);
    const int z_lo = u_lo - std::min(zlo_off, 0), z_hi = u_hi - std::max(zhi_off, 0);
    const int o_lo = z_lo - std::min(olo, 0), o_hi = z_hi - std::max(ohi, 0);
    if (o_hi - o_lo + 1 < 32) return HG_EUNSUP;   // not a near-identity geometry
    F.HL = o_lo;
    F.nown = o_hi - o_lo + 1;
    F.nwin = (int)((w2 + F.nown - 1) / F.nown);
    F.RB = stat ? 126 : 128;                 // static path: bands start at multiples of 6
    F.nband = (int)((h2 + F.RB - 1) / F.RB);
    const int mode = stat ? (r3 ? 4 : 3) : (dpp ? (on_rows ? 2 : 1) : 0);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (x_dtype) {
    case HG_BF16:
        switch (y_dtype) {
        case HG_BF16: return pipeline_channels<__bf16, __bf16>(x, kernel, bias, y, F, C, O, G, mode, st);
        case HG_F32: return pipeline_channels<__bf16, float>(x, kernel, bias, y, F, C, O, G, mode, st);
        default: return HG_EDTYPE;
        }
    case HG_F16:
        switch (y_dtype) {
        case HG_F16: return pipeline_channels<_Float16, _Float16>(x, kernel, bias, y, F, C, O, G, mode, st);
        case HG_F32: return pipeline_channels<_Float16, float>(x, kernel, bias, y, F, C, O, G, mode, st);
        default: return HG_EDTYPE;
        }
    case HG_F32:
        switch (y_dtype) {
        case HG_F32: return pipeline_channels<float, float>(x, kernel, bias, y, F, C, O, G, mode, st);
        case HG_BF16: return pipeline_channels<float, __bf16>(x, kernel, bias, y, F, C, O, G, mode, st);
        default: return HG_EDTYPE;
        }
    case HG_U8:
        switch (y_dtype) {
        case HG_F32: return pipeline_channels<uint8_t, float>(x, kernel, bias, y, F, C, O, G, mode, st);
        case HG_BF16: return pipeline_channels<uint8_t, __bf16>(x, kernel, bias, y, F, C, O, G, mode, st);
        default: return HG_EDTYPE;
        }
    default:
        return HG_EDTYPE;
    }
}

// rect -> hex -> rect round trip without a conv (BASELINE config 2) in one pass: replaces
// geometry_np.hex_to_rect_resample(geometry_np.rect_to_hex_resample(x, (h1, w1)), (h1, w1))
// (geometry_np.py:358-519 then :191-356, 'bilinear' / 'linear') for the same-size lattices
// (fused.hip, MD 2); HG_EUNSUP elsewhere (run the two resamplers instead).
extern "C" int hg_pipeline_r2h_h2r(const void* x, void* y, int x_dtype, int y_dtype,
                                   int64_t planes, int64_t h, int64_t w, int64_t h1, int64_t w1,
                                   void* stream) {
    using namespace hg;
    if (planes < 0 || h < 1 || w < 1 || h1 < 1 || w1 < 1) return HG_EINVAL;
    if (h > INT_MAX / 4 || w > INT_MAX / 4 || h1 > INT_MAX / 4 || w1 > INT_MAX / 4) return HG_ESHAPE;
    if (planes == 0) return HG_OK;
    if (!x || !y) return HG_EINVAL;
    return fused_rt_try(x, y, x_dtype, y_dtype, planes, h, w, h1, w1,
                        reinterpret_cast<hipStream_t>(stream));
}
