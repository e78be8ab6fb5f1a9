// fused4.hip — the headline pass (rect -> hex -> HexConv2d(r=2) -> hex -> rect, bf16 in and out,
// C = O = 3) with FOUR columns per lane (round 4): lane l owns columns ce .. ce + 3,
// ce = W0 + 4 l, of a 256-column window (240 owned, 8 + 8 halo), as two (even, odd) pairs
// A = (ce, ce + 1) and B = (ce + 2, ce + 3).  Everything else is k_fused MD 0 (fused_kernel.h):
// the per-wave row table and row classes, the per-lane column weights and column classes, the
// packed 7-tap stencil with 21 weight pairs in SGPRs, the folded same-size h2r, the 6-step blocks.
//
// Why: per owned column the 2-column kernel spends a neighbour exchange (DPP + pair copies) on
// every pair, 1/16 of its work on the 8-column window halo and reads 1.107x its input bytes;
// here the neighbours of pair A are pair B's values (no DPP), the halo is 1/32 and the reads
// ~1.04x; 8-B loads and stores per lane (walk6: the access pattern alone 0.615 -> 0.657 of
// 8 TB/s at 42-row bands, 0.73 at 18-24; profiles/r04/walk6_b.txt).  Registers: 29 of the 32
// weight pairs in SGPRs (106 SGPRs) and two rect rows of prefetch: 136 VGPRs, 3 waves per SIMD
// (round 6; one row of prefetch at 124 VGPRs and 4 waves was rounds 4-5's choice).
//
// Domain: fused_try's (same-size lattice, padding 1, value 0) with bf16 in and out, C = O = 3,
// groups 1, w and w2 multiples of 4.  (Round 5 also built this layout for HexConv2d alone and
// for the round trip, and a per-wave LDS-DMA row ring and cache-policy variants of this kernel:
// all measured slower; removed in round 6.)  Results within the fp32 rounding of k_fused MD 0 (the same
// products and sums per output; a tap order may differ), checked against the oracle chain.
#include <climits>
#include <cmath>
#include <cstdlib>

#include "fused_kernel.h"

namespace hg {

#ifndef F4_RB_
#define F4_RB_ 30                      // output rows per band (multiple of 6; 30 the most even across boxes: profiles/r04/f4)
#endif
#ifndef F4_PD
#define F4_PD 2                        // rect rows loaded ahead of use (1..4): 2 at 136 VGPRs, 3
                                       // waves per SIMD, is 0.9-2.1 % faster than 1 at 124 VGPRs
                                       // and 4 waves once the odd bands walk upwards (round 6,
                                       // profiles/r06/fused4_pd*_ab*.txt)
#endif
#ifndef F4_WPS
#define F4_WPS 29                      // weight pairs in SGPRs (the rest in VGPRs): 102 SGPRs
#endif
#ifndef F4_ORDER
#define F4_ORDER 0                     // workgroup order (A/B): 0 group fastest, 1 band fastest
#endif
#ifndef F4_WPE
#define F4_WPE 3                       // waves per SIMD asked of the register allocator
#endif
#ifndef F4_REV
#define F4_REV 1                       // odd full bands walk upwards (shared halo rows in L2, below)
#endif
constexpr int F4_GW = 4, F4_THREADS = 256;
constexpr int F4_HL = 8, F4_OWN = 240;  // window halo (left) and owned columns
constexpr int F4_RB = F4_RB_;
static_assert(F4_RB % 6 == 0 && F4_RB > 0, "bands are whole 6-step blocks");

typedef unsigned f4_u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void f4_unpack(f4_u2 r, fu_f2& a, fu_f2& b, unsigned hi16) {
    a = fu_f2{__builtin_bit_cast(float, r.x << 16), __builtin_bit_cast(float, r.x & hi16)};
    b = fu_f2{__builtin_bit_cast(float, r.y << 16), __builtin_bit_cast(float, r.y & hi16)};
}

// rect -> hex -> HexConv2d -> hex -> rect (the headline); OP = the stencil's tap column class
// at padding 1 ((even_odd_offset + 1) & 1).
//
// Band direction (F4_REV, round 6): a band reads its 30 output rows' rect rows plus 2 halo rows
// on each side, and the halo rows of two neighbouring bands are the same 4 rows.  Walking every
// band downwards, band k + 1 reads them first (at its start) and band k last (at its end), a
// whole band walk later, when they have long left the L2: the vertical halo comes from HBM
// twice (34 / 30 = 1.133x the input bytes).  With F4_REV the odd full bands walk upwards, so the
// two bands of a shared boundary reach it at the same time (both at their start, or both at
// their end) while they run side by side on one XCD.  A reversed band produces the same u rows
// (the vertical blend keeps its operand order), but each conv row then accumulates its below
// taps first and its above taps last: the same products, summed in another order (fp32
// rounding level; the bias still comes first).
template <int OP>
__global__ __launch_bounds__(F4_THREADS) __attribute__((amdgpu_waves_per_eu(F4_WPE)))
void k_fused4(const __bf16* __restrict__ x, const float* __restrict__ kern,
              const float* __restrict__ bias, __bf16* __restrict__ y, FusedGeom F) {
    constexpr int C = 3, O = 3;
    constexpr int PD = F4_PD;
    static_assert(PD >= 1 && PD <= 4, "raw ring: rows k+2 .. k+1+PD in flight in 6 slots");
    constexpr int RB = F4_RB, NLUT = RB + 2;
    __shared__ float4 lut_all[F4_GW][NLUT];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* const lut = lut_all[wslot];
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (F.nwin + F4_GW - 1) / F4_GW;
    // block -> (window group, band, image): group fastest (F4_ORDER 0) or band fastest (1)
    const int grp = (int)(F4_ORDER == 1 ? (blk / F.nband) % ngrp : blk % ngrp);
    const int band = (int)(F4_ORDER == 1 ? blk % F.nband : (blk / ngrp) % F.nband);
    const int64_t b = blk / ((int64_t)ngrp * F.nband);
    if (b >= F.B) return;                            // uniform per workgroup
    const int win = grp * F4_GW + wslot;             // may be >= nwin: runs, owns nothing
    const int W0 = win * F4_OWN - F4_HL;
    const int ce = W0 + 4 * lane;                    // columns ce .. ce + 3 (pairs A, B)
    const int s0 = band * RB;
    const int s1 = min(s0 + RB, F.h2);
    const bool up = F4_REV && (band & 1) && s1 - s0 == RB;   // uniform

    // ---- row table (fp64 lattice math, geometry_np.py:440-486), as k_fused -------------
    // entry e: u row s0 - 1 + e = {a, b, c}: u[r] = a x[r-1] + b x[r] + c x[r+1]
    for (int e = lane; e < NLUT; e += 64) {
        const int r = s0 - 1 + e;
        float4 t = {0.f, 0.f, 0.f, 0.f};
        if (r >= 0 && r < F.h1) {
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
    int rc;
    {
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

    // ---- per-lane column weights of the two pairs (geometry_np.py:441-449, 514-517) -------
    // with the h2r 0.75 folded in (u' = 0.75 u, as k_fused MD 0)
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
#pragma unroll
            for (int t = 0; t < 3; ++t) wr[t] *= 0.75f;
        }
    const bool any_l = __builtin_amdgcn_ballot_w64(we[0][0] != 0.f || wo[0][0] != 0.f ||
                                                   we[1][0] != 0.f || wo[1][0] != 0.f) != 0;
    const bool any_r = __builtin_amdgcn_ballot_w64(we[0][2] != 0.f || wo[0][2] != 0.f ||
                                                   we[1][2] != 0.f || wo[1][2] != 0.f) != 0;
    const int cd = !any_r ? 1 : (!any_l ? 2 : 0);

    // owned lanes 2 .. 61 (w2 % 4 == 0: a lane is wholly inside or outside the raster)
    const bool own = lane >= F4_HL / 4 && lane < (F4_HL + F4_OWN) / 4 && ce >= 0 && ce < F.w2 &&
                     win < F.nwin;

    // ---- buffers ----------------------------------------------------------------------
    const int64_t cstride = (int64_t)F.h * F.w, ostride = (int64_t)F.h2 * F.w2;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + b * C * cstride), (short)0, (int)(C * cstride * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + b * O * ostride), (short)0, (int)(O * ostride * 2), 0x00020000);
    const int lc = min(max(ce, 0), F.w - 4);         // clamped load column (x 0 weights outside)
    const unsigned xoff = (unsigned)lc * 2u;
    const unsigned yoff = own ? (unsigned)ce * 2u : 0x80000000u;
    const unsigned xplane = (unsigned)(cstride * 2), yplane = (unsigned)(ostride * 2);
    const unsigned xrow = (unsigned)F.w * 2u, yrow = (unsigned)F.w2 * 2u;
    auto row_off = [&](int r) -> unsigned {
        return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(r, 0), F.h - 1) * xrow));
    };

    // ---- weights (29 pairs in SGPRs, the rest opaque VGPR pairs) and bias ---------------
    int vz = 0;
    asm volatile("" : "+v"(vz));
    constexpr int NW = O * C * 7, NWP = (NW + 1) / 2;
    constexpr int NWS = F4_WPS < NWP ? F4_WPS : NWP;
    float wk[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) wk[i] = kern[i + (i / 2 < NWS ? 0 : vz)];
    fu_f2 wkp[NWP];
#pragma unroll
    for (int i = 0; i < NWP; ++i) {
        wkp[i] = fu_f2{wk[2 * i], 2 * i + 1 < NW ? wk[2 * i + 1] : 0.f};
        if (i >= NWS) asm volatile("" : "+v"(wkp[i]));
    }
    float bv[O];
#pragma unroll
    for (int o = 0; o < O; ++o) bv[o] = bias ? bias[o + vz] * 0.75f : 0.f;
    fu_f2 bvp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        bvp[i] = fu_f2{bv[2 * i], 2 * i + 1 < O ? bv[2 * i + 1] : 0.f};
        asm volatile("" : "+v"(bvp[i]));
    }
    float c13 = 1.f / 3.f;
    asm volatile("" : "+v"(c13));
    // h2r neighbours outside the raster (:303-323): pair B's right neighbour (even rows) and
    // pair A's left neighbour (odd rows); the inner ones are always inside
    const float wn_f = (ce + 4 < F.w2) ? c13 : 0.f;
    const float wp_f = (ce - 1 >= 0) ? c13 : 0.f;
    unsigned hi16 = 0xffff0000u;
    asm volatile("" : "+v"(hi16));

    // A band is walked in steps k = 0 .. s1 - s0 - 1 over output rows row(k): downwards
    // (row(k) = s0 + k) or, UP, upwards (row(k) = s1 - 1 - k).  Rect row / u row / conv row
    // row(k) lives in ring slot k mod 6 / k mod 3, so the slots and the row parities are
    // compile-time per step of a 6-step block in both directions.
    auto run = [&](auto CDc, auto RCc, auto UPc) {
        constexpr int CD = decltype(CDc)::value;
        constexpr int RC = decltype(RCc)::value;
        constexpr bool UP = decltype(UPc)::value;
        auto row = [&](int k) { return UP ? s1 - 1 - k : s0 + k; };
        // row-table entry of u row row(j)
        auto lut_e = [&](int j) { return UP ? RB - j : j + 1; };
        f4_u2 raw[6][C];                    // rect rows in flight, slot k % 6
        fu_f2 XA[3][C], XB[3][C];           // rect rows as f32 pairs A / B, slot k % 3
        fu_f2 ZA[3][O], ZB[3][O];           // conv rows being accumulated, slot k % 3

        // live false: the loads return zeros without a memory access (an offset past the buffer)
        auto issue = [&](auto SLc, int r, bool live = true) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned so = row_off(r);
            const unsigned vo = live ? xoff : 0x80000000u;
#pragma unroll
            for (int c = 0; c < C; ++c) raw[SL][c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, vo, so + c * xplane, 0);
        };
        auto convert = [&](auto RSc, auto XSc) {
            constexpr int RS = decltype(RSc)::value, XS = decltype(XSc)::value;
#pragma unroll
            for (int c = 0; c < C; ++c) f4_unpack(raw[RS][c], XA[XS][c], XB[XS][c], hi16);
        };

        // u row row(j), j = PH + 1, from rect rows row(PH), row(PH+1), row(PH+2) (slots S0, S1,
        // S2), scattered into conv rows row(PH+2) (started here with the bias: slot S2), row(PH+1)
        // (centre: S1) and row(PH) (completed here: S0).  Downwards the started row is the one
        // below (u row = its 'above' row: taps 0, 1), upwards the one above (taps 5, 6).
        auto urow = [&](auto PHc, float4 L, auto CENc, auto BELc) {
            constexpr int PH = decltype(PHc)::value;
            constexpr bool CEN = decltype(CENc)::value, BEL = decltype(BELc)::value;
            constexpr int S0 = fu_mod(PH, 3), S1 = fu_mod(PH + 1, 3), S2 = fu_mod(PH + 2, 3);
            // slots of rect rows r - 1 and r + 1 (r = row(PH + 1))
            constexpr int XM = UP ? S2 : S0, XQ = UP ? S0 : S2;
            // parity of the started / completed rows (row(PH) and row(PH + 2)); s0 and, for an
            // UP band, s1 are even
            constexpr int PB = UP ? fu_mod(PH + 1, 2) : fu_mod(PH, 2), PC = 1 - PB;
            constexpr int TN = UP ? 5 : 0, TD = UP ? 0 : 5;   // first tap of started / completed row
            const fu_f2 Lxy = {L.x, L.y}, Lzw = {L.z, L.w};
            fu_sfor<0, C>([&](auto Cc) {
                constexpr int c = decltype(Cc)::value;
                float ue[2], uo[2];
                // vertical blend, packed (as k_fused), for both pairs: a x[r-1] + b x[r] + c x[r+1]
                auto vblend = [&](const fu_f2 (&X)[3][C]) {
                    if constexpr (RC == 1) return fu_pfma<1, false>(Lxy, X[S1][c], fu_pmul<0>(Lxy, X[XM][c]));
                    else if constexpr (RC == 2) return fu_pfma<0, false>(Lzw, X[XQ][c], fu_pmul<1>(Lxy, X[S1][c]));
                    else return fu_pfma<0, false>(Lzw, X[XQ][c], fu_pfma<1, false>(Lxy, X[S1][c], fu_pmul<0>(Lxy, X[XM][c])));
                };
                const fu_f2 VA = vblend(XA), VB = vblend(XB);
                // horizontal blend: columns ce .. ce+3 = VA.x VA.y VB.x VB.y; the lane's left
                // neighbour column is the previous lane's VB.y, its right one the next lane's VA.x
                if constexpr (CD == 1) {            // taps q-1, q
                    ue[0] = fmaf(we[0][1], VA.x, we[0][0] * f_prev(VB.y));
                    uo[0] = fmaf(wo[0][1], VA.y, wo[0][0] * VA.x);
                    ue[1] = fmaf(we[1][1], VB.x, we[1][0] * VA.y);
                    uo[1] = fmaf(wo[1][1], VB.y, wo[1][0] * VB.x);
                } else if constexpr (CD == 2) {     // taps q, q+1
                    ue[0] = fmaf(we[0][2], VA.y, we[0][1] * VA.x);
                    uo[0] = fmaf(wo[0][2], VB.x, wo[0][1] * VA.y);
                    ue[1] = fmaf(we[1][2], VB.y, we[1][1] * VB.x);
                    uo[1] = fmaf(wo[1][2], f_next(VA.x), wo[1][1] * VB.y);
                } else {
                    const float pl = f_prev(VB.y), nx = f_next(VA.x);
                    ue[0] = fmaf(we[0][2], VA.y, fmaf(we[0][1], VA.x, we[0][0] * pl));
                    uo[0] = fmaf(wo[0][2], VB.x, fmaf(wo[0][1], VA.y, wo[0][0] * VA.x));
                    ue[1] = fmaf(we[1][2], VB.y, fmaf(we[1][1], VB.x, we[1][0] * VA.y));
                    uo[1] = fmaf(wo[1][2], nx, fmaf(wo[1][1], VB.y, wo[1][0] * VB.x));
                }
                // the stencil's column-shifted pairs (u[ce+s], u[ce+1+s]) for both pairs:
                // s = 0: own; s = 1: (uo_k, ue_{k+1}); s = -1: (uo_{k-1}, ue_k); s = 2: pair k+1
                const float nue = f_next(ue[0]);                 // next lane's u[ce + 4]
                const fu_f2 U0[2] = {fu_f2{ue[0], uo[0]}, fu_f2{ue[1], uo[1]}};
                const fu_f2 U1[2] = {fu_f2{uo[0], ue[1]}, fu_f2{uo[1], nue}};
                const fu_f2 Um[2] = {fu_f2{f_prev(uo[1]), ue[0]}, fu_f2{uo[0], ue[1]}};
                const fu_f2 U2[2] = {U0[1], fu_f2{nue, OP == 0 ? f_next(uo[0]) : 0.f}};
                fu_sfor<0, O>([&](auto OOc) {
                    constexpr int o = decltype(OOc)::value;
                    constexpr int j0 = (o * C + c) * 7;
                    auto tapk = [&](auto Tc, fu_f2& zA, fu_f2& zB, int par) {
                        constexpr int j = j0 + decltype(Tc)::value;
                        constexpr bool WS = (j >> 1) < NWS;
                        const int s = fu_tap_shift(decltype(Tc)::value, par, OP);
                        const fu_f2 aA = s == -1 ? Um[0] : (s == 0 ? U0[0] : (s == 1 ? U1[0] : U2[0]));
                        const fu_f2 aB = s == -1 ? Um[1] : (s == 0 ? U0[1] : (s == 1 ? U1[1] : U2[1]));
                        zA = fu_pfma<j & 1, WS>(wkp[j >> 1], aA, zA);
                        zB = fu_pfma<j & 1, WS>(wkp[j >> 1], aB, zB);
                    };
                    if constexpr (c == 0) {       // the first tap of the started row adds the bias
                        constexpr int jb = j0 + TN;
                        constexpr bool WS = (jb >> 1) < NWS;
                        const int s = fu_tap_shift(TN, PB, OP);
                        const fu_f2 aA = s == -1 ? Um[0] : (s == 0 ? U0[0] : (s == 1 ? U1[0] : U2[0]));
                        const fu_f2 aB = s == -1 ? Um[1] : (s == 0 ? U0[1] : (s == 1 ? U1[1] : U2[1]));
                        ZA[S2][o] = fu_pfma_b<jb & 1, o & 1, WS>(wkp[jb >> 1], aA, bvp[o >> 1]);
                        ZB[S2][o] = fu_pfma_b<jb & 1, o & 1, WS>(wkp[jb >> 1], aB, bvp[o >> 1]);
                    } else {
                        tapk(IC<TN>{}, ZA[S2][o], ZB[S2][o], PB);
                    }
                    tapk(IC<TN + 1>{}, ZA[S2][o], ZB[S2][o], PB);
                    if constexpr (CEN) {
                        tapk(IC<2>{}, ZA[S1][o], ZB[S1][o], PC);
                        tapk(IC<3>{}, ZA[S1][o], ZB[S1][o], PC);
                        tapk(IC<4>{}, ZA[S1][o], ZB[S1][o], PC);
                    }
                    if constexpr (BEL) {
                        tapk(IC<TD>{}, ZA[S0][o], ZB[S0][o], PB);
                        tapk(IC<TD + 1>{}, ZA[S0][o], ZB[S0][o], PB);
                    }
                });
            });
        };

        // conv row row(PH) (slot PH % 3) -> output row row(PH) (the folded same-size h2r: even
        // rows z'[b] + z'[b+1] / 3, odd rows z'[b-1] / 3 + z'[b], geometry_np.py:347-354)
        auto out_row = [&](auto PHc, int k) {
            constexpr int PH = decltype(PHc)::value;
            constexpr int S0 = PH % 3;
            constexpr int PAR = UP ? (PH + 1) & 1 : PH & 1;
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)row(k) * yrow));
#pragma unroll
            for (int o = 0; o < O; ++o) {
                const fu_f2 zA = ZA[S0][o], zB = ZB[S0][o];
                float o0, o1, o2, o3;
                if constexpr (PAR == 0) {
                    o0 = fmaf(c13, zA.y, zA.x);
                    o1 = fmaf(c13, zB.x, zA.y);
                    o2 = fmaf(c13, zB.y, zB.x);
                    o3 = fmaf(wn_f, f_next(zA.x), zB.y);
                } else {
                    o0 = fmaf(wp_f, f_prev(zB.y), zA.x);
                    o1 = fmaf(c13, zA.x, zA.y);
                    o2 = fmaf(c13, zA.y, zB.x);
                    o3 = fmaf(c13, zB.x, zB.y);
                }
                typedef __bf16 t2v __attribute__((ext_vector_type(2)));
                const f4_u2 v = {__builtin_bit_cast(unsigned, t2v{(__bf16)o0, (__bf16)o1}),
                                 __builtin_bit_cast(unsigned, t2v{(__bf16)o2, (__bf16)o3})};
                __builtin_amdgcn_raw_buffer_store_b64(v, yrs, yoff, so + o * yplane, 0);
            }
        };

        // ---- prologue: u rows row(-1) and row(0) ----------------------------------------
        {
            f4_u2 t0[C], t1[C], t2[C];
            const unsigned o0 = row_off(row(-2)), o1 = row_off(row(-1)), o2 = row_off(row(0));
#pragma unroll
            for (int c = 0; c < C; ++c) {
                t0[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o0 + c * xplane, 0);
                t1[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o1 + c * xplane, 0);
                t2[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o2 + c * xplane, 0);
            }
            issue(IC<1>{}, row(1));
#pragma unroll
            for (int i = 0; i < PD; ++i) {          // ring: rect rows row(2) .. row(1 + PD)
                if (i == 0) issue(IC<2>{}, row(2));
                if (i == 1) issue(IC<3>{}, row(3));
                if (i == 2) issue(IC<4>{}, row(4));
                if (i == 3) issue(IC<5>{}, row(5));
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                f4_unpack(t0[c], XA[1][c], XB[1][c], hi16);   // row(-2) -> slot 1
                f4_unpack(t1[c], XA[2][c], XB[2][c], hi16);   // row(-1) -> slot 2
                f4_unpack(t2[c], XA[0][c], XB[0][c], hi16);   // row(0)  -> slot 0
            }
        }
        urow(IC<-2>{}, lut[lut_e(-1)], std::false_type{}, std::false_type{});   // u row(-1): start only
        convert(IC<1>{}, IC<1>{});                                              // row(1) -> slot 1
        urow(IC<-1>{}, lut[lut_e(0)], std::true_type{}, std::false_type{});     // u row(0): start, centre
        __builtin_amdgcn_s_waitcnt(0x0f70);                                     // vmcnt(0)

        // ---- main loop -----------------------------------------------------------------
        const int n = s1 - s0;
        float4 lnext = lut[lut_e(1)];
        auto step = [&](auto PHc, int k) {
            constexpr int PH = decltype(PHc)::value;
            __builtin_amdgcn_sched_barrier(0);
            convert(IC<(PH + 2) % 6>{}, IC<(PH + 2) % 3>{});            // rect row row(k+2)
            // (a row past the band's last halo row is never read: its load goes out of range,
            // no memory access, instead of a 31st row from HBM)
            issue(IC<(PH + 2 + PD) % 6>{}, row(min(k + 2 + PD, n + 1)), k + 2 + PD <= n + 1);
            const float4 L = lnext;
            lnext = lut[min(max(lut_e(k + 2), 0), NLUT - 1)];
            urow(PHc, L, std::true_type{}, std::true_type{});           // u row row(k+1)
            out_row(PHc, k);
        };
        auto block6 = [&](int base) {
            step(IC<0>{}, base);
            step(IC<1>{}, base + 1);
            step(IC<2>{}, base + 2);
            step(IC<3>{}, base + 3);
            step(IC<4>{}, base + 4);
            step(IC<5>{}, base + 5);
        };
        int base = 0;
        for (; base + 6 <= n; base += 6) block6(base);
        if constexpr (!UP) {                            // (UP bands are whole 6-step blocks)
            if (base < n) {
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
            }
        }
    };
    auto dir = [&](auto CDc, auto RCc) {
        if (F4_REV && up) run(CDc, RCc, std::true_type{});
        else run(CDc, RCc, std::false_type{});
    };
    if (cd == 1 && rc == 1) dir(IC<1>{}, IC<1>{});
    else if (cd == 1 && rc == 2) dir(IC<1>{}, IC<2>{});
    else if (cd == 2 && rc == 1) dir(IC<2>{}, IC<1>{});
    else if (cd == 2 && rc == 2) dir(IC<2>{}, IC<2>{});
    else dir(IC<0>{}, IC<0>{});
}

// The 4-column kernel for a call fused_try has validated (same-size lattice, padding 1,
// value 0); HG_EUNSUP outside its narrower domain (the caller runs k_fused).
int fused4_try(const void* x, const float* k, const float* bias, void* y, int x_dtype, int y_dtype,
               int C, int O, int G, const FusedGeom& F0, int op, hipStream_t st) {
    if (env_is("HYGRID_FUSED4", "0")) return HG_EUNSUP;   // A/B switch: the 2-column kernel
    if (x_dtype != HG_BF16 || y_dtype != HG_BF16 || C != 3 || O != 3 || G != 1) return HG_EUNSUP;
    if ((F0.w % 4) || (F0.w2 % 4) || F0.w < 4) return HG_EUNSUP;
    FusedGeom F = F0;
    F.nwin = (int)((F.w2 + F4_OWN - 1) / F4_OWN);
    F.nband = (int)((F.h2 + F4_RB - 1) / F4_RB);
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + F4_GW - 1) / F4_GW);
    if (blocks > INT_MAX) return HG_EUNSUP;
    const dim3 grid((unsigned)blocks), blk(F4_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused4<1>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
    else
        hipLaunchKernelGGL((k_fused4<0>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
    return launch_status();
}

}  // namespace hg

namespace hg {
// band rows / owned columns / left halo of the 4-column kernel (hg_fused_layout(6, ...): tests
// place edge inputs from it)
void fused4_layout(int* band_rows, int* win_own, int* win_halo) {
    *band_rows = F4_RB;
    *win_own = F4_OWN;
    *win_halo = F4_HL;
}
}  // namespace hg
