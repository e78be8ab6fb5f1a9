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
// weight pairs in SGPRs (102 SGPRs) and one rect row of prefetch keep it at 124 VGPRs, 4 waves
// per SIMD (21 pairs / 2 rows ahead: 150 VGPRs, 3 waves; both 1-3 % faster than k_fused MD 0
// in in-process A/Bs on three boxes, profiles/r04/f4/).
//
// Domain: fused_try's (same-size lattice, padding 1, value 0) with bf16 in and out, C = O = 3,
// groups 1, w and w2 multiples of 4.  Results within the fp32 rounding of k_fused MD 0 (the same
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
#define F4_PD 1                        // rect rows loaded ahead of use (1..4): 1 fits 124 VGPRs
#endif
#ifndef F4_WPS
#define F4_WPS 29                      // weight pairs in SGPRs (the rest in VGPRs): 102 SGPRs
#endif
#ifndef F4_ORDER
#define F4_ORDER 0                     // workgroup order (A/B): 0 group fastest, 1 band fastest
#endif
#ifndef F4_WPE
#define F4_WPE 4                       // waves per SIMD asked of the register allocator
#endif
#ifndef F4_DMA
#define F4_DMA 0                       // rect rows by per-wave LDS-DMA into a 6-row LDS ring (2-3
                                       // steps ahead, no VGPRs, no workgroup barrier) instead of
                                       // the register ring
#endif
#ifndef F4_SAUX
#define F4_SAUX 0                      // cache-policy bits of the output stores (A/B: 2 nt, 16 sc1)
#endif
#ifndef F4_LAUX
#define F4_LAUX 0                      // ... of the rect-row loads
#endif
#ifndef F4_DIAG_NOBEL
#define F4_DIAG_NOBEL 0                // diagnostic (wrong results): skip the stencil's 'below' taps
                                       // (36 of 132 packed FMAs per step) to test whether compute and
                                       // memory time add or overlap
#endif
#ifndef F4_DIAG_NOFP64
#define F4_DIAG_NOFP64 0               // diagnostic (wrong results): row table and column weights
                                       // from constants instead of the fp64 lattice (prologue cost)
#endif
#ifndef F4_NOMEM
#define F4_NOMEM 0                     // diagnostic floor: every row load / store hits row 0 of its
                                       // plane (cache-resident), the arithmetic unchanged (1: loads
                                       // and stores, 2: loads only, 3: stores only)
#endif
constexpr int F4_GW = 4, F4_THREADS = 256;
constexpr int F4_HL = 8, F4_OWN = 240;  // window halo (left) and owned columns
constexpr int F4_RB = F4_RB_;
#ifndef F4_RB_CONV_
#define F4_RB_CONV_ 18                 // MD 1: output rows per band (k_fused MD 1's fastest)
#endif
constexpr int F4_RB_CONV = F4_RB_CONV_;
static_assert(F4_RB_CONV % 6 == 0 && F4_RB_CONV > 0, "bands are whole 6-step blocks");
static_assert(F4_RB % 6 == 0 && F4_RB > 0, "bands are whole 6-step blocks");

typedef unsigned f4_u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void f4_unpack(f4_u2 r, fu_f2& a, fu_f2& b, unsigned hi16) {
    a = fu_f2{__builtin_bit_cast(float, r.x << 16), __builtin_bit_cast(float, r.x & hi16)};
    b = fu_f2{__builtin_bit_cast(float, r.y << 16), __builtin_bit_cast(float, r.y & hi16)};
}

// MD 0: rect -> hex -> HexConv2d -> hex -> rect (the headline).  MD 1: HexConv2d alone
// (HexFrames.py:96-169, radius 2, stride 1, padding 1, pad value 0), as k_fused MD 1: the u rows
// are the input rows (zeros outside the raster), no r2h / h2r, the conv rows stored as they
// complete; the band length is F4_RB_CONV.
template <int OP, int MD>
__global__ __launch_bounds__(F4_THREADS) __attribute__((amdgpu_waves_per_eu(F4_WPE)))
void k_fused4(const __bf16* __restrict__ x, const float* __restrict__ kern,
              const float* __restrict__ bias, __bf16* __restrict__ y, FusedGeom F) {
    constexpr int C = 3, O = 3;
    constexpr bool UIN = MD == 1;                    // u rows = input rows
    constexpr int PD = F4_PD;
    static_assert(PD >= 1 && PD <= 4, "raw ring: rows a2+2 .. a2+1+PD in flight in 6 slots");
    constexpr int NLUT_MAX = (F4_RB > F4_RB_CONV ? F4_RB : F4_RB_CONV) + 2;
    __shared__ float4 lut_all[F4_GW][NLUT_MAX];
    // DMA: per wave 6 row slots of 3 x 512 B (plane c of rect row R at slot (R - s0 + 2) % 6,
    // bytes c * 512 + 8 * lane = this lane's 4 columns); pairs of slots (0,1) (2,3) (4,5) are
    // contiguous, so two rows are three 1-KiB LDS-DMA pieces
    constexpr bool DMA = F4_DMA;
    constexpr int RSLOT = 3 * 512;
    __shared__ __attribute__((aligned(16))) unsigned char ring_all[DMA ? F4_GW : 1][DMA ? 6 * RSLOT : 16];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* const lut = lut_all[wslot];
    const unsigned char* const ring = ring_all[DMA ? wslot : 0];
    const unsigned ring_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)ring_all[DMA ? wslot : 0];
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (F.nwin + F4_GW - 1) / F4_GW;
    // block -> (window group, band, image): group fastest (F4_ORDER 0) or band fastest (1: the
    // bands of one window group run side by side, sharing their 4 halo rows in L2)
    // (2: group fastest, then image, then band: the waves resident together walk the same
    // rows of many images)
    const int grp = (int)(F4_ORDER == 1 ? (blk / F.nband) % ngrp : blk % ngrp);
    const int band = (int)(F4_ORDER == 1 ? blk % F.nband
                           : F4_ORDER == 2 ? blk / ((int64_t)ngrp * F.B) : (blk / ngrp) % F.nband);
    const int64_t b = F4_ORDER == 2 ? (blk / ngrp) % F.B : blk / ((int64_t)ngrp * F.nband);
    if (band >= F.nband) return;
    if (b >= F.B) return;                            // uniform per workgroup
    const int win = grp * F4_GW + wslot;             // may be >= nwin: runs, owns nothing
    const int W0 = win * F4_OWN - F4_HL;
    const int ce = W0 + 4 * lane;                    // columns ce .. ce + 3 (pairs A, B)
    constexpr int RB = MD == 1 ? F4_RB_CONV : F4_RB, NLUT = RB + 2;
    const int s0 = band * RB;
    const int s1 = min(s0 + RB, F.h2);

    // ---- row table (fp64 lattice math, geometry_np.py:440-486), as k_fused -------------
    for (int e = lane; e < NLUT; e += 64) {
        const int r = s0 - 1 + e;
        float4 t = {0.f, 0.f, 0.f, 0.f};
        if (UIN) {
            t.y = (r >= 0 && r < F.h) ? 1.f : 0.f;       // u row r = input row r; 0: padding row
        } else if (F4_DIAG_NOFP64) {
            t.x = 0.25f; t.y = 0.75f;
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
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
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

    // ---- per-lane column weights of the two pairs (geometry_np.py:441-449, 514-517) -------
    // with the h2r 0.75 folded in (u' = 0.75 u: FU_FOLD of k_fused)
    float we[2][3], wo[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float* wr = s ? wo[k] : we[k];
            wr[0] = wr[1] = wr[2] = 0.f;
            const int q = ce + 2 * k + s;
            if (F4_DIAG_NOFP64) {
                wr[0] = 0.25f; wr[1] = 0.75f;
            } else if (!UIN && q >= 0 && q < F.w1) {
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
    const bool colin = ce >= 0 && ce < F.w;          // MD 1: the lane's input columns (w % 4 == 0)

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
    auto row_off = [&](int k) -> unsigned {
        if (F4_NOMEM == 1 || F4_NOMEM == 2) return 0u;
        return (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)min(max(k, 0), F.h - 1) * xrow));
    };
    // DMA: piece j of a row pair (A, B) is 1 KiB: half-wave h (lanes 32 h .. 32 h + 31) moves the
    // 512-B plane row 2 j + h of [A0 A1 A2 B0 B1 B2], lane l the 16 B of columns W0 + 8 (l % 32)
    // .. + 7; columns left or right of the raster are out of the buffer range (zeros)
    const int dgc = W0 + 8 * (lane & 31);
    const unsigned dcol = (dgc >= 0 && dgc < F.w) ? (unsigned)dgc * 2u : 0x80000000u;
    const bool dhi = lane >= 32;
    const unsigned dv0 = dcol + (dhi ? xplane : 0u);              // A0 | A1   (+ row A)
    const unsigned dv1 = dcol + (dhi ? 0u : 2u * xplane);         // A2 | B0   (+ row A, hi: + B - A)
    const unsigned dv2 = dcol + (dhi ? 2u * xplane : xplane);     // B1 | B2   (+ row B)
    // rows R, R + 1 into the slot pair starting at even slot PS (inline asm: hipcc does not see
    // these loads, so it adds no vmcnt(0) before LDS reads; the waits are counted in step())
    auto dma_pair = [&](int R, auto PSc) {
        constexpr int PS = decltype(PSc)::value;
        const unsigned rA = row_off(R), rB = row_off(R + 1);
        const unsigned v1 = dv1 + (dhi ? rB - rA : 0u);
        const unsigned l0 = (unsigned)__builtin_amdgcn_readfirstlane((int)(ring_lds + PS * RSLOT));
        const unsigned l1 = l0 + 1024u, l2 = l0 + 2048u;
        unsigned keep;
        const unsigned a0 = dv0, a2 = dv2;
        const __amdgpu_buffer_rsrc_t rs = xrs;
        asm volatile("s_mov_b32 %0, m0\n\t"
                     "s_mov_b32 m0, %4\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %1, %7, %8 offen lds\n\t"
                     "s_mov_b32 m0, %5\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %2, %7, %8 offen lds\n\t"
                     "s_mov_b32 m0, %6\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %3, %7, %9 offen lds\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(a0), "v"(v1), "v"(a2), "s"(l0), "s"(l1), "s"(l2), "s"(rs), "s"(rA), "s"(rB)
                     : "memory");
    };
    auto dma_read = [&](int R, f4_u2 (&r)[3]) {
        const unsigned char* const src = ring + fu_mod(R - s0 + 2, 6) * RSLOT + 8 * lane;
#pragma unroll
        for (int c = 0; c < 3; ++c) r[c] = *reinterpret_cast<const f4_u2*>(src + c * 512);
    };

    // ---- weights (21 pairs in SGPRs, the rest opaque VGPR pairs) and bias ---------------
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
    for (int o = 0; o < O; ++o) bv[o] = bias ? bias[o + vz] * (MD == 0 ? 0.75f : 1.f) : 0.f;
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

    auto run = [&](auto CDc, auto RCc) {
        constexpr int CD = decltype(CDc)::value;
        constexpr int RC = decltype(RCc)::value;
        f4_u2 raw[6][C];                    // rect rows in flight, slot (row - s0) % 6
        fu_f2 XA[3][C], XB[3][C];           // rect rows as f32 pairs A / B, slot (row - s0) % 3
        fu_f2 ZA[3][O], ZB[3][O];           // conv rows being accumulated, slot (row - s0) % 3

        auto issue = [&](auto SLc, int k) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned so = row_off(k);
#pragma unroll
            for (int c = 0; c < C; ++c) raw[SL][c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, so + c * xplane, F4_LAUX);
        };
        auto convert = [&](auto RSc, auto XSc) {
            constexpr int RS = decltype(RSc)::value, XS = decltype(XSc)::value;
#pragma unroll
            for (int c = 0; c < C; ++c) f4_unpack(raw[RS][c], XA[XS][c], XB[XS][c], hi16);
        };

        // u row r (= s0 + PH + 1) from rect rows r-1, r, r+1 (XP slots PH, PH+1, PH+2 mod 3),
        // scattered into conv rows r+1 (above; slot PH+2, started with the bias), r (centre;
        // slot PH+1) and r-1 (below; slot PH)
        auto urow = [&](auto PHc, float4 L, auto CENc, auto BELc) {
            constexpr int PH = decltype(PHc)::value;
            constexpr bool CEN = decltype(CENc)::value, BEL = decltype(BELc)::value;
            constexpr int S0 = fu_mod(PH, 3), S1 = fu_mod(PH + 1, 3), S2 = fu_mod(PH + 2, 3);
            constexpr int PB = fu_mod(PH, 2), PC = 1 - PB;
            const fu_f2 Lxy = {L.x, L.y}, Lzw = {L.z, L.w};
            fu_sfor<0, C>([&](auto Cc) {
                constexpr int c = decltype(Cc)::value;
                float ue[2], uo[2];
                if constexpr (UIN) {                // MD 1: u = input row r, 0 outside (padding 1)
                    if constexpr (RC == 1) {        // interior band and window: no selects
                        ue[0] = XA[S1][c].x; uo[0] = XA[S1][c].y;
                        ue[1] = XB[S1][c].x; uo[1] = XB[S1][c].y;
                    } else {
                        const bool in_ = colin && L.y != 0.f;
                        ue[0] = in_ ? XA[S1][c].x : 0.f; uo[0] = in_ ? XA[S1][c].y : 0.f;
                        ue[1] = in_ ? XB[S1][c].x : 0.f; uo[1] = in_ ? XB[S1][c].y : 0.f;
                    }
                } else {
                // vertical blend, packed (k_fused FU_VPK), for both pairs
                auto vblend = [&](const fu_f2 (&X)[3][C]) {
                    if constexpr (RC == 1) return fu_pfma<1, false>(Lxy, X[S1][c], fu_pmul<0>(Lxy, X[S0][c]));
                    else if constexpr (RC == 2) return fu_pfma<0, false>(Lzw, X[S2][c], fu_pmul<1>(Lxy, X[S1][c]));
                    else return fu_pfma<0, false>(Lzw, X[S2][c], fu_pfma<1, false>(Lxy, X[S1][c], fu_pmul<0>(Lxy, X[S0][c])));
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
                    if constexpr (c == 0) {       // the first tap of conv row r+1 adds the bias
                        constexpr bool WS = (j0 >> 1) < NWS;
                        const int s = fu_tap_shift(0, PB, OP);
                        const fu_f2 aA = s == -1 ? Um[0] : (s == 0 ? U0[0] : (s == 1 ? U1[0] : U2[0]));
                        const fu_f2 aB = s == -1 ? Um[1] : (s == 0 ? U0[1] : (s == 1 ? U1[1] : U2[1]));
                        ZA[S2][o] = fu_pfma_b<j0 & 1, o & 1, WS>(wkp[j0 >> 1], aA, bvp[o >> 1]);
                        ZB[S2][o] = fu_pfma_b<j0 & 1, o & 1, WS>(wkp[j0 >> 1], aB, bvp[o >> 1]);
                    } else {
                        tapk(IC<0>{}, ZA[S2][o], ZB[S2][o], PB);
                    }
                    tapk(IC<1>{}, ZA[S2][o], ZB[S2][o], PB);
                    if constexpr (CEN) {
                        tapk(IC<2>{}, ZA[S1][o], ZB[S1][o], PC);
                        tapk(IC<3>{}, ZA[S1][o], ZB[S1][o], PC);
                        tapk(IC<4>{}, ZA[S1][o], ZB[S1][o], PC);
                    }
                    if constexpr (BEL && !F4_DIAG_NOBEL) {
                        tapk(IC<5>{}, ZA[S0][o], ZB[S0][o], PB);
                        tapk(IC<6>{}, ZA[S0][o], ZB[S0][o], PB);
                    }
                });
            });
        };

        // conv row a2 (slot PH % 3, parity PH % 2) -> output row a2 (the folded same-size h2r:
        // even rows z'[b] + z'[b+1] / 3, odd rows z'[b-1] / 3 + z'[b], geometry_np.py:347-354)
        auto out_row = [&](auto PHc, int a2) {
            constexpr int PH = decltype(PHc)::value;
            constexpr int S0 = PH % 3;
            const unsigned so = (F4_NOMEM == 1 || F4_NOMEM == 3) ? 0u : (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a2 * yrow));
#pragma unroll
            for (int o = 0; o < O; ++o) {
                const fu_f2 zA = ZA[S0][o], zB = ZB[S0][o];
                float o0, o1, o2, o3;
                if constexpr (MD == 1) {            // HexConv2d output row as is
                    o0 = zA.x; o1 = zA.y; o2 = zB.x; o3 = zB.y;
                } else if constexpr ((PH & 1) == 0) {
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
                __builtin_amdgcn_raw_buffer_store_b64(v, yrs, yoff, so + o * yplane, F4_SAUX);
            }
        };

        // ---- prologue: u rows s0-1 and s0 -----------------------------------------------
        if constexpr (DMA) {
            dma_pair(s0 - 2, IC<0>{});
            dma_pair(s0, IC<2>{});
            dma_pair(s0 + 2, IC<4>{});
            __builtin_amdgcn_s_waitcnt(0x0f70);                         // vmcnt(0)
            asm volatile("" ::: "memory");
            f4_u2 t0[C], t1[C], t2[C];
            dma_read(s0 - 2, t0);
            dma_read(s0 - 1, t1);
            dma_read(s0, t2);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                f4_unpack(t0[c], XA[1][c], XB[1][c], hi16);   // row s0-2 -> slot 1
                f4_unpack(t1[c], XA[2][c], XB[2][c], hi16);   // row s0-1 -> slot 2
                f4_unpack(t2[c], XA[0][c], XB[0][c], hi16);   // row s0   -> slot 0
            }
            urow(IC<-2>{}, lut[0], std::false_type{}, std::false_type{});
            dma_read(s0 + 1, t0);
#pragma unroll
            for (int c = 0; c < C; ++c) f4_unpack(t0[c], XA[1][c], XB[1][c], hi16);   // row s0+1
            urow(IC<-1>{}, lut[1], std::true_type{}, std::false_type{});
        } else {
        {
            f4_u2 t0[C], t1[C], t2[C];
            const unsigned o0 = row_off(s0 - 2), o1 = row_off(s0 - 1), o2 = row_off(s0);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                t0[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o0 + c * xplane, 0);
                t1[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o1 + c * xplane, 0);
                t2[c] = __builtin_amdgcn_raw_buffer_load_b64(xrs, xoff, o2 + c * xplane, 0);
            }
            issue(IC<1>{}, s0 + 1);
#pragma unroll
            for (int i = 0; i < PD; ++i) {          // ring: rect rows s0+2 .. s0+1+PD
                if (i == 0) issue(IC<2>{}, s0 + 2);
                if (i == 1) issue(IC<3>{}, s0 + 3);
                if (i == 2) issue(IC<4>{}, s0 + 4);
                if (i == 3) issue(IC<5>{}, s0 + 5);
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                f4_unpack(t0[c], XA[1][c], XB[1][c], hi16);   // row s0-2 -> slot 1
                f4_unpack(t1[c], XA[2][c], XB[2][c], hi16);   // row s0-1 -> slot 2
                f4_unpack(t2[c], XA[0][c], XB[0][c], hi16);   // row s0   -> slot 0
            }
        }
        urow(IC<-2>{}, lut[0], std::false_type{}, std::false_type{});   // u row s0-1: above only
        convert(IC<1>{}, IC<1>{});                                      // row s0+1 -> slot 1
        urow(IC<-1>{}, lut[1], std::true_type{}, std::false_type{});    // u row s0: above, centre
        __builtin_amdgcn_s_waitcnt(0x0f70);                             // vmcnt(0)
        }

        // ---- main loop -----------------------------------------------------------------
        float4 lnext = lut[2];
        auto step = [&](auto PHc, int a2) {
            constexpr int PH = decltype(PHc)::value;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DMA) {
                // rect row a2+2 landed once at most the operations issued after its last piece
                // are outstanding (vmcnt counts LDS-DMA and stores together, in issue order):
                // even steps read the first row of the pair issued two steps back (after its
                // piece 1: piece 2 + 2 x 3 stores), odd steps the second row of the pair issued
                // three steps back (after piece 2: 3 x 3 stores + one pair); the prologue drains
                constexpr int N = (PH & 1) ? 12 : 7;
                __builtin_amdgcn_s_waitcnt((0x0f70 & ~0xf) | (N & 0xf));
                asm volatile("" ::: "memory");
                f4_u2 r[C];
                dma_read(a2 + 2, r);
#pragma unroll
                for (int c = 0; c < C; ++c) f4_unpack(r[c], XA[(PH + 2) % 3][c], XB[(PH + 2) % 3][c], hi16);
                if constexpr ((PH & 1) == 0) dma_pair(a2 + 4, IC<PH % 6>{});   // rows a2+4, a2+5
            } else {
            convert(IC<(PH + 2) % 6>{}, IC<(PH + 2) % 3>{});            // rect row a2+2
            issue(IC<(PH + 2 + PD) % 6>{}, a2 + 2 + PD);
            }
            const float4 L = lnext;
            lnext = lut[min(a2 - s0 + 3, NLUT - 1)];
            urow(PHc, L, std::true_type{}, std::true_type{});           // u row a2+1
            out_row(PHc, a2);
        };
        auto block6 = [&](int base) {
            step(IC<0>{}, base);
            step(IC<1>{}, base + 1);
            step(IC<2>{}, base + 2);
            step(IC<3>{}, base + 3);
            step(IC<4>{}, base + 4);
            step(IC<5>{}, base + 5);
        };
        auto tail = [&](int base) {
            if (base >= s1) return;
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
        };
        int base = s0;
        for (; base + 6 <= s1; base += 6) block6(base);
        tail(base);
        if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): no LDS-DMA in flight at exit
    };
    if constexpr (UIN) {
        (void)cd; (void)rc;
        // every u row of the band (s0 - 1 .. s1) and every lane's columns inside the input: the
        // padding selects drop out (RC 1 marks that loop for MD 1)
        const bool inner = s0 >= 1 && s1 + 1 <= F.h && __builtin_amdgcn_ballot_w64(!colin) == 0;
        if (inner) run(IC<0>{}, IC<1>{});
        else run(IC<0>{}, IC<0>{});
        return;
    }
    if (cd == 1 && rc == 1) run(IC<1>{}, IC<1>{});
    else if (cd == 1 && rc == 2) run(IC<1>{}, IC<2>{});
    else if (cd == 2 && rc == 1) run(IC<2>{}, IC<1>{});
    else if (cd == 2 && rc == 2) run(IC<2>{}, IC<2>{});
    else run(IC<0>{}, IC<0>{});
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
        hipLaunchKernelGGL((k_fused4<1, 0>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
    else
        hipLaunchKernelGGL((k_fused4<0, 0>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
    return launch_status();
}

// HexConv2d alone (radius 2, stride 1, padding 1, pad value 0, no epilogue) on the 4-column
// kernel (MD 1): bf16 in and out, C = O = 3, groups 1, w a multiple of 4; HG_EUNSUP otherwise
// (the caller runs k_fused MD 1).  op = tap column class at padding 1 ((off + 1) & 1).
int fconv4_try(const void* x, const float* k, const float* bias, void* y, int x_dtype, int y_dtype,
               int64_t batch, int C, int O, int G, int64_t h, int64_t w, int op, hipStream_t st) {
    // Opt-in (HYGRID_FCONV4=1): at 18-row bands 1.7 % SLOWER than k_fused MD 1 on the 4K bf16
    // b128 conv (2.710 vs 2.664 ms, profiles/r05/fconv4_ab.txt); bit-identical to it.
    if (!env_is("HYGRID_FCONV4", "1")) return HG_EUNSUP;
    if (x_dtype != HG_BF16 || y_dtype != HG_BF16 || C != 3 || O != 3 || G != 1) return HG_EUNSUP;
    if ((w % 4) || w < 4 || h < 1 || batch < 1) return HG_EUNSUP;
    if (3 * h * w * 2 >= ((int64_t)1 << 31)) return HG_EUNSUP;   // 32-bit offsets per image
    FusedGeom F = {};
    F.B = batch;
    F.h = F.h1 = F.h2 = (int)h;
    F.w = F.w1 = F.w2 = (int)w;
    F.nwin = (int)((w + F4_OWN - 1) / F4_OWN);
    F.nband = (int)((h + F4_RB_CONV - 1) / F4_RB_CONV);
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + F4_GW - 1) / F4_GW);
    if (blocks > INT_MAX) return HG_EUNSUP;
    const dim3 grid((unsigned)blocks), blk(F4_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused4<1, 1>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
    else
        hipLaunchKernelGGL((k_fused4<0, 1>), grid, blk, 0, st, (const __bf16*)x, k, bias, (__bf16*)y, F);
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
// the same for the HexConv2d mode (hg_fused_layout(8, ...))
void fconv4_layout(int* band_rows, int* win_own, int* win_halo) {
    *band_rows = F4_RB_CONV;
    *win_own = F4_OWN;
    *win_halo = F4_HL;
}
}  // namespace hg
