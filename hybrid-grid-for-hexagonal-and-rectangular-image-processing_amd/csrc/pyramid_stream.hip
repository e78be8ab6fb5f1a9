// pyramid_stream.hip — row-streaming form of one hex-pyramid level (BASELINE config 5):
//     Z = hexresize(HexConv2d_depthwise(X), (h1, w1))   for a 2x downsample
// The reference runs the two stages as separate calls: HexConv2d(C, C, off, 2,
// padding=1, groups=C) (HexFrames.py:96-169) and hexresize (geometry_np.py:520-681,
// 'linear').  k_pyr_level (pyramid.hip) stages 2-D tiles in LDS with two barriers per
// plane and spends most of its wave time parked; this kernel keeps everything in
// registers, like the fused pipeline (fused_kernel.h):
//
//  * one wavefront owns a window of 128 input columns (lane l <-> hex columns
//    W0 + 2l, W0 + 2l + 1, one dword of 16-bit input) of one image, all C channels,
//    and walks a band of output rows; lanes 2..61 own output column b = W0/2 + l;
//  * output row a needs conv rows R0 = i_n(a), R1 = R0 + 1 (geometry_np.py:601-620),
//    i.e. input rows R0 - 1 .. R0 + 2; for a 2x downsample i_n(a) - 2a is 0 or 1, so a
//    step consumes two new input rows, loaded two steps ahead into a 10-row register
//    ring (every input row is loaded once);
//  * conv rows R0, R1 at the lane's two columns: 7 taps x 2 columns x 2 rows, the
//    neighbour columns one DPP wave shift away (zeros outside the raster = padding 1);
//  * the triangle (geometry_np.py:612-648): p1 = (R0, c0), p2 = (R1, c1) if i_f > j_f
//    else (R0, c0 + 1), p3 = (R1, c1 + 1) with c0 = j_n - (i_n+1)//2,
//    c1 = j_n - (i_n+2)//2 (fp64 lattice per lane and row, the reference's expression
//    order); c0 - 2b in {-1, 0, 1} (host-checked), so every vertex is the lane's own
//    conv value or a neighbour lane's, picked with selects; vertices outside the raster
//    read 0 (:636-648);
//  * weights: the barycentric coordinates of the triangle in the lattice's (i, j) index
//    frame, where the reference's Cartesian frame (:651-656) is an affine image of it:
//    flag: (1 - i_f, i_f - j_f, j_f), else (1 - j_f, j_f - i_f, i_f) — the reference's
//    S1/S, S2/S, S3/S (:673-678) up to fp64 rounding, then rounded to fp32.
// Out-of-domain calls (other size ratios, odd widths, C not in {1, 3}) return HG_EUNSUP
// and k_pyr_level runs.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "lattice.h"

namespace hg {

constexpr int PS_THREADS = 256;    // 4 waves = 4 adjacent windows
constexpr int PS_OWN = 60;         // output columns per window (lanes 2..61)
#ifndef PS_RB_
#define PS_RB_ 30
#endif
constexpr int PS_RB = PS_RB_;      // output rows per band (multiple of 5 and 6: ring periods)

struct PyrStreamGeom {
    int64_t B;
    int h, w, h1, w1;
    int nwin, nband;
    Axis xs, ys;                   // hexresize lattice axes (geometry_np.py:570-582)
    Axis rxs, rys;                 // FR: rect_to_hex lattice axes (h, w) -> (h, w) (:415-422)
    const float* taps;             // [C][7]
    const float* bias;             // [C] or null
};

__device__ __forceinline__ float ps_prev(float v) {   // v[l-1], 0 at lane 0
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x138 /*wave_shr:1*/, 0xf, 0xf, true));
}
__device__ __forceinline__ float ps_next(float v) {   // v[l+1], 0 at lane 63
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
        __builtin_bit_cast(int, v), 0x130 /*wave_shl:1*/, 0xf, 0xf, true));
}

// r=2, padding-1 taps (HexFrames.py:108-118 in the type-1 frame; as fused_kernel.h):
// tap t of a conv row of parity par reads row +(ii-1), column +shift (shift in -1..2)
__host__ __device__ constexpr int ps_tap_ii(int t) { return t < 2 ? 0 : (t < 5 ? 1 : 2); }
__host__ __device__ constexpr int ps_tap_col(int t) {
    return t < 2 ? 1 + 2 * t : (t < 5 ? 2 * (t - 2) : 1 + 2 * (t - 5));
}
__host__ __device__ constexpr int ps_tap_shift(int t, int par, int op) {
    return ((1 + par + ps_tap_col(t) - ((((par + ps_tap_ii(t)) & 1) + op) & 1)) >> 1) - 1;
}
template <int N> using PIC = std::integral_constant<int, N>;

// FR = 1: the level input is the RECT image and X = rect_to_hex(rect) (geometry_np.py:
// 358-519, bilinear, same size, near-identity lattice) is made on the fly per X row: rows
// from a 12-row rect ring (one fp32 blend of rect rows in(r), in(r) + 1 with the row weights
// of a per-wave LDS table), columns from the lane's two columns and one DPP neighbour (the
// streaming r2h's expressions, k_r2h_stream).  Config 5 then never writes or re-reads the
// full-size hex image.
template <int OP, int C, int FR, typename Tin, typename Tout>
__global__ __launch_bounds__(PS_THREADS) void k_pyr_stream(const Tin* __restrict__ x,
                                                           Tout* __restrict__ y,
                                                           PyrStreamGeom G) {
    static_assert(sizeof(Tin) == 2, "16-bit input (one dword = the lane's two columns)");
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (G.nwin + 3) / 4;
    const int grp = (int)(blk % ngrp);
    const int64_t rest = blk / ngrp;
    const int band = (int)(rest % G.nband);
    const int64_t img = rest / G.nband;
    if (img >= G.B) return;                          // uniform per workgroup
    const int win = grp * 4 + wslot;                 // may be >= nwin: runs, owns nothing
    const int W0 = win * (2 * PS_OWN) - 4;           // input column of lane 0 (even)
    const int ce = W0 + 2 * lane;                    // lane's even column; odd = ce + 1
    const int bo = W0 / 2 + lane;                    // lane's output column
    const int a0 = band * PS_RB, a1 = min(a0 + PS_RB, G.h1);
    const bool own = lane >= 2 && lane < 2 + PS_OWN && bo < G.w1 && win < G.nwin;
    const bool colin = ce >= 0 && ce < G.w;          // w even: the dword is in or out

    // ---- per-lane lattice constants (fp64, geometry_np.py:570-602) ------------------
    const double yv = axis_at(G.ys, min(max(bo, 0), G.w1 - 1));   // y_ of this column
    const double cw = ((double)G.w - 0.5) * 0.5;
    const double ch = (double)(G.h - 1) * 0.5;

    // ---- buffers -------------------------------------------------------------------
    const int64_t ipl = (int64_t)G.h * G.w, opl = (int64_t)G.h1 * G.w1;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + img * C * ipl), (short)0, (int)(C * ipl * (int64_t)sizeof(Tin)), 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + img * C * opl), (short)0, (int)(C * opl * (int64_t)sizeof(Tout)), 0x00020000);
    const int lc = min(max(ce, 0), G.w - 2);
    // FR: rect columns outside the raster load as zeros (buffer range check), as the
    // streaming r2h reads them
    const unsigned xoff = (FR && !colin) ? 0x80000000u : (unsigned)lc * (unsigned)sizeof(Tin);
    const unsigned yoff = own ? (unsigned)bo * (unsigned)sizeof(Tout) : 0x80000000u;
    const unsigned xplane = (unsigned)(ipl * (int64_t)sizeof(Tin));
    const unsigned yplane = (unsigned)(opl * (int64_t)sizeof(Tout));
    const unsigned xrow = (unsigned)G.w * (unsigned)sizeof(Tin);
    const unsigned yrow = (unsigned)G.w1 * (unsigned)sizeof(Tout);

    // taps and bias in VGPRs (an SGPR operand halves the VALU issue rate on gfx950)
    int vz = 0;
    asm volatile("" : "+v"(vz));
    float wk[C * 7], bv[C];
#pragma unroll
    for (int i = 0; i < C * 7; ++i) wk[i] = G.taps[i + vz];
#pragma unroll
    for (int c = 0; c < C; ++c) bv[c] = G.bias ? G.bias[c + vz] : 0.f;

    // ---- input ring: rows rb0 + k in slot k % NR ------------------------------------
    // hex input: rows 2*a0 - 1 ..; FR: rect rows 2*a0 - 2 .. (X rows 2a-1+E .. 2a+2+E need
    // rect rows 2a-2 .. 2a+4)
    constexpr int NR = FR ? 12 : 10, PER = NR / 2;      // ring slots, steps per ring period
    const int rb0 = 2 * a0 - 1 - FR;
    unsigned raw[NR][C];
    auto issue = [&](auto SLc, int r) {
        constexpr int SL = decltype(SLc)::value;
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane(
            (int)((unsigned)min(max(r, 0), G.h - 1) * xrow));
#pragma unroll
        for (int c = 0; c < C; ++c)
            raw[SL][c] = __builtin_amdgcn_raw_buffer_load_b32(xrs, xoff, so + c * xplane, 0);
    };
    // input row -> f32 pair, zero outside the raster (the conv's constant-0 padding)
    auto xrowf = [&](auto SLc, int r, int c, float& e, float& o) {
        constexpr int SL = decltype(SLc)::value;
        const bool in = colin && r >= 0 && r < G.h;
        const unsigned v = raw[SL][c];
        e = in ? (float)__builtin_bit_cast(Tin, (unsigned short)(v & 0xffffu)) : 0.f;
        o = in ? (float)__builtin_bit_cast(Tin, (unsigned short)(v >> 16)) : 0.f;
    };

    // FR: per-wave table of the r2h rows of X rows 2*a0 - 1 + lane (geometry_np.py:440-449):
    // {in(r) - r + 1, weight of rect row in+1, weight of row in, validity bits}
    __shared__ float4 plut_all[PS_THREADS / 64][FR ? 64 : 1];
    float fjv[2] = {0.f, 0.f}, gjv[2] = {0.f, 0.f};
    bool leftv[2] = {false, false}, deadv[2] = {true, true};
    if constexpr (FR) {
        float4* plut = plut_all[wslot];
        const int r = 2 * a0 - 1 + lane;
        float4 t = {0.f, 0.f, 0.f, 0.f};
        if (r >= 0 && r < G.h) {
            const double i_ = axis_at(G.rxs, r) + (double)(G.h - 1) * 0.5;
            const int in = (int)i_;
            const double fi = i_ - (double)(float)in;
            t.x = (float)(in - r + 1);
            t.y = (float)fi;                          // row in + 1 (:515 c0 = fi)
            t.z = (float)(1.0 - fi);                  // row in
            t.w = (float)((in >= 0 && in < G.h ? 1 : 0) | (in + 1 >= 0 && in + 1 < G.h ? 2 : 0));
        }
        plut[lane] = t;
        // the lane's two columns (geometry_np.py:441-449): taps jn, jn + 1 with jn - q in
        // {-1, 0}; a column with no tap inside the raster is dead (both taps read 0)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int q = ce + k;
            if (q >= 0 && q < G.w) {
                const double j_ = axis_at(G.rys, q) + (double)(G.w - 1) * 0.5;
                const int jn = (int)j_;
                const double jf = j_ - (double)(float)jn;
                fjv[k] = (float)jf;
                gjv[k] = (float)(1.0 - jf);
                leftv[k] = jn < q;
                deadv[k] = !((jn >= 0 && jn < G.w) || (jn + 1 >= 0 && jn + 1 < G.w));
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0): own-wave LDS writes
        __builtin_amdgcn_wave_barrier();
    }
    // FR: X row r (table entry L) from rect rows in(r), in(r)+1 = ring slots S0 + sel, S0 +
    // sel + 1 (S0 = slot of rect row r - 1), the r2h blend of k_r2h_stream in fp32
    auto xrow_fr = [&](auto S0c, const float4 L, int r, int c, float& e, float& o) {
        constexpr int S0 = decltype(S0c)::value;
        const bool sel = L.x != 0.f;
        const unsigned ra = sel ? raw[(S0 + 1) % NR][c] : raw[S0][c];
        const unsigned rbv = sel ? raw[(S0 + 2) % NR][c] : raw[(S0 + 1) % NR][c];
        const unsigned val = (unsigned)L.w;
        float ae = (float)__builtin_bit_cast(Tin, (unsigned short)(ra & 0xffffu));
        float ao = (float)__builtin_bit_cast(Tin, (unsigned short)(ra >> 16));
        float be = (float)__builtin_bit_cast(Tin, (unsigned short)(rbv & 0xffffu));
        float bo_ = (float)__builtin_bit_cast(Tin, (unsigned short)(rbv >> 16));
        if (!(val & 1u)) { ae = 0.f; ao = 0.f; }           // uniform: a dead rect row
        if (!(val & 2u)) { be = 0.f; bo_ = 0.f; }
        const float te = L.y * be + L.z * ae, to = L.y * bo_ + L.z * ao;   // :515-516
        const float tm = ps_prev(to), tp = ps_next(te);   // columns ce - 1, ce + 2
        const float t1e = deadv[0] ? 0.f : (leftv[0] ? tm : te);
        const float t2e = deadv[0] ? 0.f : (leftv[0] ? te : to);
        const float t1o = deadv[1] ? 0.f : (leftv[1] ? te : to);
        const float t2o = deadv[1] ? 0.f : (leftv[1] ? to : tp);
        const bool in = colin && r >= 0 && r < G.h;          // X outside the raster: padding
        e = in ? fjv[0] * t2e + gjv[0] * t1e : 0.f;          // :517
        o = in ? fjv[1] * t2o + gjv[1] * t1o : 0.f;
    };

    // one output row a (ring offset K = a - a0 mod 5, static); E = i_n(a) - 2a
    // FR: X rows R0+1, R0+2 of a step, the next step's rows R0-1, R0 when both steps have
    // E = 0 (each X row is then made once); xc_ok says the cache holds them
    float xce[2][C], xco[2][C];
    bool xc_ok = false;
    auto step = [&](auto Kc, auto Ec, auto CACHEDc, int a, const double i_, int i_n) {
        constexpr int K = decltype(Kc)::value, E = decltype(Ec)::value;
        constexpr bool CACHED = decltype(CACHEDc)::value;
        // lattice of this (row, lane) (geometry_np.py:601-623)
        const double i_f = i_ - (double)(float)i_n;
        const double j_ = 0.5 * i_ + yv + cw;
        const int j_n = (int)j_;
        const double j_f = j_ - (double)(float)j_n;
        const bool flag = i_f > j_f;
        const float wa = (float)(flag ? 1.0 - i_f : 1.0 - j_f);
        const float wb = (float)(flag ? i_f - j_f : j_f - i_f);
        const float wg = (float)(flag ? j_f : i_f);
        const int R0 = i_n, R1 = i_n + 1;
        const int c0 = j_n - (i_n + 1) / 2, c1 = j_n - (i_n + 2) / 2;
        const int d0 = c0 - 2 * bo, d1 = c1 - 2 * bo;   // d0 in {-1,0,1}, d1 in {-2..1}
        // vertex validity (geometry_np.py:628-639); R0 >= 0 and R0 < h always
        const bool r1in = R1 < G.h;
        const bool v1 = c0 >= 0 && c0 < G.w;
        const bool v2 = flag ? (r1in && c1 >= 0 && c1 < G.w) : (c0 + 1 >= 0 && c0 + 1 < G.w);
        const bool v3 = r1in && c1 + 1 >= 0 && c1 + 1 < G.w;
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)a * yrow));
        float4 LT[4];                                  // FR: table rows of X rows R0-1 .. R0+2
        if constexpr (FR) {
#pragma unroll
            for (int k = 0; k < 4; ++k) LT[k] = plut_all[wslot][2 * (a - a0) + E + k];
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            // input rows R0-1 .. R0+2 = 2a-1+E .. 2a+2+E: ring slots (2K+E .. 2K+E+3) % 10;
            // FR: X rows made from rect rows, rect row R0 - 2 + k' in slot (2K+E+k') % 12
            float xe[4], xo[4];
            if constexpr (FR) {
                if constexpr (CACHED) {
                    xe[0] = xce[0][c]; xo[0] = xco[0][c];
                    xe[1] = xce[1][c]; xo[1] = xco[1][c];
                } else {
                    xrow_fr(PIC<(2 * K + E) % NR>{}, LT[0], R0 - 1, c, xe[0], xo[0]);
                    xrow_fr(PIC<(2 * K + E + 1) % NR>{}, LT[1], R0, c, xe[1], xo[1]);
                }
                xrow_fr(PIC<(2 * K + E + 2) % NR>{}, LT[2], R0 + 1, c, xe[2], xo[2]);
                xrow_fr(PIC<(2 * K + E + 3) % NR>{}, LT[3], R0 + 2, c, xe[3], xo[3]);
                xce[0][c] = xe[2]; xco[0][c] = xo[2];
                xce[1][c] = xe[3]; xco[1][c] = xo[3];
            } else {
                xrowf(PIC<(2 * K + E) % NR>{}, R0 - 1, c, xe[0], xo[0]);
                xrowf(PIC<(2 * K + E + 1) % NR>{}, R0, c, xe[1], xo[1]);
                xrowf(PIC<(2 * K + E + 2) % NR>{}, R0 + 1, c, xe[2], xo[2]);
                xrowf(PIC<(2 * K + E + 3) % NR>{}, R0 + 2, c, xe[3], xo[3]);
            }
            float pe[4], ne[4], no[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pe[k] = ps_prev(xo[k]);                 // column ce - 1
                ne[k] = ps_next(xe[k]);                 // column ce + 2
                no[k] = OP == 0 ? ps_next(xo[k]) : 0.f; // column ce + 3
            }
            const float* w = &wk[c * 7];
            // conv row R0 + q (parity (E + q) & 1) from input rows k = q + ii
            auto conv = [&](auto Qc, float& ye, float& yo) {
                constexpr int Q = decltype(Qc)::value, PAR = (E + Q) & 1;
                ye = bv[c];
                yo = bv[c];
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int k = Q + ps_tap_ii(t), s = ps_tap_shift(t, PAR, OP);
                    const float ae = s == -1 ? pe[k] : (s == 0 ? xe[k] : (s == 1 ? xo[k] : ne[k]));
                    const float ao = s == -1 ? xe[k] : (s == 0 ? xo[k] : (s == 1 ? ne[k] : no[k]));
                    ye = fmaf(w[t], ae, ye);
                    yo = fmaf(w[t], ao, yo);
                }
            };
            float y0e, y0o, y1e, y1o;
            conv(PIC<0>{}, y0e, y0o);
            conv(PIC<1>{}, y1e, y1o);
            // vertices: row R0 at columns 2b + d0 (+1), row R1 at 2b + d1 (+1)
            const float y0pm = ps_prev(y0o), y0ne = ps_next(y0e);
            const float y1pe = ps_prev(y1e), y1po = ps_prev(y1o), y1ne = ps_next(y1e);
            const float p1 = d0 < 0 ? y0pm : (d0 == 0 ? y0e : y0o);
            const float p2a = d0 < 0 ? y0e : (d0 == 0 ? y0o : y0ne);
            const float p2b = d1 < -1 ? y1pe : (d1 == -1 ? y1po : (d1 == 0 ? y1e : y1o));
            const float p3 = d1 < -1 ? y1po : (d1 == -1 ? y1e : (d1 == 0 ? y1o : y1ne));
            const float q1 = v1 ? p1 : 0.f;
            const float q2 = v2 ? (flag ? p2b : p2a) : 0.f;
            const float q3 = v3 ? p3 : 0.f;
            const float z = fmaf(wg, q3, fmaf(wb, q2, wa * q1));
            __builtin_amdgcn_raw_buffer_store_b16(
                __builtin_bit_cast(unsigned short, (Tout)z), yrs, yoff, so + c * yplane, 0);
        }
    };

    // per-row lattice (uniform; fp64 on every lane)
    auto row_lat = [&](int a, double& i_, int& i_n) {
        i_ = axis_at(G.xs, a) + ch;
        i_n = __builtin_amdgcn_readfirstlane((int)i_);
    };
    // step a (= a0 + K + PER m) with its prefetch of input rows 2a+6, 2a+7 (FR: rect rows
    // 2a+7, 2a+8)
    auto full = [&](auto Kc, int a) {
        constexpr int K = decltype(Kc)::value;
        issue(PIC<(2 * K + 7 + 2 * FR) % NR>{}, 2 * a + 6 + FR);
        issue(PIC<(2 * K + 8 + 2 * FR) % NR>{}, 2 * a + 7 + FR);
        double i_;
        int i_n;
        row_lat(a, i_, i_n);
        if (i_n == 2 * a) {
            if (FR && xc_ok) step(Kc, PIC<0>{}, std::true_type{}, a, i_, i_n);
            else step(Kc, PIC<0>{}, std::false_type{}, a, i_, i_n);
            xc_ok = FR;
        } else {                                  // i_n = 2a + 1 (host-checked)
            step(Kc, PIC<1>{}, std::false_type{}, a, i_, i_n);
            xc_ok = false;
        }
    };

    // prologue: input rows rb0 .. rb0 + 6 (FR: rect rows rb0 .. rb0 + 8)
    issue(PIC<0>{}, rb0);
    issue(PIC<1>{}, rb0 + 1);
    issue(PIC<2>{}, rb0 + 2);
    issue(PIC<3>{}, rb0 + 3);
    issue(PIC<4>{}, rb0 + 4);
    issue(PIC<5>{}, rb0 + 5);
    issue(PIC<6>{}, rb0 + 6);
    if constexpr (FR) {
        issue(PIC<7>{}, rb0 + 7);
        issue(PIC<8>{}, rb0 + 8);
    }
    int a = a0;
    for (; a + PER <= a1; a += PER) {
        full(PIC<0>{}, a);
        full(PIC<1>{}, a + 1);
        full(PIC<2>{}, a + 2);
        full(PIC<3>{}, a + 3);
        full(PIC<4>{}, a + 4);
        if constexpr (PER == 6) full(PIC<5>{}, a + 5);
    }
    if (a < a1) {
        full(PIC<0>{}, a);
        if (a + 1 < a1) {
            full(PIC<1>{}, a + 1);
            if (a + 2 < a1) {
                full(PIC<2>{}, a + 2);
                if (a + 3 < a1) {
                    full(PIC<3>{}, a + 3);
                    if (PER == 6 && a + 4 < a1) full(PIC<4>{}, a + 4);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// The lattice class the kernel assumes, checked on the lattice itself (O(h1 + w1)):
//   * i_n(a) - 2a in {0, 1} for every output row a;
//   * c0 - 2b = floor(0.5 i_f(a) - 0.5 e(a) + g(b)) in {-1, 0, 1}, with
//     g(b) = y_(b) + (w - 0.5)/2 - 2b: bounded by the extreme row and column terms plus
//     a margin for the fp64 rounding of j_.
static bool ps_lattice_ok(const Geom& g) {
    double qmin = 1e300, qmax = -1e300, gmin = 1e300, gmax = -1e300;
    const double ch = (double)(g.h - 1) * 0.5, cw = ((double)g.w - 0.5) * 0.5;
    for (int64_t a = 0; a < g.h1; ++a) {
        const double i_ = axis_at(g.xs, a) + ch;
        const int64_t in = (int64_t)i_;
        const int64_t e = in - 2 * a;
        if (e < 0 || e > 1 || in < 0 || in >= g.h) return false;
        const double q = 0.5 * (i_ - (double)in) - 0.5 * (double)e;
        qmin = std::min(qmin, q);
        qmax = std::max(qmax, q);
    }
    for (int64_t b = 0; b < g.w1; ++b) {
        const double gb = axis_at(g.ys, b) + cw - 2.0 * (double)b;
        gmin = std::min(gmin, gb);
        gmax = std::max(gmax, gb);
    }
    // (j_ = a + 2b + q + g >= -eps: the kernel's trunc is the floor of this bound, or one
    // more for a j_ rounded just below 0 at a = b = 0, where q + g = 0)
    const double eps = 1e-6;
    return qmin + gmin - eps >= -1.0 && qmax + gmax + eps < 2.0;
}

template <int OP, int C, int FR, typename Tin, typename Tout>
static int ps_launch(const void* src, void* dst, const PyrStreamGeom& G, hipStream_t st) {
    const int64_t blocks = G.B * (int64_t)G.nband * ((G.nwin + 3) / 4);
    if (blocks > INT_MAX) return HG_ESHAPE;
    hipLaunchKernelGGL((k_pyr_stream<OP, C, FR, Tin, Tout>), dim3((unsigned)blocks),
                       dim3(PS_THREADS), 0, st, (const Tin*)src, (Tout*)dst, G);
    return launch_status();
}

template <int OP, typename Tin, typename Tout>
static int ps_channels(const void* src, void* dst, const PyrStreamGeom& G, int C, int fr,
                       hipStream_t st) {
    if (C == 3) return fr ? ps_launch<OP, 3, 1, Tin, Tout>(src, dst, G, st)
                          : ps_launch<OP, 3, 0, Tin, Tout>(src, dst, G, st);
    if (C == 1) return fr ? ps_launch<OP, 1, 1, Tin, Tout>(src, dst, G, st)
                          : ps_launch<OP, 1, 0, Tin, Tout>(src, dst, G, st);
    return HG_EUNSUP;
}

// FR: the same-size rect -> hex lattice is near-identity (every live tap within one row /
// column below the sample's own index: in - r, jn - q in {-1, 0}), checked on the lattice
static bool ps_r2h_near_identity(const Geom& g) {
    for (int64_t q = 0; q < g.w1; ++q) {
        const int64_t jn = (int64_t)(axis_at(g.ys, q) + (double)(g.w - 1) * 0.5);
        const bool live = (jn >= 0 && jn < g.w) || (jn + 1 >= 0 && jn + 1 < g.w);
        if (live && (jn - q < -1 || jn - q > 0)) return false;
    }
    for (int64_t r = 0; r < g.h1; ++r) {
        const int64_t in = (int64_t)(axis_at(g.xs, r) + (double)(g.h - 1) * 0.5);
        const bool live = (in >= 0 && in < g.h) || (in + 1 >= 0 && in + 1 < g.h);
        if (live && (in - r < -1 || in - r > 0)) return false;
    }
    return true;
}

// One pyramid level on the streaming kernel, or HG_EUNSUP (the caller runs k_pyr_level).
// from_rect: src is the rect image and the level input is its same-size rect_to_hex.
// dry: launch nothing, return HG_PYR_STREAM if the kernel would run.
int pyr_stream_try(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                   int64_t C, int64_t h, int64_t w, int64_t h1, int64_t w1, const float* taps,
                   const float* bias, int even_odd_offset, int from_rect, hipStream_t st,
                   bool dry) {
    if (C != 1 && C != 3) return HG_EUNSUP;
    if ((w & 1) || w < 2 || h < 2 || h1 < 1 || w1 < 1) return HG_EUNSUP;
    if (src_dtype != dst_dtype || (src_dtype != HG_F16 && src_dtype != HG_BF16)) return HG_EUNSUP;
    if (reinterpret_cast<uintptr_t>(src) & 3) return HG_EUNSUP;   // dword loads
    if (C * h * w * 2 >= ((int64_t)1 << 31) || C * h1 * w1 * 2 >= ((int64_t)1 << 31))
        return HG_EUNSUP;                                         // 32-bit buffer offsets
    const Geom g = make_tri(h, w, h1, w1, 0.5);
    if (!ps_lattice_ok(g)) return HG_EUNSUP;
    PyrStreamGeom G;
    G.B = batch;
    G.h = (int)h; G.w = (int)w; G.h1 = (int)h1; G.w1 = (int)w1;
    G.nwin = (int)((w1 + PS_OWN - 1) / PS_OWN);
    G.nband = (int)((h1 + PS_RB - 1) / PS_RB);
    G.xs = g.xs;
    G.ys = g.ys;
    G.taps = taps;
    G.bias = bias;
    if (from_rect) {
        static_assert(2 * PS_RB + 4 <= 64, "the per-wave r2h row table holds 64 X rows");
        const Geom r = make_r2h(h, w, h, w);
        if (!ps_r2h_near_identity(r)) return HG_EUNSUP;
        G.rxs = r.xs;
        G.rys = r.ys;
    }
    if (dry) return HG_PYR_STREAM;
    const int op = (even_odd_offset + 1) & 1;   // tap column class at padding 1
    const int fr = from_rect ? 1 : 0;
    if (src_dtype == HG_F16)
        return op ? ps_channels<1, _Float16, _Float16>(src, dst, G, (int)C, fr, st)
                  : ps_channels<0, _Float16, _Float16>(src, dst, G, (int)C, fr, st);
    return op ? ps_channels<1, __bf16, __bf16>(src, dst, G, (int)C, fr, st)
              : ps_channels<0, __bf16, __bf16>(src, dst, G, (int)C, fr, st);
}

}  // namespace hg
