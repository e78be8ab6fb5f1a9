// resample_stream.hip — row-streaming rect->hex and hex->rect kernels for the
// near-identity lattices (same-size resamples: the default `hex_dsize=None` /
// `rect_dsize=None` of geometry_np.py:373-376, :222-225, and BASELINE's configs).
//
// The general kernels (resample.hip) stage a 2-D footprint per (tile, plane) in LDS.
// When the lattice is a near identity every output sample's taps sit in the same or
// the neighbouring row and column, so a wavefront can own a window of one plane (4
// columns per lane for 16-bit data, 2 when either side is fp32: 4- or 8-byte loads and
// stores per lane) and walk a band of rows:
//
//  * r2h (geometry_np.py:440-517): output row r blends source rows in(r), in(r)+1 with
//    in(r) - r in {-1, 0} (per-row record from the fp64 lattice, one row per lane,
//    broadcast with readlane); output column q blends columns jn(q), jn(q)+1 with
//    jn(q) - q in {-1, 0} (per-lane constant).  The neighbour columns outside a lane
//    are one DPP shift away; those outside the window come from a one-dword edge load
//    issued by lanes 0 and 63 only.
//  * h2r (geometry_np.py:276-354) at (h1, w1) == (h, w): the lattice is exact
//    (i_ = a, j_ = 0.5 a + b + 0.25), so every output row of one parity is the same
//    3-tap triangle: even a: p1 = (a, b), p2 = (a, b+1); odd a: p1 = (a, b-1),
//    p2 = (a, b); p3 = (a+1, b) for both, with weights (alpha, beta, gamma) taken from
//    the shared fp64 triangle sample (lattice.h) on the host.
//
// Both evaluate exactly the general kernels' fp32 expressions in the same order
// (geometry_np.py:515-517 and :354; the library is built with -ffp-contract=off), and
// out-of-raster taps read 0 as there (:465-486, :303-323), so results are bit-identical
// to k_resample_lds for every input, NaN/Inf included.  The host (stream_try) proves
// the near-identity structure on the lattice itself before launching; anything else
// returns HG_EUNSUP and the general kernels run.
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "lattice.h"
#include "stream.h"

namespace hg {

constexpr int ST_THREADS = 256;     // 4 waves per workgroup: 4 adjacent windows
// Columns per lane: 4 when both sides are 16-bit (8-B loads and stores), 2 when either is
// fp32 (8-B fp32 loads: 16-B-per-lane rows walked by a wave measured 22 % slower than 8-B
// ones, tools/microbench/walk.hip, profiles/r02/probe/walk.txt).  Window = 64 lanes.
template <typename Tin, typename Tout>
constexpr int st_cpl() { return (sizeof(Tin) == 4 || sizeof(Tout) == 4) ? 2 : 4; }
// Rows per band (<= 128: 2 row records per lane; even: h2r row parity is static).  Short
// bands measured faster (more waves in flight over fewer rows of each image; in-process
// A/B on 4K bf16 b128, tools/ab_ops.py: r2h 2.60 -> 2.49 ms at 24, h2r 2.55 -> 2.37 ms at 16).
#ifndef ST_RB_R2H
#define ST_RB_R2H 24
#endif
#ifndef ST_RB_H2R
#define ST_RB_H2R 16
#endif
constexpr unsigned ST_OOB = 0x80000000u;   // buffer offset past num_records: loads 0, stores drop

struct StreamGeom {
    int64_t planes;
    int h, w, h1, w1;
    int nwin, nband, rb;            // windows, bands, rows per band
    Axis rxs, rys;                  // r2h axes
    float tri[2][3];                // h2r (alpha, beta, gamma) for even / odd output rows
};

template <typename T> struct Vec4Of { typedef unsigned type __attribute__((ext_vector_type(2))); };
template <> struct Vec4Of<float> { typedef unsigned type __attribute__((ext_vector_type(4))); };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t st_rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

// CPL consecutive elements (one lane's columns) as f32
template <typename T, int CPL>
__device__ __forceinline__ void st_load(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff,
                                        float* v) {
    if constexpr (sizeof(T) == 2 && CPL == 4) {
        const typename Vec4Of<T>::type r = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        typedef T t4 __attribute__((ext_vector_type(4)));
        const t4 e = __builtin_bit_cast(t4, r);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (float)e[k];
    } else if constexpr (sizeof(T) == 2) {
        typedef T t2 __attribute__((ext_vector_type(2)));
        const t2 e = __builtin_bit_cast(t2, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
        v[0] = (float)e[0];
        v[1] = (float)e[1];
    } else if constexpr (CPL == 4) {
        // whole-vector bit_cast: extracting lanes of the integer vector and casting each
        // (bit_cast(float, r[k])) is miscompiled by this toolchain's demanded-elements
        // narrowing of buffer loads (every element read as element 0)
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 e = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = e[k];
    } else {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 e = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
        v[0] = e[0];
        v[1] = e[1];
    }
}
// one dword holding the element at the window edge: lo / hi half for 16-bit types
template <typename T>
__device__ __forceinline__ void st_load_edge(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                             unsigned soff, float* lo, float* hi) {
    const unsigned r = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
    if constexpr (sizeof(T) == 2) {
        *lo = (float)__builtin_bit_cast(T, (unsigned short)(r & 0xffffu));
        *hi = (float)__builtin_bit_cast(T, (unsigned short)(r >> 16));
    } else {
        *lo = *hi = __builtin_bit_cast(float, r);
    }
}
template <typename T, int CPL>
__device__ __forceinline__ void st_store(const float* v, __amdgpu_buffer_rsrc_t rs, unsigned voff,
                                         unsigned soff) {
    if constexpr (sizeof(T) == 2 && CPL == 4) {
        typedef T t4 __attribute__((ext_vector_type(4)));
        const t4 e = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(typename Vec4Of<T>::type, e), rs,
                                              voff, soff, 0);
    } else if constexpr (sizeof(T) == 2) {
        typedef T t2 __attribute__((ext_vector_type(2)));
        const t2 e = {(T)v[0], (T)v[1]};
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, e), rs, voff, soff, 0);
    } else if constexpr (CPL == 4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 e = {v[0], v[1], v[2], v[3]};
        hg_store_b128(__builtin_bit_cast(hg_u4v, e), rs, voff, soff);
    } else {
        typedef float f2 __attribute__((ext_vector_type(2)));
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const f2 e = {v[0], v[1]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, e), rs, voff, soff, 0);
    }
}

// result[l] = v[l-1] (lane 0: old);  result[l] = v[l+1] (lane 63: old)
__device__ __forceinline__ float st_prev(float v, float old) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        __builtin_bit_cast(int, old), __builtin_bit_cast(int, v), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
}
__device__ __forceinline__ float st_next(float v, float old) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        __builtin_bit_cast(int, old), __builtin_bit_cast(int, v), 0x130 /*wave_shl:1*/, 0xf, 0xf, false));
}

// one source row as seen by a lane: its CPL columns and the window-edge dword halves
template <int CPL>
struct StRow {
    float v[CPL], el, eh;
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int k = 0; k < CPL; ++k) v[k] = 0.f;
        el = eh = 0.f;
    }
};

// A row in flight: the raw main dwords and the edge dword, converted by st_cvt where the
// row is first used (one trip after its loads were issued: the loads of trip k + 1 fly
// while trip k computes).
template <typename T, int CPL>
struct StRaw {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    static constexpr int NB = (int)sizeof(T) * CPL;
    typedef std::conditional_t<NB == 4, unsigned, std::conditional_t<NB == 8, u2, u4>> M;
    M m;
    unsigned e;
};
template <typename T, int CPL>
__device__ __forceinline__ void st_issue(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned eoff,
                                         unsigned soff, StRaw<T, CPL>& R) {
    constexpr int NB = StRaw<T, CPL>::NB;
    if constexpr (NB == 4) R.m = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
    else if constexpr (NB == 8) R.m = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    else R.m = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
    R.e = __builtin_amdgcn_raw_buffer_load_b32(rs, eoff, soff, 0);
}
// (whole-vector bit_casts: see st_load)
template <typename T, int CPL>
__device__ __forceinline__ void st_cvt(const StRaw<T, CPL>& R, bool zero, StRow<CPL>& out) {
    if constexpr (sizeof(T) == 2) {
        typedef T tv __attribute__((ext_vector_type(CPL)));
        const tv e = __builtin_bit_cast(tv, R.m);
#pragma unroll
        for (int k = 0; k < CPL; ++k) out.v[k] = (float)e[k];
        out.el = (float)__builtin_bit_cast(T, (unsigned short)(R.e & 0xffffu));
        out.eh = (float)__builtin_bit_cast(T, (unsigned short)(R.e >> 16));
    } else {
        typedef float fv __attribute__((ext_vector_type(CPL)));
        const fv e = __builtin_bit_cast(fv, R.m);
#pragma unroll
        for (int k = 0; k < CPL; ++k) out.v[k] = e[k];
        out.el = out.eh = __builtin_bit_cast(float, R.e);
    }
    if (zero) out.zero();                               // uniform
}

struct WaveUnit {
    int64_t plane;
    int win, s0, s1;
    bool live;
};

__device__ __forceinline__ WaveUnit st_unit(const StreamGeom& S, int nrows) {
    WaveUnit u;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (S.nwin + 3) / 4;
    const int grp = (int)(blk % ngrp);
    const int64_t rest = blk / ngrp;
    const int band = (int)(rest % S.nband);
    u.plane = rest / S.nband;
    u.win = grp * 4 + wslot;
    u.s0 = band * S.rb;
    u.s1 = min(u.s0 + S.rb, nrows);
    u.live = u.plane < S.planes && u.win < S.nwin;
    return u;
}

// ---------------------------------------------------------------------------
// rect -> hex, bilinear (geometry_np.py:358-519)
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout, int CPL = st_cpl<Tin, Tout>()>
__global__ __launch_bounds__(ST_THREADS) void k_r2h_stream(const Tin* __restrict__ x,
                                                           Tout* __restrict__ y, StreamGeom S) {
    const WaveUnit u = st_unit(S, S.h1);
    if (!u.live) return;                          // wave-uniform; no barriers below
    const int lane = threadIdx.x & 63;
    constexpr int ST_COLS = 64 * CPL;             // window columns
    using StRow = hg::StRow<CPL>;
    const int W0 = u.win * ST_COLS;
    const int ce = W0 + CPL * lane;               // this lane's first column

    // per-row records, row s0 + 64 k + lane (fp64 lattice, geometry_np.py:440-449)
    int rin[2];
    float rc0[2], rc1[2];
    unsigned rval[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int r = u.s0 + 64 * k + lane;
        rin[k] = 0; rc0[k] = 0.f; rc1[k] = 0.f; rval[k] = 0;
        if (r < S.h1) {
            const double i_ = axis_at(S.rxs, r) + (double)(S.h - 1) * 0.5;
            const int in = (int)i_;
            const double fi = i_ - (double)(float)in;
            rin[k] = in;
            rc0[k] = (float)fi;                   // weight of row in+1 (:515 c0 = fi)
            rc1[k] = (float)(1.0 - fi);           // weight of row in
            rval[k] = (in >= 0 && in < S.h ? 1u : 0u) | (in + 1 >= 0 && in + 1 < S.h ? 2u : 0u);
        }
    }
    // per-column records (constant over rows): jn - q in {-1, 0}, fj, 1 - fj
    // (a column with no tap inside the raster, e.g. q = w1 - 1 where jn = w, is "dead":
    // both taps read 0 as in the general kernel)
    float fj[CPL], gj[CPL];
    bool left[CPL], dead[CPL];                        // jn == q - 1; no live tap
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int q = ce + k;
        fj[k] = 0.f; gj[k] = 0.f; left[k] = false; dead[k] = true;
        if (q < S.w1) {
            const double j_ = axis_at(S.rys, q) + (double)(S.w - 1) * 0.5;
            const int jn = (int)j_;
            const double jf = j_ - (double)(float)jn;
            fj[k] = (float)jf;
            gj[k] = (float)(1.0 - jf);
            left[k] = jn < q;
            dead[k] = !((jn >= 0 && jn < S.w) || (jn + 1 >= 0 && jn + 1 < S.w));
        }
    }

    const int64_t ipl = (int64_t)S.h * S.w, opl = (int64_t)S.h1 * S.w1;
    const __amdgpu_buffer_rsrc_t xrs = st_rsrc(x + u.plane * ipl, ipl * (int64_t)sizeof(Tin));
    const __amdgpu_buffer_rsrc_t yrs = st_rsrc(y + u.plane * opl, opl * (int64_t)sizeof(Tout));
    // lanes whose columns are outside the raster read zeros (w % CPL == 0: all or none)
    const unsigned xoff = ce < S.w ? (unsigned)ce * (unsigned)sizeof(Tin) : ST_OOB;
    const unsigned yoff = ce < S.w1 ? (unsigned)ce * (unsigned)sizeof(Tout) : ST_OOB;
    // edge dword: lane 0 -> column W0-1 (16-bit: dword W0-2..W0-1, hi half), lane 63 ->
    // column W0+64*CPL (lo half); zero outside the raster, no access for other lanes
    constexpr int EB = sizeof(Tin) == 2 ? 2 : 1;
    unsigned eoff = ST_OOB;
    if (lane == 0 && W0 > 0) eoff = (unsigned)(W0 - EB) * (unsigned)sizeof(Tin);
    if (lane == 63 && W0 + ST_COLS < S.w) eoff = (unsigned)(W0 + ST_COLS) * (unsigned)sizeof(Tin);
    const unsigned xrow = (unsigned)S.w * (unsigned)sizeof(Tin);
    const unsigned yrow = (unsigned)S.w1 * (unsigned)sizeof(Tout);

    // Register ring of source rows: every row is loaded once (one main + one edge load);
    // rows outside the raster read as zeros (:478-486), so the taps of a row with
    // in(r) - r in {-1, 0} need no further masking.
    auto load_row = [&](int rr, StRow& R) {
        const unsigned so = (unsigned)min(max(rr, 0), S.h - 1) * xrow;
        st_load<Tin, CPL>(xrs, xoff, so, R.v);
        st_load_edge<Tin>(xrs, eoff, so, &R.el, &R.eh);
        if (rr < 0 || rr >= S.h) R.zero();            // uniform
    };
    // output row r from source rows r-1, r, r+1
    auto row = [&](int r, const StRow& Rm, const StRow& Rc, const StRow& Rp) {
        if (r >= u.s1) return;                        // uniform (last trip of a band)
        const int e = r - u.s0, k = e >> 6, l = e & 63;
        const int in = __builtin_amdgcn_readlane(k ? rin[1] : rin[0], l);
        const float c0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
            __builtin_bit_cast(int, k ? rc0[1] : rc0[0]), l));
        const float c1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
            __builtin_bit_cast(int, k ? rc1[1] : rc1[0]), l));
        const unsigned val = (unsigned)__builtin_amdgcn_readlane((int)(k ? rval[1] : rval[0]), l);
        const bool up = in != r;                      // in == r - 1 (else in == r)
        StRow A = up ? Rm : Rc, B = up ? Rc : Rp;     // rows in, in + 1
        if (!(val & 1u)) A.zero();                    // a dead row (no live tap): all zero
        if (!(val & 2u)) B.zero();
        // vertical blend per column, t = c0 * P(in+1) + c1 * P(in)   (:515-516)
        float t[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) t[c] = c0 * B.v[c] + c1 * A.v[c];
        const float tl = c0 * B.eh + c1 * A.eh;       // column W0-1 (meaningful on lane 0)
        const float tr = c0 * B.el + c1 * A.el;       // column W0+64*CPL (lane 63)
        const float tm = st_prev(t[CPL - 1], tl);           // column ce - 1
        const float tp = st_next(t[0], tr);           // column ce + CPL
        float o[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const float tc_m = c == 0 ? tm : t[c - 1];
            const float tc_p = c == CPL - 1 ? tp : t[c + 1];
            const float t1 = dead[c] ? 0.f : (left[c] ? tc_m : t[c]);   // column jn
            const float t2 = dead[c] ? 0.f : (left[c] ? t[c] : tc_p);   // column jn + 1
            o[c] = fj[c] * t2 + gj[c] * t1;           // :517
        }
        st_store<Tout, CPL>(o, yrs, yoff, (unsigned)r * yrow);
    };
    // four output rows per trip: four new source rows (r0+1 .. r0+4) issue together;
    // readlane is convergent, so the compiler would not unroll this loop by itself
    StRow P0, P1;
    load_row(u.s0 - 1, P0);
    load_row(u.s0, P1);
    // rows r0+1 .. r0+4 of the next trip are issued before this trip's rows are computed
    // (4K bf16 b128: 2.50 -> 2.39 ms, tools/ab_ops.py)
    StRaw<Tin, CPL> Q[4];
    auto issue4 = [&](int r1) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st_issue<Tin, CPL>(xrs, xoff, eoff, (unsigned)min(max(r1 + k, 0), S.h - 1) * xrow, Q[k]);
    };
    issue4(u.s0 + 1);
    for (int r0 = u.s0; r0 < u.s1; r0 += 4) {
        StRow N0, N1, N2, N3;
        st_cvt<Tin, CPL>(Q[0], r0 + 1 >= S.h, N0);
        st_cvt<Tin, CPL>(Q[1], r0 + 2 >= S.h, N1);
        st_cvt<Tin, CPL>(Q[2], r0 + 3 >= S.h, N2);
        st_cvt<Tin, CPL>(Q[3], r0 + 4 >= S.h, N3);
        if (r0 + 4 < u.s1) issue4(r0 + 5);            // uniform
        row(r0, P0, P1, N0);
        row(r0 + 1, P1, N0, N1);
        row(r0 + 2, N0, N1, N2);
        row(r0 + 3, N1, N2, N3);
        P0 = N2;
        P1 = N3;
    }
}

// ---------------------------------------------------------------------------
// hex -> rect, linear, same size (geometry_np.py:191-356)
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout, int CPL = st_cpl<Tin, Tout>()>
__global__ __launch_bounds__(ST_THREADS) void k_h2r_stream(const Tin* __restrict__ x,
                                                           Tout* __restrict__ y, StreamGeom S) {
    const WaveUnit u = st_unit(S, S.h1);
    if (!u.live) return;
    const int lane = threadIdx.x & 63;
    constexpr int ST_COLS = 64 * CPL;             // window columns
    using StRow = hg::StRow<CPL>;
    const int W0 = u.win * ST_COLS;
    const int ce = W0 + CPL * lane;
    const int64_t pl = (int64_t)S.h * S.w;        // h1 == h, w1 == w
    const __amdgpu_buffer_rsrc_t xrs = st_rsrc(x + u.plane * pl, pl * (int64_t)sizeof(Tin));
    const __amdgpu_buffer_rsrc_t yrs = st_rsrc(y + u.plane * pl, pl * (int64_t)sizeof(Tout));
    const unsigned xoff = ce < S.w ? (unsigned)ce * (unsigned)sizeof(Tin) : ST_OOB;
    const unsigned yoff = ce < S.w ? (unsigned)ce * (unsigned)sizeof(Tout) : ST_OOB;
    constexpr int EB = sizeof(Tin) == 2 ? 2 : 1;
    unsigned eoff = ST_OOB;
    if (lane == 0 && W0 > 0) eoff = (unsigned)(W0 - EB) * (unsigned)sizeof(Tin);
    if (lane == 63 && W0 + ST_COLS < S.w) eoff = (unsigned)(W0 + ST_COLS) * (unsigned)sizeof(Tin);
    const unsigned xrow = (unsigned)S.w * (unsigned)sizeof(Tin);
    const unsigned yrow = (unsigned)S.w * (unsigned)sizeof(Tout);

    auto load_row = [&](int rr, StRow& R) {       // ring row; zeros outside the raster
        const unsigned so = (unsigned)min(rr, S.h - 1) * xrow;
        st_load<Tin, CPL>(xrs, xoff, so, R.v);
        st_load_edge<Tin>(xrs, eoff, so, &R.el, &R.eh);
        if (rr >= S.h) R.zero();                      // uniform
    };
    // output row a from hex rows a (Z) and a + 1 (N; zero below the raster, :303-323)
    auto row = [&](int a, auto ODDc, const StRow& Z, const StRow& N) {
        constexpr bool odd = decltype(ODDc)::value;
        if (a >= u.s1) return;                        // uniform (last trip of a band)
        const float al = S.tri[odd][0], be = S.tri[odd][1], ga = S.tri[odd][2];
        float o[CPL];
        if constexpr (!odd) {                         // p1 = (a, b), p2 = (a, b+1)
            const float zp = st_next(Z.v[0], Z.el);   // column ce + CPL
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float p2 = c == CPL - 1 ? zp : Z.v[c + 1];
                o[c] = al * Z.v[c] + be * p2 + ga * N.v[c];   // :354
            }
        } else {                                      // p1 = (a, b-1), p2 = (a, b)
            const float zm = st_prev(Z.v[CPL - 1], Z.eh);   // column ce - 1
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const float p1 = c == 0 ? zm : Z.v[c - 1];
                o[c] = al * p1 + be * Z.v[c] + ga * N.v[c];
            }
        }
        st_store<Tout, CPL>(o, yrs, yoff, (unsigned)a * yrow);
    };
    // bands start on even rows (S.rb is even): four rows per trip, parity static,
    // every hex row loaded once
    // (issuing the next trip's rows first, as k_r2h_stream does, measured 1.5 % slower here)
    StRow P;
    load_row(u.s0, P);
    for (int a = u.s0; a < u.s1; a += 4) {
        StRow N0, N1, N2, N3;
        load_row(a + 1, N0);
        load_row(a + 2, N1);
        load_row(a + 3, N2);
        load_row(a + 4, N3);
        row(a, std::false_type{}, P, N0);
        row(a + 1, std::true_type{}, N0, N1);
        row(a + 2, std::false_type{}, N1, N2);
        row(a + 3, std::true_type{}, N2, N3);
        P = N3;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout>
static int stream_launch(int op, const void* src, void* dst, const StreamGeom& S, hipStream_t st) {
    const int64_t blocks = S.planes * (int64_t)S.nband * ((S.nwin + 3) / 4);
    if (blocks > INT_MAX) return HG_EUNSUP;
    if (blocks == 0) return HG_OK;
    if (op == HG_OP_RECT_TO_HEX)
        hipLaunchKernelGGL((k_r2h_stream<Tin, Tout>), dim3((unsigned)blocks), dim3(ST_THREADS), 0, st,
                           (const Tin*)src, (Tout*)dst, S);
    else
        hipLaunchKernelGGL((k_h2r_stream<Tin, Tout>), dim3((unsigned)blocks), dim3(ST_THREADS), 0, st,
                           (const Tin*)src, (Tout*)dst, S);
    return launch_status();
}

// r2h rows / columns: every live tap within one row / column below the sample's
// own index (the structure k_r2h_stream assumes), proven on the fp64 lattice.
static bool r2h_near_identity(const Geom& g) {
    for (int64_t q = 0; q < g.w1; ++q) {
        const double j_ = axis_at(g.ys, q) + (double)(g.w - 1) * 0.5;
        const int64_t jn = (int64_t)j_;
        const bool live = (jn >= 0 && jn < g.w) || (jn + 1 >= 0 && jn + 1 < g.w);
        if (live && (jn - q < -1 || jn - q > 0)) return false;
    }
    for (int64_t r = 0; r < g.h1; ++r) {
        const double i_ = axis_at(g.xs, r) + (double)(g.h - 1) * 0.5;
        const int64_t in = (int64_t)i_;
        const bool live = (in >= 0 && in < g.h) || (in + 1 >= 0 && in + 1 < g.h);
        if (live && (in - r < -1 || in - r > 0)) return false;
    }
    return true;
}

// same-size h2r: the triangle of every even (odd) output row is the one of row 0 (1);
// checked on the lattice for both parities at an interior and both border columns
static bool h2r_exact(const Geom& g, float tri[2][3]) {
    if (g.h1 != g.h || g.w1 != g.w || g.h < 2 || g.w < 2) return false;
    for (int par = 0; par < 2; ++par) {
        const int64_t cols[3] = {0, 1, g.w - 1};
        for (int i = 0; i < 3; ++i) {
            const int64_t b = cols[i];
            for (int64_t a = par; a < g.h && a < par + 4; a += 2) {
                const TriSample s = tri_sample(g, a, b);
                const int64_t c1 = par ? b - 1 : b, c2 = par ? b : b + 1;
                if (s.i_n != a || s.r[0] != a || s.c[0] != c1 || s.r[1] != a || s.c[1] != c2 ||
                    s.r[2] != a + 1 || s.c[2] != b)
                    return false;
                const float t[3] = {(float)s.alpha, (float)s.beta, (float)s.gamma};
                if (i == 0 && a == par) {
                    tri[par][0] = t[0]; tri[par][1] = t[1]; tri[par][2] = t[2];
                } else if (t[0] != tri[par][0] || t[1] != tri[par][1] || t[2] != tri[par][2]) {
                    return false;
                }
            }
        }
    }
    return true;
}

int stream_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
               int64_t w, int64_t h1, int64_t w1, hipStream_t st, bool dry) {
    if (env_is("HYGRID_STREAM", "0")) return HG_EUNSUP;   // A/B switch: general kernels only
    if (op != HG_OP_RECT_TO_HEX && op != HG_OP_HEX_TO_RECT) return HG_EUNSUP;
    auto small = [](int dt) { return dt == HG_BF16 || dt == HG_F16 || dt == HG_F32; };
    if (!small(sdt) || !small(ddt)) return HG_EUNSUP;   // f32 accumulator types only
    if (planes <= 0 || h < 2 || w < 4 || h1 < 1 || w1 < 4) return HG_EUNSUP;
    const int cpl = (sdt == HG_F32 || ddt == HG_F32) ? 2 : 4;   // = st_cpl<Tin, Tout>()
    if ((w % cpl) || (w1 % cpl)) return HG_EUNSUP;       // a lane's columns: all in or out
    if (h * w * 4 >= ((int64_t)1 << 31) || h1 * w1 * 4 >= ((int64_t)1 << 31)) return HG_EUNSUP;
    StreamGeom S = {};
    S.planes = planes;
    S.h = (int)h; S.w = (int)w; S.h1 = (int)h1; S.w1 = (int)w1;
    if (op == HG_OP_RECT_TO_HEX) {
        const Geom g = make_r2h(h, w, h1, w1);
        if (!r2h_near_identity(g)) return HG_EUNSUP;
        S.rxs = g.xs;
        S.rys = g.ys;
    } else {
        const Geom g = make_tri(h, w, h1, w1, 0.75);
        if (!h2r_exact(g, S.tri)) return HG_EUNSUP;
    }
    S.nwin = (int)((w1 + 64 * cpl - 1) / (64 * cpl));
    S.rb = op == HG_OP_RECT_TO_HEX ? ST_RB_R2H : ST_RB_H2R;
    S.nband = (int)((h1 + S.rb - 1) / S.rb);
    if (dry) return HG_OK;
    if (sdt == HG_BF16 && ddt == HG_BF16) return stream_launch<__bf16, __bf16>(op, src, dst, S, st);
    if (sdt == HG_F16 && ddt == HG_F16) return stream_launch<_Float16, _Float16>(op, src, dst, S, st);
    if (sdt == HG_F32 && ddt == HG_F32) return stream_launch<float, float>(op, src, dst, S, st);
    if (sdt == HG_BF16 && ddt == HG_F32) return stream_launch<__bf16, float>(op, src, dst, S, st);
    if (sdt == HG_F16 && ddt == HG_F32) return stream_launch<_Float16, float>(op, src, dst, S, st);
    if (sdt == HG_F32 && ddt == HG_BF16) return stream_launch<float, __bf16>(op, src, dst, S, st);
    if (sdt == HG_F32 && ddt == HG_F16) return stream_launch<float, _Float16>(op, src, dst, S, st);
    return HG_EUNSUP;
}

}  // namespace hg
