// resample_down.hip — row-streaming rect->hex resampler for the ~2x downsampling lattices of
// the reference's own entry points:
//   * IMAGE.ConvertToHexagon (Image.py:111-116): rect_to_hex_resample(image, (h//2, w//2),
//     'nearest') on the image's own dtype (u8 from GDAL);
//   * the geometry_np demo (geometry_np.py:772-776): rect_to_hex_resample(image, (256, 341),
//     'bilinear') on an ADE image, ratio ~2.
// Tried by hg_rect_to_hex after the near-identity streaming kernels; HG_EUNSUP (nothing
// launched) outside its domain, which the host checks exactly on the lattice (O(h1 + w1)).
//
// The r2h lattice is separable (geometry_np.py:415-448): row a of the output reads source
// rows i_n(a), i_n(a) + 1 with weights (1 - i_f, i_f), column b reads source columns j_n(b),
// j_n(b) + 1 with (1 - j_f, j_f).  'nearest' picks the tap of the smallest
// (x_ - p_x)^2 + (y_ - p_y)^2 (:499-506); that distance compares the centred coordinate x_
// with the uncentred index p_x, so for h, w >= 2 the first tap (i_n, j_n) always wins — the
// host proves it per row and per column (fp64 squares, monotone rounding), and the kernel
// copies tap 1 (or 0 outside the raster, :465-486).
//
// Execution model.  A wavefront owns a window of 64 * K output columns (lane l <-> columns
// b0 = W0 + K l .. b0 + K - 1, K = 4 / sizeof(Tin): one dword of input elements) of one plane
// and walks a band of DN_RB output rows.  For a ~2x column ratio every tap column of the
// lane's K outputs lies in the 16 source bytes [2 b0 E - 4, 2 b0 E + 12) (clamped into the
// row at the raster's edges; host-checked), so per source row the lane issues one 16-byte
// load and assembles each output's taps with two v_perm_b32 byte selects + an OR (selectors
// fixed per lane for the whole band: the column lattice does not depend on the row; a tap
// outside the raster selects the constant zero byte).  Source rows are per output row and
// uniform: a per-wave LDS row table holds their byte offsets (out of the buffer range for rows outside the raster, so the load returns
// zeros, as the reference's masked gather) and the fp32 row weights.  Rows are loaded DN_PD
// steps ahead into a register ring; every referenced source row is read once (nearest reads
// only the rows its lattice references: half of them at a 2x ratio).
//
// Bilinear arithmetic is the general kernel's blend (resample.hip, geometry_np.py:514-517):
// t1 = i_f p3 + (1 - i_f) p1, t2 = i_f p4 + (1 - i_f) p2, out = j_f t2 + (1 - j_f) t1 in
// fp32 without contraction, so the outputs are bit-identical to k_resample_lds.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "common.h"
#include "lattice.h"
#include "stream.h"

namespace hg {

constexpr int DN_THREADS = 256;   // 4 independent waves: 4 adjacent windows of one band
constexpr int DN_RB = 32;         // output rows per band
constexpr int DN_PD = 4;          // output rows whose source rows are in flight

struct DownGeom {
    int64_t planes;
    int h, w, h1, w1;
    int nwin, nband;
    Axis xs, ys;
};

template <typename T> struct DnUnpack;
template <> struct DnUnpack<__bf16> {
    static __device__ __forceinline__ float lo(unsigned d) { return __builtin_bit_cast(float, d << 16); }
    static __device__ __forceinline__ float hi(unsigned d) { return __builtin_bit_cast(float, d & 0xffff0000u); }
};
template <> struct DnUnpack<_Float16> {
    static __device__ __forceinline__ float lo(unsigned d) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(d & 0xffffu));
    }
    static __device__ __forceinline__ float hi(unsigned d) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(d >> 16));
    }
};

typedef unsigned dn_u4 __attribute__((ext_vector_type(4)));

// first byte of a lane's 16-byte source chunk: 4 bytes left of its first tap column's
// nominal 2 b0, clamped into the row (host and kernel share this definition)
__host__ __device__ constexpr int dn_chunk(int b0, int E, int w) {
    return (2 * b0 * E - 4 < 0 ? 0 : (2 * b0 * E - 4 > w * E - 16 ? w * E - 16 : 2 * b0 * E - 4));
}
template <int B, int E, typename F>
__device__ __forceinline__ void dn_sfor(F&& f) {   // f(IC<B>), ..., f(IC<E-1>)
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        dn_sfor<B + 1, E>(f);
    }
}

template <typename Tin, typename Tout, bool NEAR>
__global__ __launch_bounds__(DN_THREADS) void k_r2h_down(const Tin* __restrict__ x,
                                                         Tout* __restrict__ y, DownGeom D) {
    constexpr int E = (int)sizeof(Tin);   // 1 or 2 bytes per source element
    constexpr int K = 4 / E;              // output columns per lane
    constexpr int NT = NEAR ? 1 : 2;      // source rows per output row
    constexpr int NO = NEAR ? 1 : K;      // assembled dwords per source row (nearest: the
                                          // K outputs; bilinear: one (tap0, tap1) pair per output)
    constexpr int GW = DN_THREADS / 64;
    constexpr int NL = DN_RB + DN_PD;     // row-table entries (the band + the look-ahead)
    static_assert(NEAR || E == 2, "bilinear: 16-bit float inputs");
    // per-wave row table: {offset of source row i_n, of i_n + 1, bits of (float)i_f,
    // bits of (float)(1 - i_f)}
    __shared__ int4 lut_all[GW][NL];

    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int4* lut = lut_all[wslot];
    const int64_t blk = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x);
    const int ngrp = (D.nwin + GW - 1) / GW;
    const int grp = (int)(blk % ngrp);
    const int64_t rest = blk / ngrp;
    const int band = (int)(rest % D.nband);
    const int64_t p = rest / D.nband;
    if (p >= D.planes) return;                      // uniform per workgroup
    const int win = grp * GW + wslot;
    const int b0 = (win * 64 + lane) * K;           // first output column of this lane
    const int s0 = band * DN_RB;
    const int s1 = min(s0 + DN_RB, D.h1);
    const unsigned OOB = 0x80000000u;               // past the buffer range: loads read 0

    // ---- row table (fp64 lattice, geometry_np.py:440-448) -----------------------------
    const unsigned xrow = (unsigned)D.w * (unsigned)E;
    for (int e = lane; e < NL; e += 64) {
        const int a = s0 + e;
        int4 t = {(int)OOB, (int)OOB, 0, 0};
        if (a < s1) {                               // rows past the band are never loaded
            const double i_ = axis_at(D.xs, a) + (double)(D.h - 1) * 0.5;
            const int in = (int)i_;
            const double f = i_ - (double)(float)in;
            if (in >= 0 && in < D.h) t.x = (int)((unsigned)in * xrow);
            if (in + 1 >= 0 && in + 1 < D.h) t.y = (int)((unsigned)(in + 1) * xrow);
            t.z = __builtin_bit_cast(int, (float)f);
            t.w = __builtin_bit_cast(int, (float)(1.0 - f));
        }
        lut[e] = t;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);             // lgkmcnt(0): own-wave LDS writes
    __builtin_amdgcn_wave_barrier();

    // ---- per-lane column lattice: byte selectors and column weights --------------------
    // chunk byte c of a source row <-> source byte cs + c (cs clamped into the row, so the
    // 16-byte load never leaves the row); dwords D0..D3.
    // out dword n = perm(D1, D0, s01[n]) | perm(D3, D2, s23[n]) (0x0c = constant zero byte)
    unsigned s01[NO], s23[NO];
    float fj[K], gj[K];
    for (int n = 0; n < NO; ++n) { s01[n] = 0x0c0c0c0cu; s23[n] = 0x0c0c0c0cu; }
    for (int k = 0; k < K; ++k) { fj[k] = 0.f; gj[k] = 0.f; }
    const bool own = b0 < D.w1;
    // a ragged width (w1 % K != 0) leaves one partial lane per row: it stores element-wise
    const int nown = min(K, D.w1 - b0);
    const bool ragged = __builtin_amdgcn_ballot_w64(own && nown < K) != 0;   // uniform
    const int cs = dn_chunk(b0, E, D.w);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int b = b0 + k;
        if (b >= D.w1) continue;
        const double j_ = axis_at(D.ys, b) + (double)(D.w - 1) * 0.5;
        const int jn = (int)j_;
        const double jf = j_ - (double)(float)jn;
        fj[k] = (float)jf;
        gj[k] = (float)(1.0 - jf);
#pragma unroll
        for (int t = 0; t < (NEAR ? 1 : 2); ++t) {
            const int col = jn + t;
            if (col < 0 || col >= D.w) continue;    // outside the raster: zero bytes
            const int q = col * E - cs;             // chunk byte of the element (host: 0..16-E)
#pragma unroll
            for (int eb = 0; eb < E; ++eb) {
                // result byte: nearest -> output k's byte eb; bilinear -> pair dword k, tap t
                const int n = NEAR ? 0 : k;
                const int rb = NEAR ? k * E + eb : t * E + eb;
                const int c = q + eb;
                const unsigned m = ~(0xffu << (8 * rb));
                if (c < 8) s01[n] = (s01[n] & m) | ((unsigned)c << (8 * rb));
                else s23[n] = (s23[n] & m) | ((unsigned)(c - 8) << (8 * rb));
            }
        }
    }

    // ---- buffers -----------------------------------------------------------------------
    const int64_t ipl = (int64_t)D.h * D.w, opl = (int64_t)D.h1 * D.w1;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + p * ipl), (short)0, (int)(ipl * E), 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + p * opl), (short)0, (int)(opl * (int64_t)sizeof(Tout)), 0x00020000);
    const unsigned xoff = (unsigned)cs;
    const unsigned yrow = (unsigned)D.w1 * (unsigned)sizeof(Tout);
    const unsigned yoff = own ? (unsigned)b0 * (unsigned)sizeof(Tout) : OOB;

    dn_u4 ring[DN_PD + 1][NT];
    auto issue = [&](auto SLc, int i) {             // source rows of band row i -> slot SL
        constexpr int SL = decltype(SLc)::value;
        const int4 t = lut[i];
        // a row offset out of range makes the whole address out of range (the lane offset
        // is < 2^20 and the planes are < 2^31 - 2^20 bytes, host-checked)
        ring[SL][0] = __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff + (unsigned)t.x, 0, 0);
        if constexpr (!NEAR)
            ring[SL][1] = __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff + (unsigned)t.y, 0, 0);
    };
    auto pick = [&](const dn_u4& d, int n) -> unsigned {
        return __builtin_amdgcn_perm(d.y, d.x, s01[n]) | __builtin_amdgcn_perm(d.w, d.z, s23[n]);
    };
    auto out_row = [&](auto SLc, int i) {           // band row i from slot SL
        constexpr int SL = decltype(SLc)::value;
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(s0 + i) * yrow));
        if constexpr (NEAR) {
            const unsigned v = pick(ring[SL][0], 0);
            if (!ragged || nown == K) {
                __builtin_amdgcn_raw_buffer_store_b32(v, yrs, yoff, so, 0);
            } else if (own) {
#pragma unroll
                for (int k = 0; k < K - 1; ++k) {
                    if (k >= nown) break;
                    if constexpr (E == 1)
                        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(v >> (8 * k)), yrs,
                                                             yoff + k, so, 0);
                    else
                        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(v >> (16 * k)), yrs,
                                                              yoff + 2 * k, so, 0);
                }
            }
        } else {
            const int4 t = lut[i];
            const float c0 = __builtin_bit_cast(float, t.z), c1 = __builtin_bit_cast(float, t.w);
            float o[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const unsigned r0 = pick(ring[SL][0], k), r1 = pick(ring[SL][1], k);
                const float v0 = DnUnpack<Tin>::lo(r0), v1 = DnUnpack<Tin>::hi(r0);   // p1, p2
                const float v2 = DnUnpack<Tin>::lo(r1), v3 = DnUnpack<Tin>::hi(r1);   // p3, p4
                const float t1 = c0 * v2 + c1 * v0;     // geometry_np.py:515
                const float t2 = c0 * v3 + c1 * v1;     // :516
                o[k] = fj[k] * t2 + gj[k] * t1;         // :517
            }
            if (ragged && own && nown < K) {   // K = 2: the lane's first output only
                if constexpr (sizeof(Tout) == 2)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (Tout)o[0]),
                                                          yrs, yoff, so, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[0]), yrs,
                                                          yoff, so, 0);
            } else if constexpr (sizeof(Tout) == 2) {
                typedef Tout t2v __attribute__((ext_vector_type(2)));
                const t2v pk = {(Tout)o[0], (Tout)o[1]};
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, pk), yrs, yoff, so, 0);
            } else {
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(
                    u2v{__builtin_bit_cast(unsigned, o[0]), __builtin_bit_cast(unsigned, o[1])},
                    yrs, yoff, so, 0);
            }
        }
    };

    // ---- the band: DN_PD rows in flight, fully unrolled (constant ring slots) ----------
    issue(std::integral_constant<int, 0>{}, 0);
    issue(std::integral_constant<int, 1>{}, 1);
    issue(std::integral_constant<int, 2>{}, 2);
    issue(std::integral_constant<int, 3>{}, 3);
    static_assert(DN_PD == 4, "prologue issues DN_PD rows");
    auto step = [&](auto Ic) {
        constexpr int I = decltype(Ic)::value;
        issue(std::integral_constant<int, (I + DN_PD) % (DN_PD + 1)>{}, I + DN_PD);
        if (s0 + I < s1) out_row(std::integral_constant<int, I % (DN_PD + 1)>{}, I);
    };
    dn_sfor<0, DN_RB>(step);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Every valid tap column of every lane inside the lane's 16-byte chunk; nearest: tap 1 is
// the argmin of every sample (|x_ - i_n| <= |x_ - i_n - 1| per row, the same per column:
// then d1 <= d2, d3, d4 under monotone fp64 rounding, and argmin takes the first minimum).
static bool down_lattice_ok(const Geom& g, int E, bool near) {
    const int K = 4 / E;
    for (int64_t b = 0; b < g.w1; ++b) {
        const double y_ = axis_at(g.ys, b);
        const double j_ = y_ + (double)(g.w - 1) * 0.5;
        const int64_t jn = (int64_t)j_;
        const int64_t b0 = b - b % K;
        const int64_t cs = dn_chunk((int)b0, E, (int)g.w);
        for (int t = 0; t < (near ? 1 : 2); ++t) {
            const int64_t col = jn + t;
            if (col < 0 || col >= g.w) continue;
            const int64_t q = col * E - cs;
            if (q < 0 || q + E > 16) return false;
        }
        if (near) {
            const double d0 = y_ - (double)jn, d1 = y_ - (double)(jn + 1);
            if (!(d0 * d0 <= d1 * d1)) return false;
        }
    }
    if (near) {
        for (int64_t a = 0; a < g.h1; ++a) {
            const double x_ = axis_at(g.xs, a);
            const int64_t in = (int64_t)(x_ + (double)(g.h - 1) * 0.5);
            const double d0 = x_ - (double)in, d1 = x_ - (double)(in + 1);
            if (!(d0 * d0 <= d1 * d1)) return false;
        }
    }
    return true;
}

template <typename Tin, typename Tout, bool NEAR>
static int down_launch(const void* src, void* dst, const DownGeom& D, hipStream_t st) {
    const int64_t blocks = D.planes * (int64_t)D.nband * ((D.nwin + 3) / 4);
    if (blocks > INT_MAX) return HG_ESHAPE;
    hipLaunchKernelGGL((k_r2h_down<Tin, Tout, NEAR>), dim3((unsigned)blocks), dim3(DN_THREADS), 0,
                       st, (const Tin*)src, (Tout*)dst, D);
    return launch_status();
}

int down_try(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h, int64_t w,
             int64_t h1, int64_t w1, int interp, hipStream_t st, bool dry) {
    if (env_is("HYGRID_DOWN", "0")) return HG_EUNSUP;   // A/B switch: general kernels only
    const bool near = interp == HG_NEAREST;
    int E;
    if (near) {
        if (sdt != ddt) return HG_EUNSUP;
        E = dtype_size(sdt);
        if (E != 1 && E != 2) return HG_EUNSUP;
    } else {
        if (sdt != HG_BF16 && sdt != HG_F16) return HG_EUNSUP;
        if (ddt != HG_BF16 && ddt != HG_F16 && ddt != HG_F32) return HG_EUNSUP;
        E = 2;
    }
    const int K = 4 / E;
    const int osz = near ? E : dtype_size(ddt);
    if (planes < 1 || h < 2 || w < 2 || h1 < 1 || w1 < 1) return HG_EUNSUP;
    // chunks inside the row; rows of a byte length that is not a multiple of 4 start at
    // unaligned addresses (gfx9 runs its buffer loads in unaligned-access mode; the parity
    // tests cover odd widths)
    if (w * E < 16 || w * E > (1 << 19)) return HG_EUNSUP;
    if (h * w * E >= ((int64_t)1 << 31) - ((int64_t)1 << 20) ||
        h1 * w1 * osz >= ((int64_t)1 << 31) - ((int64_t)1 << 20))
        return HG_EUNSUP;
    const Geom g = make_r2h(h, w, h1, w1);
    if (!down_lattice_ok(g, E, near)) return HG_EUNSUP;
    DownGeom D;
    D.planes = planes;
    D.h = (int)h; D.w = (int)w; D.h1 = (int)h1; D.w1 = (int)w1;
    D.xs = g.xs;
    D.ys = g.ys;
    D.nwin = (int)((w1 + 64 * K - 1) / (64 * K));
    D.nband = (int)((h1 + DN_RB - 1) / DN_RB);
    if (dry) return HG_OK;
    if (near) {
        if (E == 1) return down_launch<uint8_t, uint8_t, true>(src, dst, D, st);
        return down_launch<uint16_t, uint16_t, true>(src, dst, D, st);
    }
    if (sdt == HG_BF16) {
        if (ddt == HG_BF16) return down_launch<__bf16, __bf16, false>(src, dst, D, st);
        if (ddt == HG_F16) return down_launch<__bf16, _Float16, false>(src, dst, D, st);
        return down_launch<__bf16, float, false>(src, dst, D, st);
    }
    if (ddt == HG_BF16) return down_launch<_Float16, __bf16, false>(src, dst, D, st);
    if (ddt == HG_F16) return down_launch<_Float16, _Float16, false>(src, dst, D, st);
    return down_launch<_Float16, float, false>(src, dst, D, st);
}

}  // namespace hg
