// pyramid_fused.hip — one hex-pyramid level (BASELINE config 5) on the streaming fused
// kernel (fused_kernel.h, MD 3 from the rect image, MD 4 from a hex image):
//     Z = hexresize(HexConv2d_depthwise(X), (h2, w2))      for a 2x downsample
// The reference chains HexConv2d(C, C, off, 2, padding=1, groups=C) (HexFrames.py:96-169)
// and hexresize (geometry_np.py:520-681, 'linear'), after rect_to_hex (geometry_np.py:
// 358-519, bilinear, same size) for the first level.  The kernel is the headline pipeline's
// row walk — u rows from the rect image (r2h) or the input rows, the 7-tap stencil as packed
// FMAs into three conv-row accumulators — with the hexresize triangle as its output stage:
// every second step completes the two conv rows one output row reads.  Tried first by
// hg_hex_pyramid_level (pyramid.hip); returns HG_EUNSUP outside its domain (then
// k_pyr_stream, then k_pyr_level).  With `dry` nothing is launched and the kernel that
// would run (HG_PYR_FUSED / HG_PYR_FUSED_SHORT) is returned.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "fused_kernel.h"

namespace hg {

template <typename Tin, typename Tout, int C, int MD>
static int pf_launch(const void* x, const float* taps, const float* bias, void* y,
                     const FusedGeom& F, int op, hipStream_t st) {
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + FU_GW - 1) / FU_GW);
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(FU_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, C, C, 1, MD>), grid, blk, 0, st, (const Tin*)x,
                           taps, bias, (Tout*)y, F);
    else
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, C, C, 0, MD>), grid, blk, 0, st, (const Tin*)x,
                           taps, bias, (Tout*)y, F);
    return launch_status();
}

template <typename Tin, typename Tout>
static int pf_channels(const void* x, const float* taps, const float* bias, void* y,
                       const FusedGeom& F, int C, int md, int op, hipStream_t st) {
#define HG_PF_MD(CC)                                                                          \
    switch (md) {                                                                             \
    case 3: return pf_launch<Tin, Tout, CC, 3>(x, taps, bias, y, F, op, st);                  \
    case 4: return pf_launch<Tin, Tout, CC, 4>(x, taps, bias, y, F, op, st);                  \
    default: return pf_launch<Tin, Tout, CC, 5>(x, taps, bias, y, F, op, st);                 \
    }
    if (C == 3) { HG_PF_MD(3) }
    if (C == 1) { HG_PF_MD(1) }
#undef HG_PF_MD
    return HG_EUNSUP;
}

// The hexresize lattice class the output stage assumes, checked on the lattice itself
// (O(h2 + w2)): i_n(a) - 2a in {0, 1} for every output row, and 1 only where conv row
// i_n(a) + 1 is outside the raster (the kernel has conv row 2a + 2 only one step later);
// 2a + 1 < h1 (the step that outputs row a exists); c0 - 2b in {-1, 0, 1} and
// c1 - 2b in {-2 .. 1} (bounded by the extreme row and column terms plus a margin for the
// fp64 rounding of j_, as k_pyr_stream's check).
static bool pf_lattice_ok(const Geom& g) {
    double qmin = 1e300, qmax = -1e300, gmin = 1e300, gmax = -1e300;
    const double ch = (double)(g.h - 1) * 0.5, cw = ((double)g.w - 0.5) * 0.5;
    for (int64_t a = 0; a < g.h1; ++a) {
        const double i_ = axis_at(g.xs, a) + ch;
        const int64_t in = (int64_t)i_;
        const int64_t e = in - 2 * a;
        if (e < 0 || e > 1 || in < 0 || in >= g.h || 2 * a + 1 >= g.h) return false;
        if (e == 1 && in + 1 < g.h) return false;
        const double q = 0.5 * (i_ - (double)in) - 0.5 * (double)e;
        qmin = std::min(qmin, q);
        qmax = std::max(qmax, q);
    }
    for (int64_t b = 0; b < g.w1; ++b) {
        const double gb = axis_at(g.ys, b) + cw - 2.0 * (double)b;
        gmin = std::min(gmin, gb);
        gmax = std::max(gmax, gb);
    }
    const double eps = 1e-6;
    return qmin + gmin - eps >= -1.0 && qmax + gmax + eps < 2.0;
}

// FR: the same-size rect -> hex lattice is the near-identity one the fused kernel's u rows
// assume (every live tap within one row / column below the sample: in - r, jn - q in {-1, 0})
static bool pf_r2h_ok(const Geom& g) {
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

int pyr_fused_try(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                  int64_t C, int64_t h, int64_t w, int64_t h1, int64_t w1, const float* taps,
                  const float* bias, int even_odd_offset, int from_rect, hipStream_t st,
                  bool dry) {
    if (C != 1 && C != 3) return HG_EUNSUP;
    if ((w & 1) || w < 2 || h < 2 || h1 < 1 || w1 < 1 || batch < 1) return HG_EUNSUP;
    if (src_dtype != HG_F16 && src_dtype != HG_BF16) return HG_EUNSUP;
    if (dst_dtype != src_dtype && dst_dtype != HG_F32) return HG_EUNSUP;
    if (reinterpret_cast<uintptr_t>(src) & 3) return HG_EUNSUP;   // dword loads
    // 32-bit buffer offsets, including the past-the-range loads and stores
    if (C * h * w * 2 >= ((int64_t)1 << 31) || C * h1 * w1 * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;
    const Geom g = make_tri(h, w, h1, w1, 0.5);
    if (!pf_lattice_ok(g)) return HG_EUNSUP;
    FusedGeom F = {};
    F.B = batch;
    F.h = (int)h; F.w = (int)w;           // input (rect for MD 3, hex for MD 4)
    F.h1 = (int)h; F.w1 = (int)w;         // hex / conv image: same size
    F.h2 = (int)h1; F.w2 = (int)w1;       // level output
    F.txs = g.xs;
    F.tys = g.ys;
    if (from_rect) {
        const Geom r = make_r2h(h, w, h, w);
        if (!pf_r2h_ok(r)) return HG_EUNSUP;
        F.rxs = r.xs;
        F.rys = r.ys;
    }
    F.nwin = (int)((w1 + FU_OWN / 2 - 1) / (FU_OWN / 2));
    // From a hex image: a level whose 60-row bands give fewer than six rounds of waves over
    // the chip (256 CUs x 4 SIMDs x 4 waves) runs on short bands (MD 5): the last round of a
    // launch that is only a few rounds long is mostly idle.  A/B switch HYGRID_PYR_SHORT=0/1
    // (exactly "0" or "1"; anything else: the rule above).
    int md = from_rect ? 3 : 4;
    if (!from_rect) {
        const int64_t waves = batch * ((h + fu_rb(4) - 1) / fu_rb(4)) * (int64_t)F.nwin;
        bool shrt = waves < 6 * 4096;
        if (env_is("HYGRID_PYR_SHORT", "1")) shrt = true;
        if (env_is("HYGRID_PYR_SHORT", "0")) shrt = false;
        if (shrt) md = 5;
    }
    if (dry) return md == 5 ? HG_PYR_FUSED_SHORT : HG_PYR_FUSED;
    F.nband = (int)((h + fu_rb(md) - 1) / fu_rb(md));
    const int op = (even_odd_offset + 1) & 1;   // tap column class at padding 1
    if (src_dtype == HG_F16)
        return dst_dtype == HG_F32 ? pf_channels<_Float16, float>(src, taps, bias, dst, F, (int)C, md, op, st)
                                   : pf_channels<_Float16, _Float16>(src, taps, bias, dst, F, (int)C, md, op, st);
    return dst_dtype == HG_F32 ? pf_channels<__bf16, float>(src, taps, bias, dst, F, (int)C, md, op, st)
                               : pf_channels<__bf16, __bf16>(src, taps, bias, dst, F, (int)C, md, op, st);
}

}  // namespace hg
