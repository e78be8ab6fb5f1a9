// fused.hip — streaming rect -> hex -> HexConv2d(r=2) -> hex -> rect pass, two
// columns per lane (the headline path of hg_pipeline_r2h_conv_h2r).
//
// The reference chains rect_to_hex_resample (geometry_np.py:358-519, bilinear),
// HexConv2d (HexFrames.py:96-169, radius 2, stride 1, padding 1, constant 0) and
// hex_to_rect_resample (geometry_np.py:191-356, linear).  This kernel covers the
// geometry every same-size round trip has, and checks it on the host:
//   * r2h rows:    u row r blends rect rows in(r), in(r)+1 with in(r) - r in {-1, 0}
//                  wherever a tap is inside the raster (geometry_np.py:440-486);
//   * r2h columns: hex column q blends rect columns jn, jn+1 with jn - q in {-1, 0};
//   * h2r:         (h2, w2) == (ho, wo), so the triangle lattice is exact:
//                  i_ = a, j_ = 0.5a + b + 0.25 (:276-277) -> even rows
//                  0.75 z[b] + 0.25 z[b+1], odd rows 0.25 z[b-1] + 0.75 z[b] (:347-354).
// Everything else goes to pipeline.hip's kernels.
//
// Execution model.  One wavefront owns a 128-column window (lane l <-> columns
// W0 + 2l, W0 + 2l + 1 in every stage's column space) of one image and walks a band
// of 126 output rows.  Per output row a2 (one "step"):
//   1. rect row a2+2 arrives in registers (loaded PD steps earlier; every rect row is
//      loaded exactly once — a 3-row register ring, not a (in, in+1) pair per row);
//   2. v = a*x[r-1] + b*x[r] + c*x[r+1] for u row r = a2+1 (uniform row weights from a
//      per-wave LDS table, validity folded in);
//   3. u = wl*v[q-1] + wc*v[q] + wr*v[q+1] (per-column weights; the neighbour columns
//      are the lane's other column or one DPP wave shift away);
//   4. u row r is scattered into the three conv rows it feeds (r-1 below, r centre,
//      r+1 above; 7 taps x C x O FMAs with weights in VGPRs), so only the newest u row
//      and three accumulator rows are live;
//   5. conv row a2 is complete: the fixed two-tap h2r filter, cvt, one dword store per
//      output channel (non-owned lanes store past the buffer range: dropped).
// The step loop is unrolled by 6 = lcm(3 ring slots, 2 row parities), so ring slots
// and tap offsets are compile-time constants and no register moves between steps.
#include <climits>
#include <cmath>
#include <cstdlib>

#include "fused_kernel.h"

namespace hg {

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout, int C, int O, int G>
static int fused_launch(const void* x, const float* k, const float* bias, void* y,
                        const FusedGeom& F, int op, hipStream_t st) {
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + FU_GW - 1) / FU_GW);
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(FU_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, O, G, 1>), grid, blk, 0, st, (const Tin*)x, k,
                           bias, (Tout*)y, F);
    else
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, O, G, 0>), grid, blk, 0, st, (const Tin*)x, k,
                           bias, (Tout*)y, F);
    return launch_status();
}

template <typename Tin, typename Tout>
static int fused_channels(const void* x, const float* k, const float* b, void* y,
                          const FusedGeom& F, int C, int O, int G, int op, hipStream_t st) {
    if (C == 3 && O == 3 && G == 1) return fused_launch<Tin, Tout, 3, 3, 1>(x, k, b, y, F, op, st);
    if (C == 3 && O == 3 && G == 3) return fused_launch<Tin, Tout, 3, 3, 3>(x, k, b, y, F, op, st);
    if (C == 1 && O == 1 && G == 1) return fused_launch<Tin, Tout, 1, 1, 1>(x, k, b, y, F, op, st);
    return HG_EUNSUP;
}

// Does the same-size streaming kernel cover this call?  All checks are exact on the
// lattice the kernel would compute (O(h1 + w1) fp64 on the host).
static bool fused_geometry_ok(const Geom& g) {
    for (int64_t q = 0; q < g.w1; ++q) {            // r2h columns: jn - q in {-1, 0}
        const double j_ = axis_at(g.ys, q) + (double)(g.w - 1) * 0.5;
        const int64_t jn = (int64_t)j_;
        const bool live = (jn >= 0 && jn < g.w) || (jn + 1 >= 0 && jn + 1 < g.w);
        if (live && (jn - q < -1 || jn - q > 0)) return false;
    }
    for (int64_t r = 0; r < g.h1; ++r) {            // r2h rows: in - r in {-1, 0}
        const double i_ = axis_at(g.xs, r) + (double)(g.h - 1) * 0.5;
        const int64_t in = (int64_t)i_;
        const bool live = (in >= 0 && in < g.h) || (in + 1 >= 0 && in + 1 < g.h);
        if (live && (in - r < -1 || in - r > 0)) return false;
    }
    return true;
}

// Round trip rect -> hex -> rect without the conv (MD 2), one plane per "image" (C = 1):
// geometry_np.hex_to_rect_resample(rect_to_hex_resample(x, (h1, w1)), (h1, w1)) with the hex
// image kept on chip in fp32.
int fused_rt_try(const void* x, void* y, int x_dtype, int y_dtype, int64_t planes, int64_t h,
                 int64_t w, int64_t h1, int64_t w1, hipStream_t st) {
    if (env_is("HYGRID_FUSED2", "0")) return HG_EUNSUP;   // A/B switch for measurements
    if ((w & 1) || (w1 & 1) || w < 2 || h1 < 1 || planes < 1) return HG_EUNSUP;
    if (x_dtype != HG_BF16 && x_dtype != HG_F16 && x_dtype != HG_F32) return HG_EUNSUP;
    if (y_dtype != HG_BF16 && y_dtype != HG_F16 && y_dtype != HG_F32) return HG_EUNSUP;
    if (h * w * 8 >= ((int64_t)1 << 31) || h1 * w1 * 4 >= ((int64_t)1 << 31)) return HG_EUNSUP;
    const Geom g = make_r2h(h, w, h1, w1);
    if (!fused_geometry_ok(g)) return HG_EUNSUP;
    FusedGeom F;
    F.B = planes;
    F.h = (int)h; F.w = (int)w; F.h1 = (int)h1; F.w1 = (int)w1; F.h2 = (int)h1; F.w2 = (int)w1;
    F.rxs = g.xs;
    F.rys = g.ys;
    F.nwin = (int)((w1 + FU_OWN - 1) / FU_OWN);
    F.nband = (int)((h1 + fu_rb(2) - 1) / fu_rb(2));
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + FU_GW - 1) / FU_GW);
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(FU_THREADS);
#define HG_RT(TI, TO)                                                                          \
    hipLaunchKernelGGL((k_fused<TI, TO, 1, 1, 1, 0, 2>), grid, blk, 0, st, (const TI*)x,        \
                       (const float*)nullptr, (const float*)nullptr, (TO*)y, F);               \
    return launch_status();
    if (x_dtype == HG_F32 && y_dtype == HG_F32) { HG_RT(float, float) }
    if (x_dtype == HG_BF16 && y_dtype == HG_BF16) { HG_RT(__bf16, __bf16) }
    if (x_dtype == HG_F16 && y_dtype == HG_F16) { HG_RT(_Float16, _Float16) }
    if (x_dtype == HG_BF16 && y_dtype == HG_F32) { HG_RT(__bf16, float) }
    if (x_dtype == HG_F16 && y_dtype == HG_F32) { HG_RT(_Float16, float) }
#undef HG_RT
    return HG_EUNSUP;
}

// fused4.hip: the 4-column variant of MD 0 (bf16, C = O = 3), or HG_EUNSUP
int fused4_try(const void* x, const float* k, const float* bias, void* y, int x_dtype, int y_dtype,
               int C, int O, int G, const FusedGeom& F0, int op, hipStream_t st);

int fused_try(const void* x, const float* kernel, const float* bias, void* y, int x_dtype,
              int y_dtype, int64_t batch, int C, int O, int G, int64_t h, int64_t w,
              int64_t h1, int64_t w1, int64_t h2, int64_t w2, int padding, int op,
              double pad_value, hipStream_t st) {
    if (env_is("HYGRID_FUSED2", "0")) return HG_EUNSUP;   // A/B switch for measurements
    if (padding != 1 || pad_value != 0.0) return HG_EUNSUP;
    if (h2 != h1 || w2 != w1) return HG_EUNSUP;       // ho = h1, wo = w1 at padding 1
    if ((w & 1) || (w1 & 1) || w < 2 || h1 < 1) return HG_EUNSUP;   // dword column pairs
    if (x_dtype != HG_BF16 && x_dtype != HG_F16 && x_dtype != HG_F32) return HG_EUNSUP;
    if (y_dtype != HG_BF16 && y_dtype != HG_F16 && y_dtype != HG_F32) return HG_EUNSUP;
    if (C * h * w * 8 >= ((int64_t)1 << 31) || O * h2 * w2 * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;   // 32-bit buffer offsets, incl. the past-the-range zero loads
    const Geom g = make_r2h(h, w, h1, w1);
    if (!fused_geometry_ok(g)) return HG_EUNSUP;
    FusedGeom F;
    F.B = batch;
    F.h = (int)h; F.w = (int)w; F.h1 = (int)h1; F.w1 = (int)w1; F.h2 = (int)h2; F.w2 = (int)w2;
    F.rxs = g.xs;
    F.rys = g.ys;
    F.nwin = (int)((w2 + FU_OWN - 1) / FU_OWN);
    F.nband = (int)((h2 + fu_rb(0) - 1) / fu_rb(0));
    {
        const int rc4 = fused4_try(x, kernel, bias, y, x_dtype, y_dtype, C, O, G, F, op, st);
        if (rc4 != HG_EUNSUP) return rc4;
    }
#if FU_MIN_INST == 2   // debugging variants: fp32 C = O = 1 only
    if (x_dtype == HG_F32 && y_dtype == HG_F32 && C == 1 && O == 1 && G == 1)
        return fused_launch<float, float, 1, 1, 1>(x, kernel, bias, y, F, op, st);
    return HG_EUNSUP;
#elif FU_MIN_INST   // tuning variants: only the headline instantiation (fast rebuilds)
    if (x_dtype == HG_BF16 && y_dtype == HG_BF16 && C == 3 && O == 3 && G == 1)
        return fused_launch<__bf16, __bf16, 3, 3, 1>(x, kernel, bias, y, F, op, st);
    return HG_EUNSUP;
#endif
    switch (x_dtype) {
    case HG_BF16:
        switch (y_dtype) {
        case HG_BF16: return fused_channels<__bf16, __bf16>(x, kernel, bias, y, F, C, O, G, op, st);
        case HG_F32: return fused_channels<__bf16, float>(x, kernel, bias, y, F, C, O, G, op, st);
        default: return HG_EUNSUP;
        }
    case HG_F16:
        switch (y_dtype) {
        case HG_F16: return fused_channels<_Float16, _Float16>(x, kernel, bias, y, F, C, O, G, op, st);
        case HG_F32: return fused_channels<_Float16, float>(x, kernel, bias, y, F, C, O, G, op, st);
        default: return HG_EUNSUP;
        }
    default:   // HG_F32
        switch (y_dtype) {
        case HG_F32: return fused_channels<float, float>(x, kernel, bias, y, F, C, O, G, op, st);
        case HG_BF16: return fused_channels<float, __bf16>(x, kernel, bias, y, F, C, O, G, op, st);
        default: return HG_EUNSUP;
        }
    }
}

}  // namespace hg

namespace hg {
void fused4_layout(int* band_rows, int* win_own, int* win_halo);
}

// md 0-2: the two-column kernel's modes; md 6: MD 0's four-column variant (fused4.hip: bf16,
// C = O = 3, widths a multiple of 4).  (md 7 / 8, round 5's four-column round trip and conv,
// were removed in round 6: HG_EINVAL.)
extern "C" int hg_fused_layout(int md, int* band_rows, int* win_own, int* win_halo) {
    if (!band_rows || !win_own || !win_halo) return HG_EINVAL;
    if (md == 6) {
        hg::fused4_layout(band_rows, win_own, win_halo);
        return HG_OK;
    }
    if (md < 0 || md > 2) return HG_EINVAL;
    *band_rows = hg::fu_rb(md);
    *win_own = hg::FU_OWN;
    *win_halo = hg::FU_HL;
    return HG_OK;
}
