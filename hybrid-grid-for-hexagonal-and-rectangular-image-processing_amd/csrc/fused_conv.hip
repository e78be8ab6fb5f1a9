// fused_conv.hip — HexConv2d(radius 2, stride 1, padding 1, pad value 0) on the
// two-column streaming kernel (fused_kernel.h, MD 1), tried first by the conv fast path
// (conv_stream.hip).  HexFrames.py:96-169: output (B, O, h, w) fp32-accumulated from
// the 7 taps of the type1 geometry (HexFrames.py:417-445) with the padded border of the
// reference (zeros).  Lane l owns columns W0+2l, W0+2l+1; per step one input row is
// loaded (PD rows ahead) and scattered into the three conv rows it feeds.
#include <climits>
#include <cstdlib>

#include "fused_kernel.h"

namespace hg {

template <typename Tin, typename Tout, int C, int O, int G>
static int fconv_launch(const void* x, const float* k, const float* bias, void* y,
                        const FusedGeom& F, int op, hipStream_t st) {
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + FU_GW - 1) / FU_GW);
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(FU_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, O, G, 1, 1>), grid, blk, 0, st, (const Tin*)x, k,
                           bias, (Tout*)y, F);
    else
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, O, G, 0, 1>), grid, blk, 0, st, (const Tin*)x, k,
                           bias, (Tout*)y, F);
    return launch_status();
}

template <typename Tin, typename Tout>
static int fconv_channels(const void* x, const float* k, const float* b, void* y,
                          const FusedGeom& F, int C, int O, int G, int op, hipStream_t st) {
    if (C == 3 && O == 3 && G == 1) return fconv_launch<Tin, Tout, 3, 3, 1>(x, k, b, y, F, op, st);
    if (C == 3 && O == 3 && G == 3) return fconv_launch<Tin, Tout, 3, 3, 3>(x, k, b, y, F, op, st);
    if (C == 1 && O == 1 && G == 1) return fconv_launch<Tin, Tout, 1, 1, 1>(x, k, b, y, F, op, st);
    return HG_EUNSUP;
}

int fused_conv_try(const void* x, const float* kernel, const float* bias, void* y, int x_dtype,
                   int y_dtype, int64_t batch, int C, int O, int G, int64_t h, int64_t w,
                   int padding, int off, double pad_value, bool epilogue, hipStream_t st) {
    if (env_is("HYGRID_FCONV", "0")) return HG_EUNSUP;   // A/B switch: conv_stream kernel
    if (epilogue || padding != 1 || pad_value != 0.0) return HG_EUNSUP;
    if ((w & 1) || w < 2 || h < 1 || batch < 1) return HG_EUNSUP;   // dword column pairs
    if (C * h * w * 8 >= ((int64_t)1 << 31) || O * h * w * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;   // 32-bit buffer offsets, incl. the past-the-range zero loads
    FusedGeom F = {};
    F.B = batch;
    F.h = F.h1 = F.h2 = (int)h;
    F.w = F.w1 = F.w2 = (int)w;
    F.nwin = (int)((w + FU_OWN - 1) / FU_OWN);
    F.nband = (int)((h + fu_rb(1) - 1) / fu_rb(1));
    const int op = (off + padding) & 1;
    if (x_dtype == HG_BF16 && y_dtype == HG_BF16)
        return fconv_channels<__bf16, __bf16>(x, kernel, bias, y, F, C, O, G, op, st);
    if (x_dtype == HG_BF16 && y_dtype == HG_F32)
        return fconv_channels<__bf16, float>(x, kernel, bias, y, F, C, O, G, op, st);
    if (x_dtype == HG_F16 && y_dtype == HG_F16)
        return fconv_channels<_Float16, _Float16>(x, kernel, bias, y, F, C, O, G, op, st);
    if (x_dtype == HG_F16 && y_dtype == HG_F32)
        return fconv_channels<_Float16, float>(x, kernel, bias, y, F, C, O, G, op, st);
    if (x_dtype == HG_F32 && y_dtype == HG_F32)
        return fconv_channels<float, float>(x, kernel, bias, y, F, C, O, G, op, st);
    return HG_EUNSUP;
}

}  // namespace hg
