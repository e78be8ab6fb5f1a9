// hexconv_geom.h — HexConv2d index geometry shared by the forward (hexconv.hip) and
// backward (hexconv_bwd.hip) kernels: the padding-mode index map, the tap table and
// the output shape (HexFrames.py:13-21, :114-118, :127-169; derivation in
// oracle/hg_oracle.c).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace hg {

// torch.nn.functional.pad index map of a padded coordinate i (un-padded frame) onto
// the raster [0, n); -1 for constant padding outside.
__host__ __device__ inline int64_t pad_map(int64_t i, int64_t n, int mode) {
    if (i >= 0 && i < n) return i;
    switch (mode) {
    case HG_PAD_REFLECT:
        while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * (n - 1) - i; }
        return i;
    case HG_PAD_REPLICATE:
        return i < 0 ? 0 : n - 1;
    case HG_PAD_CIRCULAR:
        return ((i % n) + n) % n;
    default:
        return -1;
    }
}

// Tap table in kernel-flattening order (HexFrames.py:114-118): tap t of output row
// (ro, q) reads P[s*ro + dy][s*q + dk(ro & 1)].
__host__ __device__ inline void tap_geom(int r, int s, int d, int op, int t, int* dy, int* dk0,
                                         int* dk1) {
    int n = 0;
    for (int ii = 0; ii < 2 * r - 1; ++ii) {
        int tt = ii - r + 1;
        tt = tt < 0 ? -tt : tt;
        const int ln = 2 * r - 1 - tt;
        if (t < n + ln) {
            const int m = t - n;
            const int col = tt * d + 2 * d * m;
            *dy = ii * d;
            for (int par = 0; par < 2; ++par) {
                const int y = par * s + ii * d;
                const int L = ((y & 1) + op) & 1;
                const int dk = (1 + par * s + col - L) >> 1;
                if (par == 0) *dk0 = dk; else *dk1 = dk;
            }
            return;
        }
        n += ln;
    }
}

// Output size (HexFrames.py:127-169): both strided convolutions need >= k_h rows and
// >= k_w type1 columns.
inline int conv_out_shape(int64_t h, int64_t w, int r, int s, int p, int d, int64_t* ho,
                          int64_t* wo) {
    if (r < 1 || s < 1 || d < 1 || p < 0 || h < 0 || w < 0) return HG_EINVAL;
    const int64_t kh = (int64_t)(2 * r - 2) * d + 1;
    const int64_t kw = (int64_t)2 * d * (2 * r - 2) + 1;
    const int64_t H = h + 2 * p, W = w + 2 * p;
    if (H < kh || 2 * W - s < kw) return HG_ESHAPE;
    *ho = (H - kh) / s + 1;
    *wo = (2 * W - s - kw) / (2 * s) + 1;
    return HG_OK;
}

// Argument checks shared by forward and backward (torch's pad rules for the modes).
inline int conv_check_args(int64_t batch, int64_t C, int64_t O, int64_t h, int64_t w,
                           int groups, int padding, int pad_mode) {
    if (batch < 0 || C < 1 || O < 1 || groups < 1) return HG_EINVAL;
    if (C % groups || O % groups) return HG_EINVAL;
    if (pad_mode < HG_PAD_CONSTANT || pad_mode > HG_PAD_CIRCULAR) return HG_EINVAL;
    if (pad_mode == HG_PAD_REFLECT && padding > 0 && (padding >= h || padding >= w))
        return HG_ESHAPE;
    if (pad_mode != HG_PAD_CONSTANT && padding > 0 && (h == 0 || w == 0)) return HG_ESHAPE;
    if (pad_mode == HG_PAD_CIRCULAR && (padding > h || padding > w)) return HG_ESHAPE;
    return HG_OK;
}

}  // namespace hg
