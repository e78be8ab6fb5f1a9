// formats.hip — hex raster storage formats: pure memory permutes.
//
// type1 ("double-width offset") raster, HexFrames.heximage_to_type1 (HexFrames.py:417-445)
// and HEXIMAGE.GenerateType1Image (HexImage.py:139-153): an (h, w) offset-row hex image
// becomes (h, 2w+1) with
//     T[y][2k + L(y)] = T[y][2k + 1 + L(y)] = x[y][k],   L(y) = (y % 2 + off) % 2,
// and zeros elsewhere (the reference builds it with repeat / insert / append per row).
// type2 (HexFrames.py:446-449, HexImage.py:154-170) is type1 with every row doubled.
// Decoding (HEXIMAGE(data=..., heximagetype=1|2), HexImage.py:108-111, and
// type1_to_heximage, HexFrames.py:450-458) is a strided gather, provided here as a
// generic 2-D strided copy.  Both kernels are element-size generic (1/2/4/8 bytes):
// one thread per output element, consecutive threads on consecutive output columns
// (coalesced stores; the type1 reads hit each source element twice from L1/L2).
#include <algorithm>
#include <climits>

#include "common.h"

namespace hg {

constexpr int FM_THREADS = 256;

template <typename E>
__global__ __launch_bounds__(FM_THREADS) void k_to_type1(const E* __restrict__ src, E* __restrict__ dst,
                                                         int64_t planes, int64_t h, int64_t w,
                                                         int off, int rep) {
    const int64_t W1 = 2 * w + 1, H1 = h * rep;
    const int64_t total = planes * H1 * W1;
    for (int64_t i = (int64_t)blockIdx.x * FM_THREADS + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * FM_THREADS) {
        const int64_t u = i % W1, t = i / W1;
        const int64_t yy = t % H1, p = t / H1;
        const int64_t y = yy / rep;
        const int64_t L = ((y & 1) + off) & 1;
        const int64_t k = (u - L) >> 1;               // u - L in [2k, 2k+1]
        E v = E(0);
        if (u >= L && k < w) v = src[(p * h + y) * w + k];
        dst[i] = v;
    }
}

template <typename E>
__global__ __launch_bounds__(FM_THREADS) void k_strided2d(const E* __restrict__ src, E* __restrict__ dst,
                                                          int64_t planes, int64_t H, int64_t W,
                                                          int64_t r0, int64_t rs, int64_t c0,
                                                          int64_t cs, int64_t ho, int64_t wo) {
    const int64_t total = planes * ho * wo;
    for (int64_t i = (int64_t)blockIdx.x * FM_THREADS + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * FM_THREADS) {
        const int64_t j = i % wo, t = i / wo;
        const int64_t r = t % ho, p = t / ho;
        dst[i] = src[(p * H + r0 + r * rs) * W + c0 + j * cs];
    }
}

static unsigned fm_blocks(int64_t total) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((total + FM_THREADS - 1) / FM_THREADS,
                                                            1 << 20));
}

}  // namespace hg

extern "C" {

int hg_hex_to_type1(const void* src, void* dst, int elem_size, int64_t planes, int64_t h,
                    int64_t w, int even_odd_offset, int row_repeat, void* stream) {
    using namespace hg;
    if (planes < 0 || h < 0 || w < 0 || (row_repeat != 1 && row_repeat != 2)) return HG_EINVAL;
    const int64_t total = planes * h * row_repeat * (2 * w + 1);
    if (total == 0) return HG_OK;
    if (!src || !dst) return HG_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int off = even_odd_offset & 1;
    const unsigned nb = fm_blocks(total);
    switch (elem_size) {
    case 1: hipLaunchKernelGGL(k_to_type1<uint8_t>, dim3(nb), dim3(FM_THREADS), 0, st, (const uint8_t*)src, (uint8_t*)dst, planes, h, w, off, row_repeat); break;
    case 2: hipLaunchKernelGGL(k_to_type1<uint16_t>, dim3(nb), dim3(FM_THREADS), 0, st, (const uint16_t*)src, (uint16_t*)dst, planes, h, w, off, row_repeat); break;
    case 4: hipLaunchKernelGGL(k_to_type1<uint32_t>, dim3(nb), dim3(FM_THREADS), 0, st, (const uint32_t*)src, (uint32_t*)dst, planes, h, w, off, row_repeat); break;
    case 8: hipLaunchKernelGGL(k_to_type1<uint64_t>, dim3(nb), dim3(FM_THREADS), 0, st, (const uint64_t*)src, (uint64_t*)dst, planes, h, w, off, row_repeat); break;
    default: return HG_EDTYPE;
    }
    return launch_status();
}

int hg_strided_copy2d(const void* src, void* dst, int elem_size, int64_t planes, int64_t H,
                      int64_t W, int64_t row_start, int64_t row_step, int64_t col_start,
                      int64_t col_step, int64_t h_out, int64_t w_out, void* stream) {
    using namespace hg;
    if (planes < 0 || H < 0 || W < 0 || h_out < 0 || w_out < 0 || row_step < 1 || col_step < 1 ||
        row_start < 0 || col_start < 0)
        return HG_EINVAL;
    const int64_t total = planes * h_out * w_out;
    if (total == 0) return HG_OK;
    if (row_start + (h_out - 1) * row_step >= H || col_start + (w_out - 1) * col_step >= W)
        return HG_ESHAPE;
    if (!src || !dst) return HG_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const unsigned nb = fm_blocks(total);
#define HG_SC(E) hipLaunchKernelGGL(k_strided2d<E>, dim3(nb), dim3(FM_THREADS), 0, st, (const E*)src, \
                                    (E*)dst, planes, H, W, row_start, row_step, col_start, col_step,  \
                                    h_out, w_out)
    switch (elem_size) {
    case 1: HG_SC(uint8_t); break;
    case 2: HG_SC(uint16_t); break;
    case 4: HG_SC(uint32_t); break;
    case 8: HG_SC(uint64_t); break;
    default: return HG_EDTYPE;
    }
#undef HG_SC
    return launch_status();
}

}  // extern "C"
