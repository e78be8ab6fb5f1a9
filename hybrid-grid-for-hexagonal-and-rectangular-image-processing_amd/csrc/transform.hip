// transform.hip — gfx950 kernel for image_geometric_transformation: an affine
// homography of a hex raster onto a new hex lattice.
//
// Reference: /root/reference/HyGrid/geometry_np.py:6-189 (and its torch twin
// geometry_torch.py:7-189).  The host (Python) computes what is O(h1 + w1): the output
// axes np.arange(h1_inf, h1_sup + 1, 1) / np.arange(w1_inf, w1_sup + 0.5, 1) of the
// transformed corners (:56-87) and inv(H) (:97-102).  Per output sample (a, b) the
// kernel forms the inverse-mapped point
//     X = xs[a],  Y = ys[b] + (a odd ? 0.5 : 0)                    (:80-87)
//     x_ = (Hi00*X + Hi01*Y) + Hi02,  y_ = (Hi10*X + Hi11*Y) + Hi12  (einsum, :97-102)
// then the same triangle sample as hex->rect (lattice.h tri_sample_xy, :107-187), so
// the integer maps and fp64 weights are the reference's bit for bit (the library is
// built with -ffp-contract=off).  As in the reference, H's third row is not applied
// (no perspective divide).
//
// Layout: `planes` contiguous rasters (h, w) in, (h1, w1) out.  One thread per output
// sample computes the lattice record once (fp64) and walks a chunk of planes with it;
// a wave stores 64 consecutive output samples (coalesced).  The gathers are irregular
// (rotations, shears), so no LDS staging: the source footprint of a workgroup is small
// and L2-resident.  This op is not on the headline path; its bound is the fp64 lattice
// work at small plane counts and HBM (gathers + stores) at large ones.
#include <climits>

#include "common.h"
#include "lattice.h"

namespace hg {

constexpr int TF_THREADS = 256;

struct Homog {
    double m[6];  // rows 0 and 1 of inv(H)
};

__device__ __forceinline__ TriSample homog_sample(const Geom& g, const double* __restrict__ xs,
                                                  const double* __restrict__ ys,
                                                  const Homog& hm, int64_t a, int64_t b) {
    const double X = xs[a];
    const double Y = (a & 1) ? ys[b] + 0.5 : ys[b];
    const double x_ = (hm.m[0] * X + hm.m[1] * Y) + hm.m[2];
    const double y_ = (hm.m[3] * X + hm.m[4] * Y) + hm.m[5];
    return tri_sample_xy(g, x_, y_);
}

// Linear: alpha*p1 + beta*p2 + gamma*p3 in fp64 (numpy order, :184), invalid vertices 0.
// Nearest: the first-minimum vertex (geometry_torch.py:165-173), copied bit for bit.
template <typename Tin, typename Tout, bool NEAREST>
__global__ __launch_bounds__(TF_THREADS) void k_homography(
    const Tin* __restrict__ src, Tout* __restrict__ dst, Geom g, const double* __restrict__ xs,
    const double* __restrict__ ys, Homog hm, int64_t planes, int pc) {
    const int64_t n = g.h1 * g.w1;
    const int64_t q = (int64_t)blockIdx.x * TF_THREADS + threadIdx.x;
    if (q >= n) return;
    const int64_t a = q / g.w1, b = q - a * g.w1;
    const TriSample s = homog_sample(g, xs, ys, hm, a, b);
    const int64_t p0 = (int64_t)blockIdx.y * pc;
    const int64_t p1 = p0 + pc < planes ? p0 + pc : planes;
    const int64_t hw = g.h * g.w;
    if constexpr (NEAREST) {
        const int m = s.argmin;
        const int64_t off = ((s.vk >> m) & 1) ? tri_pick_r(s, m) * g.w + tri_pick_c(s, m) : -1;
        for (int64_t p = p0; p < p1; ++p)
            dst[p * n + q] = off >= 0 ? src[p * hw + off] : (Tout)0;
    } else {
        int64_t off[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) off[k] = ((s.vk >> k) & 1) ? s.r[k] * g.w + s.c[k] : -1;
        for (int64_t p = p0; p < p1; ++p) {
            const Tin* sp = src + p * hw;
            const double v1 = off[0] >= 0 ? (double)sp[off[0]] : 0.0;
            const double v2 = off[1] >= 0 ? (double)sp[off[1]] : 0.0;
            const double v3 = off[2] >= 0 ? (double)sp[off[2]] : 0.0;
            dst[p * n + q] = (Tout)((s.alpha * v1 + s.beta * v2) + s.gamma * v3);
        }
    }
}

// Lattice maps of one transform, same layout as hg_lattice_maps, plus the mapped
// point: fmaps has 7 planes (i_f, j_f, alpha, beta, gamma, x_, y_).
__global__ void k_homography_maps(Geom g, const double* __restrict__ xs,
                                  const double* __restrict__ ys, Homog hm,
                                  int32_t* __restrict__ im, double* __restrict__ fm) {
    const int64_t n = g.h1 * g.w1;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const int64_t a = q / g.w1, b = q - a * g.w1;
    const TriSample s = homog_sample(g, xs, ys, hm, a, b);
    if (im) {
        im[q] = (int32_t)s.i_n; im[n + q] = (int32_t)s.j_n; im[2 * n + q] = s.flag;
        im[3 * n + q] = s.valid; im[4 * n + q] = s.argmin;
    }
    if (fm) {
        const double X = xs[a];
        const double Y = (a & 1) ? ys[b] + 0.5 : ys[b];
        fm[q] = s.i_f; fm[n + q] = s.j_f;
        fm[2 * n + q] = s.alpha; fm[3 * n + q] = s.beta; fm[4 * n + q] = s.gamma;
        fm[5 * n + q] = (hm.m[0] * X + hm.m[1] * Y) + hm.m[2];
        fm[6 * n + q] = (hm.m[3] * X + hm.m[4] * Y) + hm.m[5];
    }
}

static Geom homog_geom(int64_t h, int64_t w, int64_t h1, int64_t w1) {
    Geom g = make_tri(h, w, h1, w1, 0.5);   // only h, w, h1, w1, hh, ww are read
    return g;
}

static int homog_check(int64_t planes, int64_t h, int64_t w, int64_t h1, int64_t w1) {
    if (planes < 0 || h < 0 || w < 0 || h1 < 0 || w1 < 0) return HG_EINVAL;
    // the triangle records hold 32-bit rows/cols; i_n etc. are int64 in the sample
    if (h > INT_MAX / 2 || w > INT_MAX / 2 || h1 > INT_MAX / 2 || w1 > INT_MAX / 2)
        return HG_ESHAPE;
    if (h1 * w1 > (int64_t)INT_MAX * TF_THREADS) return HG_ESHAPE;
    return HG_OK;
}

template <typename Tin, typename Tout, bool NEAREST>
static int launch_homog(const void* src, void* dst, const Geom& g, const double* xs,
                        const double* ys, const Homog& hm, int64_t planes, hipStream_t s) {
    const int64_t n = g.h1 * g.w1;
    if (n == 0 || planes == 0) return HG_OK;
    const int64_t bx = (n + TF_THREADS - 1) / TF_THREADS;
    // ~8 resident waves per SIMD over 256 CUs; split planes only while the sample
    // grid alone is too small to fill the chip (the record is recomputed per chunk)
    int64_t by = (4096 + bx - 1) / bx;
    if (by > planes) by = planes;
    if (by > 65535) by = 65535;
    if (by < 1) by = 1;
    const int pc = (int)((planes + by - 1) / by);
    by = (planes + pc - 1) / pc;
    hipLaunchKernelGGL((k_homography<Tin, Tout, NEAREST>), dim3((unsigned)bx, (unsigned)by),
                       dim3(TF_THREADS), 0, s, static_cast<const Tin*>(src),
                       static_cast<Tout*>(dst), g, xs, ys, hm, planes, pc);
    return launch_status();
}

}  // namespace hg

extern "C" {

int hg_hex_homography(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t planes,
                      int64_t h, int64_t w, int64_t h1, int64_t w1, const double* xs,
                      const double* ys, const double* hinv, int interp, void* stream) {
    int st = hg::homog_check(planes, h, w, h1, w1);
    if (st) return st;
    if (!hinv) return HG_EINVAL;
    if (planes * h1 * w1 == 0) return HG_OK;
    if (!dst || !xs || !ys || (h * w > 0 && !src)) return HG_EINVAL;
    const hg::Geom g = hg::homog_geom(h, w, h1, w1);
    hg::Homog hm;
    for (int k = 0; k < 6; ++k) hm.m[k] = hinv[k];
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (interp == HG_NEAREST) {
        if (src_dtype != dst_dtype) return HG_EDTYPE;
        switch (hg::dtype_size(src_dtype)) {
        case 1: return hg::launch_homog<uint8_t, uint8_t, true>(src, dst, g, xs, ys, hm, planes, s);
        case 2: return hg::launch_homog<uint16_t, uint16_t, true>(src, dst, g, xs, ys, hm, planes, s);
        case 4: return hg::launch_homog<uint32_t, uint32_t, true>(src, dst, g, xs, ys, hm, planes, s);
        case 8: return hg::launch_homog<uint64_t, uint64_t, true>(src, dst, g, xs, ys, hm, planes, s);
        default: return HG_EDTYPE;
        }
    }
    if (interp != HG_LINEAR) return HG_EINVAL;
    HG_DISPATCH_IN(src_dtype, TIN, HG_DISPATCH_FLOAT_OUT(dst_dtype, TOUT, {
        return hg::launch_homog<TIN, TOUT, false>(src, dst, g, xs, ys, hm, planes, s);
    }));
    return HG_EDTYPE;
}

int hg_hex_homography_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, const double* xs,
                           const double* ys, const double* hinv, int32_t* imaps, double* fmaps,
                           void* stream) {
    int st = hg::homog_check(1, h, w, h1, w1);
    if (st) return st;
    if (!hinv) return HG_EINVAL;
    const int64_t n = h1 * w1;
    if (n == 0) return HG_OK;
    if ((!imaps && !fmaps) || !xs || !ys) return HG_EINVAL;
    hg::Homog hm;
    for (int k = 0; k < 6; ++k) hm.m[k] = hinv[k];
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(hg::k_homography_maps, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       hg::homog_geom(h, w, h1, w1), xs, ys, hm, imaps, fmaps);
    return hg::launch_status();
}

}  // extern "C"
