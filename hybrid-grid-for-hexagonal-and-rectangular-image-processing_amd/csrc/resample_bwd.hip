// resample_bwd.hip — gradients of the three resamplers.
//
// The reference's torch twin gets them from autograd through its fancy-index gathers
// and blends (geometry_torch.py:290-358); the NumPy path has none.  Each output
// sample of rect->hex (geometry_np.py:358-519), hex->rect (:191-356) or hexresize
// (:520-681) is a weighted sum of at most four (bilinear) or three (triangle) source
// samples with lattice-only weights, so d source is the transpose: every output
// sample scatters gy * weight onto its source taps.  The lattice is recomputed per
// output sample in fp64 exactly as the forward does (lattice.h), once per workgroup
// and reused for a chunk of planes; the scatter uses float atomics into a zeroed
// fp32 / fp64 accumulation raster (overlapping footprints: several outputs share a
// source sample).
#include <algorithm>
#include <climits>

#include "common.h"
#include "lattice.h"

namespace hg {

constexpr int RB_THREADS = 256;

// source taps and weights of output sample (a, b): n taps, flat source index and weight
template <int OP>
__device__ __forceinline__ int bwd_taps(const Geom& g, int64_t a, int64_t b, int interp,
                                        int64_t* idx, double* wt) {
    int n = 0;
    if constexpr (OP == HG_OP_RECT_TO_HEX) {
        const R2HSample s = r2h_sample(g, a, b);
        const int64_t ii[4] = {s.i_n, s.i_n, s.i_n + 1, s.i_n + 1};
        const int64_t jj[4] = {s.j_n, s.j_n + 1, s.j_n, s.j_n + 1};
        if (interp == HG_NEAREST) {                       // geometry_np.py:498-512
            if ((s.valid >> s.argmin) & 1) {
                idx[0] = (s.i_n + (s.argmin >> 1)) * g.w + s.j_n + (s.argmin & 1);   // ii / jj below
                wt[0] = 1.0;
                n = 1;
            }
        } else {                                          // :514-517
            const double fi = s.i_f, fj = s.j_f;
            const double w4[4] = {(1.0 - fj) * (1.0 - fi), fj * (1.0 - fi), (1.0 - fj) * fi, fj * fi};
            for (int k = 0; k < 4; ++k)
                if ((s.valid >> k) & 1) { idx[n] = ii[k] * g.w + jj[k]; wt[n] = w4[k]; ++n; }
        }
    } else {
        const TriSample s = tri_sample(g, a, b);
        if (interp == HG_NEAREST) {                       // geometry_torch.py:335-347
            if ((s.vk >> s.argmin) & 1) {
                idx[0] = tri_pick_r(s, s.argmin) * g.w + tri_pick_c(s, s.argmin);
                wt[0] = 1.0;
                n = 1;
            }
        } else {                                          // geometry_np.py:347-354
            const double w3[3] = {s.alpha, s.beta, s.gamma};
            for (int k = 0; k < 3; ++k)
                if ((s.vk >> k) & 1) { idx[n] = s.r[k] * g.w + s.c[k]; wt[n] = w3[k]; ++n; }
        }
    }
    return n;
}

// one thread per output sample; blockIdx.y = chunk of pc planes
template <int OP, typename A>
__global__ __launch_bounds__(RB_THREADS) void k_resample_bwd(const A* __restrict__ gy,
                                                             A* __restrict__ dx, Geom g,
                                                             int64_t planes, int interp, int pc) {
    const int64_t n_out = g.h1 * g.w1;
    const int64_t o = (int64_t)blockIdx.x * RB_THREADS + threadIdx.x;
    if (o >= n_out) return;
    const int64_t a = o / g.w1, b = o - a * g.w1;
    int64_t idx[4];
    double wt[4];
    const int n = bwd_taps<OP>(g, a, b, interp, idx, wt);
    A w[4];
    for (int k = 0; k < 4; ++k) w[k] = k < n ? (A)wt[k] : (A)0;
    const int64_t p0 = (int64_t)blockIdx.y * pc, p1 = std::min<int64_t>(p0 + pc, planes);
    const int64_t in_plane = g.h * g.w;
    for (int64_t p = p0; p < p1; ++p) {
        const A gv = gy[p * n_out + o];
        A* d = dx + p * in_plane;
        for (int k = 0; k < n; ++k) atomicAdd(&d[idx[k]], gv * w[k]);
    }
}

template <int OP, typename A>
static int resample_bwd_launch(const void* gy, void* dx, const Geom& g, int64_t planes,
                               int interp, hipStream_t st) {
    const hipError_t e = hipMemsetAsync(dx, 0, sizeof(A) * (size_t)(planes * g.h * g.w), st);
    if (e != hipSuccess) return hip_status(e);
    const int64_t n_out = g.h1 * g.w1;
    const int64_t bx = (n_out + RB_THREADS - 1) / RB_THREADS;
    if (bx > INT_MAX) return HG_ESHAPE;
    // enough workgroups to fill the chip; each reuses its lattice for pc planes
    int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(planes, (4096 + bx - 1) / bx));
    chunks = std::min<int64_t>(chunks, 65535);
    const int pc = (int)((planes + chunks - 1) / chunks);
    const dim3 grid((unsigned)bx, (unsigned)((planes + pc - 1) / pc));
    hipLaunchKernelGGL((k_resample_bwd<OP, A>), grid, dim3(RB_THREADS), 0, st, (const A*)gy,
                       (A*)dx, g, planes, interp, pc);
    return launch_status();
}

}  // namespace hg

extern "C" int hg_resample_backward(int op, const void* gy, void* dx, int acc_dtype,
                                    int64_t planes, int64_t h, int64_t w, int64_t h1, int64_t w1,
                                    int interp, void* stream) {
    using namespace hg;
    if (op < HG_OP_RECT_TO_HEX || op > HG_OP_HEXRESIZE) return HG_EINVAL;
    if (interp != HG_NEAREST && interp != HG_LINEAR) return HG_EINVAL;
    if (planes < 0 || h < 1 || w < 1 || h1 < 0 || w1 < 0) return HG_EINVAL;
    if (acc_dtype != HG_F32 && acc_dtype != HG_F64) return HG_EDTYPE;
    if (planes == 0) return HG_OK;
    if (!dx || (!gy && h1 * w1 > 0)) return HG_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (h1 * w1 == 0) {
        const size_t es = acc_dtype == HG_F64 ? 8 : 4;
        return hip_status(hipMemsetAsync(dx, 0, es * (size_t)(planes * h * w), st));
    }
    const Geom g = op == HG_OP_RECT_TO_HEX ? make_r2h(h, w, h1, w1)
                                           : make_tri(h, w, h1, w1, op == HG_OP_HEX_TO_RECT ? 0.75 : 0.5);
#define HG_RB(OPV)                                                                              \
    return acc_dtype == HG_F64 ? resample_bwd_launch<OPV, double>(gy, dx, g, planes, interp, st) \
                               : resample_bwd_launch<OPV, float>(gy, dx, g, planes, interp, st)
    if (op == HG_OP_RECT_TO_HEX) { HG_RB(HG_OP_RECT_TO_HEX); }
    if (op == HG_OP_HEX_TO_RECT) { HG_RB(HG_OP_HEX_TO_RECT); }
    HG_RB(HG_OP_HEXRESIZE);
#undef HG_RB
}
