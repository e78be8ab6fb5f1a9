// pool.hip — gfx950 kernels for hex pooling: HexPool2d, HexAdaptivePool2d and
// HexGlobalPool2d with the reference's NaN-aware max / min / average reductions
// (SURVEY.md §8f rank 4).
//
// Reference: /root/reference/HyGrid/HexFrames.py:255-343 (HexPool2d), :346-396
// (HexAdaptivePool2d), :397-410 (HexGlobalPool2d), :461-479 (max_pooling, min_pooling,
// average_pooling).  The reference gathers every window into a (b, c, hn, wn, kh*kw)
// tensor through an index array built on the host, after materialising the padded
// (and, in ceil mode, extended) input.  Here one pass reads the raster in place:
//
//   window (i, j) = rows  i*sh + [0, kh)
//                   cols  ((i % 2) * sw) / 2 + j*sw + [0, kw)        (:314-319, :382-386)
//
// of the virtual frame  P = pad(x, pad, mode, pad_value)  extended by ext_h rows at the
// bottom and ext_w columns at the right holding ext_value (the ceil-mode F.pad, :295-300);
// a frame coordinate is mapped onto x with the torch padding rules (hexconv_geom.h).
// max / min treat NaN as -inf / +inf and keep the first extreme in window order
// (torch.max / torch.min over the window); average sums the non-NaN values in window
// order, divides by their count and gives NaN for an empty count.
//
// Small windows: one thread per output, a wave stores 64 consecutive outputs.  Large
// windows (adaptive / global pooling): one 256-thread workgroup per output with a
// strided partial reduction and an LDS tree (first index kept on ties).
//
// Backward (the reference's autograd): max / min route gy to the selected element
// unless it is NaN or padding; average gives gy / count to every non-NaN element.
// Reflect / replicate / circular padding fold back onto x, so contributions are
// accumulated with float atomics into a zeroed fp32 / fp64 buffer.
//
// Bound: HBM (each input element is read once per window it belongs to; for kh <= sh,
// kw <= sw that is once) — pooling is a small share of a network's time.
#include <climits>

#include "common.h"
#include "hexconv_geom.h"

namespace hg {

constexpr int PL_THREADS = 256;
constexpr int64_t PL_LARGE = 512;   // window size from which a workgroup reduces one output

struct PoolGeom {
    int64_t planes, h, w;   // x: (planes, h, w)
    int64_t H0, W0;         // padded frame
    int64_t hn, wn;         // output
    int64_t ext_h, ext_w;
    double pad_value, ext_value;
    int pad, pad_mode, kh, kw, sh, sw, method;
};

template <typename T> struct pool_acc { using A = float; };
template <> struct pool_acc<double> { using A = double; };

// Source offset of frame coordinate (y, x): >= 0 into the plane, -1 constant padding,
// -2 ceil-mode extension.
__device__ __forceinline__ int64_t frame_src(const PoolGeom& g, int64_t y, int64_t x) {
    if (y >= g.H0 || x >= g.W0) return -2;
    const int64_t r = pad_map(y - g.pad, g.h, g.pad_mode);
    const int64_t c = pad_map(x - g.pad, g.w, g.pad_mode);
    if (r < 0 || c < 0) return -1;
    return r * g.w + c;
}

template <typename T, typename A>
__device__ __forceinline__ A frame_val(const PoolGeom& g, const T* __restrict__ sp, int64_t off) {
    if (off >= 0) return (A)sp[off];
    return off == -1 ? (A)(T)g.pad_value : (A)(T)g.ext_value;
}

// Window element k (row-major over kh x kw) of output (i, j) -> frame coordinate.
__device__ __forceinline__ void win_coord(const PoolGeom& g, int64_t i, int64_t j, int64_t k,
                                          int64_t* y, int64_t* x) {
    const int64_t dy = k / g.kw, dx = k - dy * g.kw;
    *y = i * g.sh + dy;
    *x = ((i & 1) * g.sw) / 2 + j * g.sw + dx;
}

// Running state of one reduction.  method 0 max, 1 min, 2 average.
template <typename A>
struct PoolState {
    A v;        // extreme (max/min) or sum (average)
    int64_t k;  // index of the extreme / count of non-NaN values
};

template <typename A>
__device__ __forceinline__ void pool_push(PoolState<A>& s, A v, int64_t k, int method) {
    const bool nan = v != v;
    if (method == 2) {
        if (!nan) { s.v += v; s.k += 1; }
        return;
    }
    const A inf = (A)INFINITY;
    const A u = nan ? (method == 0 ? -inf : inf) : v;
    if (s.k < 0 || (method == 0 ? u > s.v : u < s.v)) { s.v = u; s.k = k; }
}

template <typename A>
__device__ __forceinline__ PoolState<A> pool_init(int method) {
    PoolState<A> s;
    s.v = (A)0;
    s.k = method == 2 ? 0 : -1;
    return s;
}

// Merge two partial states; on equal extremes the smaller window index wins.
template <typename A>
__device__ __forceinline__ void pool_merge(PoolState<A>& s, const PoolState<A>& t, int method) {
    if (method == 2) { s.v += t.v; s.k += t.k; return; }
    if (t.k < 0) return;
    if (s.k < 0 || (method == 0 ? t.v > s.v : t.v < s.v) || (t.v == s.v && t.k < s.k)) s = t;
}

template <typename T, typename A>
__device__ __forceinline__ T pool_result(const PoolState<A>& s, int method) {
    if (method != 2) return (T)s.v;
    if (s.k == 0) return (T)NAN;
    // torch: the sum and the count are tensors of the input dtype, then divided
    return (T)((A)(T)s.v / (A)(T)(A)s.k);
}

template <typename T>
__global__ __launch_bounds__(PL_THREADS) void k_pool_small(const T* __restrict__ x,
                                                           T* __restrict__ y, PoolGeom g) {
    using A = typename pool_acc<T>::A;
    const int64_t per = g.hn * g.wn;
    const int64_t q = (int64_t)blockIdx.x * PL_THREADS + threadIdx.x;
    if (q >= g.planes * per) return;
    const int64_t p = q / per, r = q - p * per;
    const int64_t i = r / g.wn, j = r - i * g.wn;
    const T* sp = x + p * g.h * g.w;
    PoolState<A> s = pool_init<A>(g.method);
    const int64_t n = (int64_t)g.kh * g.kw;
    for (int64_t k = 0; k < n; ++k) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        pool_push(s, frame_val<T, A>(g, sp, frame_src(g, yy, xx)), k, g.method);
    }
    y[q] = pool_result<T>(s, g.method);
}

template <typename T>
__global__ __launch_bounds__(PL_THREADS) void k_pool_large(const T* __restrict__ x,
                                                           T* __restrict__ y, PoolGeom g) {
    using A = double;   // long windows: fp64 partial sums
    __shared__ A sv[PL_THREADS];
    __shared__ int64_t sk[PL_THREADS];
    const int64_t per = g.hn * g.wn;
    const int64_t q = blockIdx.x;
    const int64_t p = q / per, r = q - p * per;
    const int64_t i = r / g.wn, j = r - i * g.wn;
    const T* sp = x + p * g.h * g.w;
    const int64_t n = (int64_t)g.kh * g.kw;
    // lanes stride the window (coalesced rows); ties resolve to the smaller index in
    // pool_merge, so the first extreme in window order still wins
    PoolState<A> s = pool_init<A>(g.method);
    for (int64_t k = threadIdx.x; k < n; k += PL_THREADS) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        pool_push(s, frame_val<T, A>(g, sp, frame_src(g, yy, xx)), k, g.method);
    }
    sv[threadIdx.x] = s.v;
    sk[threadIdx.x] = s.k;
    __syncthreads();
    for (int o = PL_THREADS / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            PoolState<A> a{sv[threadIdx.x], sk[threadIdx.x]};
            const PoolState<A> b{sv[threadIdx.x + o], sk[threadIdx.x + o]};
            pool_merge(a, b, g.method);
            sv[threadIdx.x] = a.v;
            sk[threadIdx.x] = a.k;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) y[q] = pool_result<T>(PoolState<A>{sv[0], sk[0]}, g.method);
}

// ---- backward ----------------------------------------------------------------------
template <typename G>
__device__ __forceinline__ void atomic_add_g(G* p, G v) { atomicAdd(p, v); }

// Selected element of a max / min window (recomputed from x), scattered; or gy / count
// to every non-NaN element of an average window.
template <typename T, typename G>
__global__ __launch_bounds__(PL_THREADS) void k_pool_bwd_small(const T* __restrict__ x,
                                                               const G* __restrict__ gy,
                                                               G* __restrict__ dx, PoolGeom g) {
    using A = typename pool_acc<T>::A;
    const int64_t per = g.hn * g.wn;
    const int64_t q = (int64_t)blockIdx.x * PL_THREADS + threadIdx.x;
    if (q >= g.planes * per) return;
    const int64_t p = q / per, r = q - p * per;
    const int64_t i = r / g.wn, j = r - i * g.wn;
    const T* sp = x + p * g.h * g.w;
    G* dp = dx + p * g.h * g.w;
    const int64_t n = (int64_t)g.kh * g.kw;
    PoolState<A> s = pool_init<A>(g.method);
    for (int64_t k = 0; k < n; ++k) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        pool_push(s, frame_val<T, A>(g, sp, frame_src(g, yy, xx)), k, g.method);
    }
    const G gq = gy[q];
    if (g.method != 2) {
        if (s.k < 0) return;
        int64_t yy, xx;
        win_coord(g, i, j, s.k, &yy, &xx);
        const int64_t off = frame_src(g, yy, xx);
        if (off < 0) return;
        const A v = (A)sp[off];
        if (v != v) return;   // masked_fill backward: no gradient to a NaN element
        atomic_add_g(dp + off, gq);
        return;
    }
    if (s.k == 0) return;
    // torch: d sum = gy / count in the input dtype
    const G gs = (G)(T)((A)(T)(A)gq / (A)(T)(A)s.k);
    for (int64_t k = 0; k < n; ++k) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        const int64_t off = frame_src(g, yy, xx);
        if (off < 0) continue;
        const A v = (A)sp[off];
        if (v != v) continue;
        atomic_add_g(dp + off, gs);
    }
}

template <typename T, typename G>
__global__ __launch_bounds__(PL_THREADS) void k_pool_bwd_large(const T* __restrict__ x,
                                                               const G* __restrict__ gy,
                                                               G* __restrict__ dx, PoolGeom g) {
    using A = double;   // long windows: fp64 partial sums
    __shared__ A sv[PL_THREADS];
    __shared__ int64_t sk[PL_THREADS];
    const int64_t per = g.hn * g.wn;
    const int64_t q = blockIdx.x;
    const int64_t p = q / per, r = q - p * per;
    const int64_t i = r / g.wn, j = r - i * g.wn;
    const T* sp = x + p * g.h * g.w;
    G* dp = dx + p * g.h * g.w;
    const int64_t n = (int64_t)g.kh * g.kw;
    PoolState<A> s = pool_init<A>(g.method);
    for (int64_t k = threadIdx.x; k < n; k += PL_THREADS) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        pool_push(s, frame_val<T, A>(g, sp, frame_src(g, yy, xx)), k, g.method);
    }
    sv[threadIdx.x] = s.v;
    sk[threadIdx.x] = s.k;
    __syncthreads();
    for (int o = PL_THREADS / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            PoolState<A> a{sv[threadIdx.x], sk[threadIdx.x]};
            const PoolState<A> b{sv[threadIdx.x + o], sk[threadIdx.x + o]};
            pool_merge(a, b, g.method);
            sv[threadIdx.x] = a.v;
            sk[threadIdx.x] = a.k;
        }
        __syncthreads();
    }
    const PoolState<A> tot{sv[0], sk[0]};
    const G gq = gy[q];
    if (g.method != 2) {
        if (threadIdx.x != 0 || tot.k < 0) return;
        int64_t yy, xx;
        win_coord(g, i, j, tot.k, &yy, &xx);
        const int64_t off = frame_src(g, yy, xx);
        if (off < 0) return;
        const A v = (A)sp[off];
        if (v != v) return;
        atomic_add_g(dp + off, gq);
        return;
    }
    if (tot.k == 0) return;
    const G gs = (G)(T)((A)(T)(A)gq / (A)(T)(A)tot.k);
    for (int64_t k = threadIdx.x; k < n; k += PL_THREADS) {
        int64_t yy, xx;
        win_coord(g, i, j, k, &yy, &xx);
        const int64_t off = frame_src(g, yy, xx);
        if (off < 0) continue;
        const A v = (A)sp[off];
        if (v != v) continue;
        atomic_add_g(dp + off, gs);
    }
}

// ---- host --------------------------------------------------------------------------
static int pool_setup(PoolGeom* g, int method, int64_t planes, int64_t h, int64_t w, int pad,
                      int pad_mode, double pad_value, int64_t ext_h, int64_t ext_w,
                      double ext_value, int kh, int kw, int sh, int sw, int64_t hn, int64_t wn) {
    if (method < 0 || method > 2 || planes < 0 || h < 0 || w < 0 || pad < 0 || ext_h < 0 ||
        ext_w < 0 || kh < 0 || kw < 0 || sh < 1 || sw < 1 || hn < 0 || wn < 0)
        return HG_EINVAL;
    if (pad_mode < HG_PAD_CONSTANT || pad_mode > HG_PAD_CIRCULAR) return HG_EINVAL;
    if (pad > 0 && pad_mode != HG_PAD_CONSTANT && (h == 0 || w == 0)) return HG_ESHAPE;
    if (pad_mode == HG_PAD_REFLECT && pad > 0 && (pad >= h || pad >= w)) return HG_ESHAPE;
    if (pad_mode == HG_PAD_CIRCULAR && (pad > h || pad > w)) return HG_ESHAPE;
    g->planes = planes; g->h = h; g->w = w;
    g->H0 = h + 2 * (int64_t)pad; g->W0 = w + 2 * (int64_t)pad;
    g->hn = hn; g->wn = wn; g->ext_h = ext_h; g->ext_w = ext_w;
    g->pad_value = pad_value; g->ext_value = ext_value;
    g->pad = pad; g->pad_mode = pad_mode; g->kh = kh; g->kw = kw; g->sh = sh; g->sw = sw;
    g->method = method;
    if (hn == 0 || wn == 0) return HG_OK;
    if ((int64_t)kh * kw == 0 && method != 2) return HG_ESHAPE;   // max over an empty window
    // every window must lie inside the (extended) frame: the reference's gather would
    // raise IndexError, and the kernels must never read outside x
    const int64_t H = g->H0 + ext_h, W = g->W0 + ext_w;
    const int64_t shift = hn >= 2 ? sw / 2 : 0;
    if ((hn - 1) * sh + kh > H || (wn - 1) * sw + shift + kw > W) return HG_ESHAPE;
    if (planes > 0 && (hn * wn > (int64_t)INT_MAX || planes * hn * wn > (int64_t)INT_MAX * 64))
        return HG_ESHAPE;
    return HG_OK;
}

template <typename T>
static int launch_pool(const void* x, void* y, const PoolGeom& g, hipStream_t s) {
    const int64_t nout = g.planes * g.hn * g.wn;
    if (nout == 0) return HG_OK;
    if ((int64_t)g.kh * g.kw >= PL_LARGE) {
        hipLaunchKernelGGL(k_pool_large<T>, dim3((unsigned)nout), dim3(PL_THREADS), 0, s,
                           static_cast<const T*>(x), static_cast<T*>(y), g);
    } else {
        hipLaunchKernelGGL(k_pool_small<T>, dim3((unsigned)((nout + PL_THREADS - 1) / PL_THREADS)),
                           dim3(PL_THREADS), 0, s, static_cast<const T*>(x), static_cast<T*>(y), g);
    }
    return launch_status();
}

template <typename T, typename G>
static int launch_pool_bwd(const void* x, const void* gy, void* dx, const PoolGeom& g,
                           hipStream_t s) {
    const int64_t nout = g.planes * g.hn * g.wn;
    if (nout == 0) return HG_OK;
    if ((int64_t)g.kh * g.kw >= PL_LARGE) {
        hipLaunchKernelGGL((k_pool_bwd_large<T, G>), dim3((unsigned)nout), dim3(PL_THREADS), 0, s,
                           static_cast<const T*>(x), static_cast<const G*>(gy),
                           static_cast<G*>(dx), g);
    } else {
        hipLaunchKernelGGL((k_pool_bwd_small<T, G>),
                           dim3((unsigned)((nout + PL_THREADS - 1) / PL_THREADS)), dim3(PL_THREADS),
                           0, s, static_cast<const T*>(x), static_cast<const G*>(gy),
                           static_cast<G*>(dx), g);
    }
    return launch_status();
}

}  // namespace hg

extern "C" {

int hg_hex_pool2d(const void* x, void* y, int dtype, int method, int64_t planes, int64_t h,
                  int64_t w, int pad, int pad_mode, double pad_value, int64_t ext_h,
                  int64_t ext_w, double ext_value, int kh, int kw, int sh, int sw, int64_t hn,
                  int64_t wn, void* stream) {
    hg::PoolGeom g;
    int st = hg::pool_setup(&g, method, planes, h, w, pad, pad_mode, pad_value, ext_h, ext_w,
                            ext_value, kh, kw, sh, sw, hn, wn);
    if (st) return st;
    if (planes * hn * wn == 0) return HG_OK;
    if (!y || (h * w > 0 && !x)) return HG_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (dtype) {
    case HG_F16: return hg::launch_pool<_Float16>(x, y, g, s);
    case HG_BF16: return hg::launch_pool<__bf16>(x, y, g, s);
    case HG_F32: return hg::launch_pool<float>(x, y, g, s);
    case HG_F64: return hg::launch_pool<double>(x, y, g, s);
    default: return HG_EDTYPE;
    }
}

int hg_hex_pool2d_backward(const void* x, const void* gy, void* dx, int dtype, int grad_dtype,
                           int method, int64_t planes, int64_t h, int64_t w, int pad,
                           int pad_mode, double pad_value, int64_t ext_h, int64_t ext_w,
                           double ext_value, int kh, int kw, int sh, int sw, int64_t hn,
                           int64_t wn, void* stream) {
    hg::PoolGeom g;
    int st = hg::pool_setup(&g, method, planes, h, w, pad, pad_mode, pad_value, ext_h, ext_w,
                            ext_value, kh, kw, sh, sw, hn, wn);
    if (st) return st;
    if (grad_dtype != HG_F32 && grad_dtype != HG_F64) return HG_EDTYPE;
    if (planes * h * w == 0) return HG_OK;
    if (!dx || !x || (planes * hn * wn > 0 && !gy)) return HG_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    st = hg::hip_status(hipMemsetAsync(dx, 0, (size_t)(planes * h * w) * hg::dtype_size(grad_dtype),
                                       s));
    if (st) return st;
    if (grad_dtype == HG_F64) {
        switch (dtype) {
        case HG_F16: return hg::launch_pool_bwd<_Float16, double>(x, gy, dx, g, s);
        case HG_BF16: return hg::launch_pool_bwd<__bf16, double>(x, gy, dx, g, s);
        case HG_F32: return hg::launch_pool_bwd<float, double>(x, gy, dx, g, s);
        case HG_F64: return hg::launch_pool_bwd<double, double>(x, gy, dx, g, s);
        default: return HG_EDTYPE;
        }
    }
    switch (dtype) {
    case HG_F16: return hg::launch_pool_bwd<_Float16, float>(x, gy, dx, g, s);
    case HG_BF16: return hg::launch_pool_bwd<__bf16, float>(x, gy, dx, g, s);
    case HG_F32: return hg::launch_pool_bwd<float, float>(x, gy, dx, g, s);
    case HG_F64: return hg::launch_pool_bwd<double, float>(x, gy, dx, g, s);
    default: return HG_EDTYPE;
    }
}

}  // extern "C"
