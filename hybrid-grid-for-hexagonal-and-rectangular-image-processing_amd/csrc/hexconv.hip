// hexconv.hip — gfx950 HexConv2d forward as a direct hex stencil.
//
// The reference (HexFrames.py:96-169) pads, expands the image to the
// double-width "type1" raster (heximage_to_type1, :417-445), runs two strided
// dense 3x5 F.conv2d (8 of 15 taps zero) and interleaves rows: about 7x the
// compulsory traffic.  Here the type1 raster is never built.  With P the padded
// image (H' = h+2p, W' = w+2p), o' = (off+p)%2 and L(y) = ((y&1)+o')&1, tap t =
// (kernel row ii, cell m) of output (ro, q) reads
//     P[s*ro + ii*d][s*q + dk_t(ro&1)],   dk_t(par) = (1 + par*s + t*d + 2dm - L(par*s+ii*d)) >> 1
// (t = |ii-r+1|), and a column k >= W' is the type1 raster's structural zero.
// See oracle/hg_oracle.c for the derivation against the reference lines.
//
// Workgroup = 256 threads, output tile 16 rows x 128 cols, thread t owns column
// t%128 and 8 consecutive rows.  Per image and group, the tile's P footprint of
// a chunk of input channels is staged into LDS (fp32/fp64, pad rules applied
// once there), then each thread accumulates OCB output channels for its 8
// samples; kernel weights are wave-uniform (scalar loads).
#include <algorithm>
#include <climits>

#include "common.h"
#include "hexconv_geom.h"

namespace hg {

constexpr int CV_THREADS = 256;
constexpr int CV_TC = 128;
constexpr int CV_RPT = 8;
constexpr int CV_TR = 16;
constexpr int CV_MAXK = 128;          // taps: 3r^2-3r+1 <= 127 (r <= 7)
constexpr int CV_LDS_BUDGET = 56 * 1024;

struct ConvGeom {
    int64_t B, C, O, h, w, ho, wo;
    int r, s, p, d, groups, off, pad_mode;
    int K, cg, og;
    int ntx;          // tiles along output columns
    int bc;           // images per workgroup
    int cib;          // input channels staged per pass
    int nPr, pitch;   // LDS footprint rows / pitch (elements)
    int mink;         // min column tap offset over both parities
    double pad_value;
    Epilogue epi;
};

template <typename Tin, typename Tout, typename A, int OCB, int KFIX>
__global__ __launch_bounds__(CV_THREADS) void k_hexconv(const Tin* __restrict__ x,
                                                        const A* __restrict__ kern,
                                                        const A* __restrict__ bias,
                                                        Tout* __restrict__ y, ConvGeom G) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* tdy = reinterpret_cast<int*>(smem);
    int* tdk = tdy + CV_MAXK;                 // [2][CV_MAXK]
    A* tile = reinterpret_cast<A*>(smem + 3 * CV_MAXK * sizeof(int));

    const int K = KFIX ? KFIX : G.K;
    const int tid = threadIdx.x;
    const int op = (G.off + G.p) & 1;
    for (int t = tid; t < K; t += CV_THREADS) {
        int dy, d0, d1;
        tap_geom(G.r, G.s, G.d, op, t, &dy, &d0, &d1);
        tdy[t] = dy;
        tdk[t] = d0 - G.mink;
        tdk[CV_MAXK + t] = d1 - G.mink;
    }

    unsigned bx, by;
    xcd_swizzle2(&bx, &by);
    const int tx = (int)bx % G.ntx, ty = (int)bx / G.ntx;
    const int64_t r0 = (int64_t)ty * CV_TR, q0 = (int64_t)tx * CV_TC;
    const int lq = tid & (CV_TC - 1);
    const int lr0 = (tid / CV_TC) * CV_RPT;
    const int64_t q = q0 + lq;
    const int64_t Hp = G.h + 2 * G.p, Wp = G.w + 2 * G.p;
    const int64_t pr0 = (int64_t)G.s * r0;                 // first staged P row
    const int64_t pc0 = (int64_t)G.s * q0 + G.mink;        // first staged P col
    const int chan = G.nPr * G.pitch;
    const int64_t b0 = (int64_t)by * G.bc;
    const int64_t b1 = std::min<int64_t>(b0 + G.bc, G.B);
    const int64_t in_plane = G.h * G.w, out_plane = G.ho * G.wo;
    const A padv = (A)G.pad_value;
    __syncthreads();

    for (int64_t b = b0; b < b1; ++b) {
        for (int g = 0; g < G.groups; ++g) {
            for (int oc0 = 0; oc0 < G.og; oc0 += OCB) {
                A acc[CV_RPT][OCB];
#pragma unroll
                for (int j = 0; j < OCB; ++j) {
                    const int o = g * G.og + oc0 + j;
                    const A bv = (bias && oc0 + j < G.og) ? bias[o] : (A)0;
#pragma unroll
                    for (int k = 0; k < CV_RPT; ++k) acc[k][j] = bv;
                }
                for (int ci0 = 0; ci0 < G.cg; ci0 += G.cib) {
                    const int nci = std::min(G.cib, G.cg - ci0);
                    __syncthreads();
                    // stage P footprint of nci channels
                    const int per = G.nPr * G.pitch;
                    for (int e = tid; e < nci * per; e += CV_THREADS) {
                        const int cc = e / per;
                        const int rem = e - cc * per;
                        const int rr = rem / G.pitch;
                        const int kk = rem - rr * G.pitch;
                        const int64_t py = pr0 + rr, pk = pc0 + kk;
                        A v = (A)0;
                        if (py < Hp && pk >= 0 && pk < Wp) {
                            const int64_t yi = pad_map(py - G.p, G.h, G.pad_mode);
                            const int64_t xi = pad_map(pk - G.p, G.w, G.pad_mode);
                            if (yi < 0 || xi < 0) v = padv;
                            else {
                                const Tin* xp = x + (b * G.C + g * G.cg + ci0 + cc) * in_plane;
                                v = to_acc<A>(xp[yi * G.w + xi]);
                            }
                        }
                        tile[e] = v;
                    }
                    __syncthreads();
                    for (int cc = 0; cc < nci; ++cc) {
                        const A* tc = tile + cc * chan;
                        const A* kc = kern + ((int64_t)(g * G.og + oc0) * G.cg + ci0 + cc) * K;
#pragma unroll 7
                        for (int t = 0; t < K; ++t) {
                            A wv[OCB];
#pragma unroll
                            for (int j = 0; j < OCB; ++j)
                                wv[j] = (oc0 + j < G.og) ? kc[(int64_t)j * G.cg * K + t] : (A)0;
                            const int dy = tdy[t];
                            const int dke = tdk[t], dko = tdk[CV_MAXK + t];
#pragma unroll
                            for (int k = 0; k < CV_RPT; ++k) {
                                const int lr = lr0 + k;
                                const int dk = (k & 1) ? dko : dke;   // r0, lr0 even
                                const A v = tc[(G.s * lr + dy) * G.pitch + G.s * lq + dk];
#pragma unroll
                                for (int j = 0; j < OCB; ++j) acc[k][j] += wv[j] * v;
                            }
                        }
                    }
                }
                if (q < G.wo) {
#pragma unroll
                    for (int j = 0; j < OCB; ++j) {
                        if (oc0 + j >= G.og) continue;
                        Tout* yp = y + (b * G.O + g * G.og + oc0 + j) * out_plane;
#pragma unroll
                        for (int k = 0; k < CV_RPT; ++k) {
                            const int64_t ro = r0 + lr0 + k;
                            A v = acc[k][j];
                            if (G.epi.on) v = epi_apply(v, g * G.og + oc0 + j, G.epi);
                            if (ro < G.ho) yp[ro * G.wo + q] = from_acc<Tout>(v);
                        }
                    }
                }
            }
        }
    }
}

// Direct-gather fallback (footprint larger than the LDS budget: large radius or
// stride).  One thread per output sample, taps read straight from global memory.
template <typename Tin, typename Tout, typename A>
__global__ __launch_bounds__(256) void k_hexconv_direct(const Tin* __restrict__ x,
                                                        const A* __restrict__ kern,
                                                        const A* __restrict__ bias,
                                                        Tout* __restrict__ y, ConvGeom G) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = G.B * G.O * G.ho * G.wo;
    if (idx >= total) return;
    const int64_t q = idx % G.wo;
    const int64_t ro = (idx / G.wo) % G.ho;
    const int64_t o = (idx / (G.wo * G.ho)) % G.O;
    const int64_t b = idx / (G.wo * G.ho * G.O);
    const int g = (int)(o / G.og);
    const int op = (G.off + G.p) & 1;
    const int64_t Wp = G.w + 2 * G.p;
    A acc = bias ? bias[o] : (A)0;
    for (int t = 0; t < G.K; ++t) {
        int dy, d0, d1;
        tap_geom(G.r, G.s, G.d, op, t, &dy, &d0, &d1);
        const int64_t py = (int64_t)G.s * ro + dy;
        const int64_t pk = (int64_t)G.s * q + ((ro & 1) ? d1 : d0);
        if (pk >= Wp) continue;                          // type1 structural zero
        const int64_t yi = pad_map(py - G.p, G.h, G.pad_mode);
        const int64_t xi = pad_map(pk - G.p, G.w, G.pad_mode);
        for (int ci = 0; ci < G.cg; ++ci) {
            const A wv = kern[(o * G.cg + ci) * G.K + t];
            A v;
            if (yi < 0 || xi < 0) v = (A)G.pad_value;
            else v = to_acc<A>(x[((b * G.C + g * G.cg + ci) * G.h + yi) * G.w + xi]);
            acc += wv * v;
        }
    }
    if (G.epi.on) acc = epi_apply(acc, (int)o, G.epi);
    y[idx] = from_acc<Tout>(acc);
}

template <typename Tin, typename Tout, typename A, int OCB, int KFIX>
static int launch_conv(const void* x, const void* k, const void* b, void* y, ConvGeom G,
                       hipStream_t st) {
    const int64_t nty = (G.ho + CV_TR - 1) / CV_TR;
    const int64_t tiles = (int64_t)G.ntx * nty;
    int64_t nchunk = std::max<int64_t>(1, std::min<int64_t>((2048 + tiles - 1) / tiles, G.B));
    nchunk = std::min<int64_t>(nchunk, 65535);
    G.bc = (int)((G.B + nchunk - 1) / nchunk);
    const size_t shmem = 3 * CV_MAXK * sizeof(int) + (size_t)G.cib * G.nPr * G.pitch * sizeof(A);
    dim3 grid((unsigned)tiles, (unsigned)((G.B + G.bc - 1) / G.bc));
    hipLaunchKernelGGL((k_hexconv<Tin, Tout, A, OCB, KFIX>), grid, dim3(CV_THREADS), shmem, st,
                       (const Tin*)x, (const A*)k, (const A*)b, (Tout*)y, G);
    return launch_status();
}

template <typename Tin, typename Tout, typename A>
static int conv_dispatch(const void* x, const void* k, const void* b, void* y,
                         const ConvGeom& G, hipStream_t st) {
    if (G.cib == 0) {
        const int64_t total = G.B * G.O * G.ho * G.wo;
        hipLaunchKernelGGL((k_hexconv_direct<Tin, Tout, A>), dim3((unsigned)((total + 255) / 256)),
                           dim3(256), 0, st, (const Tin*)x, (const A*)k, (const A*)b, (Tout*)y, G);
        return launch_status();
    }
    const bool k7 = G.K == 7;
    if (G.og % 4 == 0 || G.og > 4) {
        return k7 ? launch_conv<Tin, Tout, A, 4, 7>(x, k, b, y, G, st)
                  : launch_conv<Tin, Tout, A, 4, 0>(x, k, b, y, G, st);
    }
    if (G.og == 3)
        return k7 ? launch_conv<Tin, Tout, A, 3, 7>(x, k, b, y, G, st)
                  : launch_conv<Tin, Tout, A, 3, 0>(x, k, b, y, G, st);
    if (G.og == 2)
        return k7 ? launch_conv<Tin, Tout, A, 2, 7>(x, k, b, y, G, st)
                  : launch_conv<Tin, Tout, A, 2, 0>(x, k, b, y, G, st);
    return k7 ? launch_conv<Tin, Tout, A, 1, 7>(x, k, b, y, G, st)
              : launch_conv<Tin, Tout, A, 1, 0>(x, k, b, y, G, st);
}

int launch_conv_stream(const void* x, const float* k, const float* b, void* y, int x_dtype,
                       int y_dtype, int64_t B, int C, int O, int64_t h, int64_t w, int p,
                       int groups, int off, double pad_value, const Epilogue& epi,
                       hipStream_t st);   // conv_stream.hip
int conv_mfma_try(const void* x, const float* k, const float* b, void* y, int x_dtype,
                  int y_dtype, int64_t B, int64_t C, int64_t O, int64_t h, int64_t w, int radius,
                  int stride, int padding, int dilation, int groups, int off, int pad_mode,
                  double pad_value, const Epilogue& epi, hipStream_t st);   // conv_mfma.hip

}  // namespace hg

extern "C" {

int hg_hexconv2d_out_shape(int64_t h, int64_t w, int radius, int stride, int padding,
                           int dilation, int64_t* ho, int64_t* wo) {
    if (!ho || !wo) return HG_EINVAL;
    return hg::conv_out_shape(h, w, radius, stride, padding, dilation, ho, wo);
}

int hg_hexconv2d(const void* x, const void* kernel, const void* bias, void* y, int x_dtype,
                 int w_dtype, int y_dtype, int64_t batch, int64_t in_channels,
                 int64_t out_channels, int64_t h, int64_t w, int radius, int stride,
                 int padding, int dilation, int groups, int even_odd_offset, int pad_mode,
                 double pad_value, void* stream) {
    return hg_hexconv2d_epilogue(x, kernel, bias, y, x_dtype, w_dtype, y_dtype, batch,
                                 in_channels, out_channels, h, w, radius, stride, padding,
                                 dilation, groups, even_odd_offset, pad_mode, pad_value, nullptr,
                                 nullptr, HG_ACT_NONE, 0.0, stream);
}

int hg_hexconv2d_epilogue(const void* x, const void* kernel, const void* bias, void* y,
                          int x_dtype, int w_dtype, int y_dtype, int64_t batch,
                          int64_t in_channels, int64_t out_channels, int64_t h, int64_t w,
                          int radius, int stride, int padding, int dilation, int groups,
                          int even_odd_offset, int pad_mode, double pad_value,
                          const void* scale, const void* shift, int act, double act_param,
                          void* stream) {
    using namespace hg;
    if (act < HG_ACT_NONE || act > HG_ACT_TANH) return HG_EINVAL;
    Epilogue epi;
    epi.scale = scale; epi.shift = shift; epi.act = act; epi.slope = act_param;
    epi.on = (scale || shift || act != HG_ACT_NONE) ? 1 : 0;
    ConvGeom G;
    int st = conv_out_shape(h, w, radius, stride, padding, dilation, &G.ho, &G.wo);
    if (st) return st;
    st = conv_check_args(batch, in_channels, out_channels, h, w, groups, padding, pad_mode);
    if (st) return st;
    G.K = 3 * radius * radius - 3 * radius + 1;
    if (G.K > CV_MAXK) return HG_EUNSUP;
    if (batch == 0 || G.ho == 0 || G.wo == 0) return HG_OK;
    if (!x || !kernel || !y) return HG_EINVAL;
    if (w_dtype != HG_F32 && w_dtype != HG_F64) return HG_EDTYPE;
    if (!dtype_is_float(y_dtype)) return HG_EDTYPE;
    if (h * w >= INT_MAX / 2 || G.ho * G.wo >= INT_MAX / 2) return HG_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (radius == 2 && stride == 1 && dilation == 1 && pad_mode == HG_PAD_CONSTANT &&
        w_dtype == HG_F32 && in_channels <= 3 && out_channels <= 3) {
        // register-streaming fast path (conv_stream.hip); EUNSUP -> generic kernel
        st = launch_conv_stream(x, (const float*)kernel, (const float*)bias, y, x_dtype, y_dtype,
                                batch, (int)in_channels, (int)out_channels, h, w, padding,
                                groups, even_odd_offset & 1, pad_value, epi, s);
        if (st != HG_EUNSUP) return st;
    }
    if (w_dtype == HG_F32) {   // wide channels: implicit GEMM on the f32 matrix cores
        st = conv_mfma_try(x, (const float*)kernel, (const float*)bias, y, x_dtype, y_dtype,
                           batch, in_channels, out_channels, h, w, radius, stride, padding,
                           dilation, groups, even_odd_offset & 1, pad_mode, pad_value, epi, s);
        if (st != HG_EUNSUP) return st;
    }
    G.B = batch; G.C = in_channels; G.O = out_channels; G.h = h; G.w = w;
    G.r = radius; G.s = stride; G.p = padding; G.d = dilation; G.groups = groups;
    G.off = even_odd_offset & 1; G.pad_mode = pad_mode; G.pad_value = pad_value;
    G.epi = epi;
    G.cg = (int)(in_channels / groups);
    G.og = (int)(out_channels / groups);
    G.ntx = (int)((G.wo + CV_TC - 1) / CV_TC);
    // column span of the taps over both row parities
    const int op = (G.off + G.p) & 1;
    int mink = INT_MAX, maxk = INT_MIN, maxdy = 0;
    for (int t = 0; t < G.K; ++t) {
        int dy, d0, d1;
        tap_geom(radius, stride, dilation, op, t, &dy, &d0, &d1);
        mink = std::min(mink, std::min(d0, d1));
        maxk = std::max(maxk, std::max(d0, d1));
        maxdy = std::max(maxdy, dy);
    }
    G.mink = mink;
    G.nPr = stride * (CV_TR - 1) + maxdy + 1;
    G.pitch = stride * (CV_TC - 1) + (maxk - mink) + 1;
    G.pitch = (G.pitch + 3) & ~3;
    const size_t esz = w_dtype == HG_F64 ? 8 : 4;
    const size_t per = (size_t)G.nPr * G.pitch * esz;
    if (per + 3 * CV_MAXK * sizeof(int) > (size_t)CV_LDS_BUDGET)
        G.cib = 0;   // footprint too large for LDS: direct-gather kernel
    else
        G.cib = (int)std::min<size_t>((size_t)G.cg,
                                      (CV_LDS_BUDGET - 3 * CV_MAXK * sizeof(int)) / per);
    G.bc = 1;
    if (w_dtype == HG_F64) {
        HG_DISPATCH_IN(x_dtype, TIN, HG_DISPATCH_FLOAT_OUT(y_dtype, TOUT, {
            return conv_dispatch<TIN, TOUT, double>(x, kernel, bias, y, G, s);
        }));
    } else {
        HG_DISPATCH_IN(x_dtype, TIN, HG_DISPATCH_FLOAT_OUT(y_dtype, TOUT, {
            return conv_dispatch<TIN, TOUT, float>(x, kernel, bias, y, G, s);
        }));
    }
    return HG_EDTYPE;
}

}  // extern "C"
