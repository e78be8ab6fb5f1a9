// hexconv_bwd.hip — HexConv2d backward on gfx950.
//
// The reference gets its gradients from torch autograd through pad ->
// heximage_to_type1 -> two strided F.conv2d -> row interleave
// (HexFrames.py:96-169, :417-445).  Here they are the exact adjoint of the
// forward index map (hexconv_geom.h; oracle/hg_oracle.c or_hexconv2d_backward is
// the CPU statement, pinned to the reference's own autograd gradients):
//   forward   y[b,o,ro,q] = bias[o] + sum_{ci,t} W[o,ci,t] * P[b,c][s*ro + dy_t][s*q + dk_t(ro&1)]
//   d bias    = sum_{b,ro,q} gy[b,o,ro,q]
//   d W       = sum_{b,ro,q} gy[b,o,ro,q] * P[b,c][...]               (k_hexconv_bwd_weight)
//   d P[Y][X] = sum_{o in group, t} W[o,ci,t] * gy[b,o,ro,q] for the unique (ro,q)
//               of each tap that reads (Y, X)                         (k_hexconv_bwd_input)
//   d x       = d P folded back through the padding mode's index map (constant
//               padding cells have no input pixel; reflect / replicate / circular
//               cells add onto the input pixel they copy).
// d input is a gather (one thread per input pixel, no atomics, deterministic).  d W
// and d bias are reductions over B*ho*wo samples: per-thread partial sums, a block
// reduction, then one float atomic per (o, ci, tap) per block.
#include <algorithm>
#include <climits>

#include "common.h"
#include "hexconv_geom.h"

namespace hg {

constexpr int BW_THREADS = 256;
constexpr int BW_MAXK = 128;          // taps 3r^2-3r+1 <= 127
constexpr int BW_NACC = 16;           // (ci, tap) weight-gradient sums per thread per pass

struct BwdGeom {
    int64_t B, C, O, h, w, ho, wo;
    int r, s, p, d, K, cg, og, op, pad_mode;
    double pad_value;
};

__device__ __forceinline__ void bw_taps(const BwdGeom& G, int* tdy, int* tdk0, int* tdk1) {
    for (int t = threadIdx.x; t < G.K; t += BW_THREADS) {
        int dy, d0, d1;
        tap_geom(G.r, G.s, G.d, G.op, t, &dy, &d0, &d1);
        tdy[t] = dy;
        tdk0[t] = d0;
        tdk1[t] = d1;
    }
    __syncthreads();
}

// d input: one thread per input sample (b, c, iy, ix).  The padded samples that map
// onto it are (iy+p, ix+p) and, for the non-constant modes, the pad-band samples
// whose pad_map lands on it.
template <typename Tx, typename A>
__global__ __launch_bounds__(BW_THREADS) void k_hexconv_bwd_input(const A* __restrict__ kern,
                                                                  const A* __restrict__ gy,
                                                                  Tx* __restrict__ dx, BwdGeom G) {
    __shared__ int tdy[BW_MAXK], tdk[2][BW_MAXK];
    bw_taps(G, tdy, tdk[0], tdk[1]);
    const int64_t total = G.B * G.C * G.h * G.w;
    const int np = G.pad_mode == HG_PAD_CONSTANT ? 0 : 2 * G.p;
    for (int64_t i = (int64_t)blockIdx.x * BW_THREADS + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * BW_THREADS) {
        const int64_t ix = i % G.w, t1 = i / G.w;
        const int64_t iy = t1 % G.h, t2 = t1 / G.h;
        const int64_t c = t2 % G.C, b = t2 / G.C;
        const int64_t g = c / G.cg, ci = c - g * G.cg;
        A acc = 0;
        for (int ey = -1; ey < np; ++ey) {
            int64_t Y = iy + G.p;
            if (ey >= 0) {                       // pad bands: rows [0, p) and [h+p, h+2p)
                Y = ey < G.p ? ey : G.h + ey;
                if (pad_map(Y - G.p, G.h, G.pad_mode) != iy) continue;
            }
            for (int ex = -1; ex < np; ++ex) {
                int64_t X = ix + G.p;
                if (ex >= 0) {
                    X = ex < G.p ? ex : G.w + ex;
                    if (pad_map(X - G.p, G.w, G.pad_mode) != ix) continue;
                }
                for (int t = 0; t < G.K; ++t) {
                    const int64_t Yr = Y - tdy[t];
                    if (Yr < 0 || Yr % G.s) continue;
                    const int64_t ro = Yr / G.s;
                    if (ro >= G.ho) continue;
                    const int64_t Xr = X - tdk[ro & 1][t];
                    if (Xr < 0 || Xr % G.s) continue;
                    const int64_t q = Xr / G.s;
                    if (q >= G.wo) continue;
                    const A* gp = gy + ((b * G.O + g * G.og) * G.ho + ro) * G.wo + q;
                    const A* kp = kern + ((g * G.og) * G.cg + ci) * G.K + t;
                    for (int oo = 0; oo < G.og; ++oo)
                        acc += kp[(int64_t)oo * G.cg * G.K] * gp[(int64_t)oo * G.ho * G.wo];
                }
            }
        }
        dx[i] = from_acc<Tx>(acc);
    }
}

template <typename A>
__device__ __forceinline__ A wave_sum(A v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// d kernel (and d bias): block (slice, o) walks the samples n = slice*256 + tid,
// step nslice*256, of the B*ho*wo output grid for output channel o, summing
// gy * P for the (ci, tap) pairs j0 .. j0+BW_NACC-1 (and gy itself for the bias).
template <typename Tx, typename A>
__global__ __launch_bounds__(BW_THREADS) void k_hexconv_bwd_weight(const Tx* __restrict__ x,
                                                                   const A* __restrict__ gy,
                                                                   A* __restrict__ dk,
                                                                   A* __restrict__ db, BwdGeom G,
                                                                   int j0) {
    __shared__ int tdy[BW_MAXK], tdk[2][BW_MAXK];
    __shared__ A red[BW_THREADS / 64][BW_NACC + 1];
    bw_taps(G, tdy, tdk[0], tdk[1]);
    const int64_t o = blockIdx.y;
    const int64_t g = o / G.og;
    const int64_t total = G.B * G.ho * G.wo;
    const int64_t Wp = G.w + 2 * G.p;
    const int nj = min(BW_NACC, G.cg * G.K - j0);
    const A padv = (A)G.pad_value;
    A acc[BW_NACC];
#pragma unroll
    for (int jj = 0; jj < BW_NACC; ++jj) acc[jj] = 0;
    A bacc = 0;
    for (int64_t n = (int64_t)blockIdx.x * BW_THREADS + threadIdx.x; n < total;
         n += (int64_t)gridDim.x * BW_THREADS) {
        const int64_t q = n % G.wo, t1 = n / G.wo;
        const int64_t ro = t1 % G.ho, b = t1 / G.ho;
        const A gv = gy[((b * G.O + o) * G.ho + ro) * G.wo + q];
        bacc += gv;
        const int par = (int)(ro & 1);
#pragma unroll
        for (int jj = 0; jj < BW_NACC; ++jj) {
            if (jj < nj) {
                const int j = j0 + jj;
                const int ci = j / G.K, t = j - ci * G.K;
                const int64_t Y = G.s * ro + tdy[t];
                const int64_t X = G.s * q + tdk[par][t];
                A v = 0;                                   // X >= W': type1 structural zero
                if (X < Wp) {
                    const int64_t ry = pad_map(Y - G.p, G.h, G.pad_mode);
                    const int64_t rx = pad_map(X - G.p, G.w, G.pad_mode);
                    v = (ry < 0 || rx < 0)
                            ? padv
                            : to_acc<A>(x[((b * G.C + g * G.cg + ci) * G.h + ry) * G.w + rx]);
                }
                acc[jj] += gv * v;
            }
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int jj = 0; jj < BW_NACC; ++jj) {
        const A sred = wave_sum(acc[jj]);
        if (lane == 0) red[wv][jj] = sred;
    }
    {
        const A sred = wave_sum(bacc);
        if (lane == 0) red[wv][BW_NACC] = sred;
    }
    __syncthreads();
    if (threadIdx.x < nj) {
        A sum = 0;
        for (int k = 0; k < BW_THREADS / 64; ++k) sum += red[k][threadIdx.x];
        atomicAdd(&dk[o * G.cg * G.K + j0 + threadIdx.x], sum);
    }
    if (db && j0 == 0 && threadIdx.x == BW_NACC) {
        A sum = 0;
        for (int k = 0; k < BW_THREADS / 64; ++k) sum += red[k][BW_NACC];
        atomicAdd(&db[o], sum);
    }
}

template <typename Tx, typename A>
static int bwd_launch(const void* x, const void* kern, const void* gy, void* dx, void* dk,
                      void* db, const BwdGeom& G, hipStream_t st) {
    if (dx) {
        const int64_t total = G.B * G.C * G.h * G.w;
        const int64_t blocks = std::min<int64_t>((total + BW_THREADS - 1) / BW_THREADS, 1 << 20);
        hipLaunchKernelGGL((k_hexconv_bwd_input<Tx, A>), dim3((unsigned)std::max<int64_t>(blocks, 1)),
                           dim3(BW_THREADS), 0, st, (const A*)kern, (const A*)gy, (Tx*)dx, G);
        const int rc = launch_status();
        if (rc) return rc;
    }
    if (dk || db) {
        const int nj = G.cg * G.K;
        if (dk) {
            const hipError_t e = hipMemsetAsync(dk, 0, sizeof(A) * (size_t)(G.O * nj), st);
            if (e != hipSuccess) return hip_status(e);
        }
        if (db) {
            const hipError_t e = hipMemsetAsync(db, 0, sizeof(A) * (size_t)G.O, st);
            if (e != hipSuccess) return hip_status(e);
        }
        const int64_t total = G.B * G.ho * G.wo;
        int64_t slices = std::max<int64_t>(1, (4096 + G.O - 1) / G.O);
        slices = std::min<int64_t>(slices, (total + BW_THREADS - 1) / BW_THREADS);
        slices = std::max<int64_t>(slices, 1);
        const dim3 grid((unsigned)slices, (unsigned)G.O);
        // pass 0 also sums the bias; with no d kernel wanted, one pass sums the bias only
        const int passes = dk ? (nj + BW_NACC - 1) / BW_NACC : 1;
        for (int pss = 0; pss < passes; ++pss) {
            hipLaunchKernelGGL((k_hexconv_bwd_weight<Tx, A>), grid, dim3(BW_THREADS), 0, st,
                               (const Tx*)x, (const A*)gy, dk ? (A*)dk : nullptr, (A*)db, G,
                               dk ? pss * BW_NACC : nj);
            const int rc = launch_status();
            if (rc) return rc;
        }
    }
    return HG_OK;
}

}  // namespace hg

extern "C" int hg_hexconv2d_backward(const void* x, const void* kernel, const void* gy, void* dx,
                                     void* dkernel, void* dbias, int x_dtype, int w_dtype,
                                     int64_t batch, int64_t in_channels, int64_t out_channels,
                                     int64_t h, int64_t w, int radius, int stride, int padding,
                                     int dilation, int groups, int even_odd_offset, int pad_mode,
                                     double pad_value, void* stream) {
    using namespace hg;
    BwdGeom G;
    int st = conv_out_shape(h, w, radius, stride, padding, dilation, &G.ho, &G.wo);
    if (st) return st;
    st = conv_check_args(batch, in_channels, out_channels, h, w, groups, padding, pad_mode);
    if (st) return st;
    G.K = 3 * radius * radius - 3 * radius + 1;
    if (G.K > BW_MAXK) return HG_EUNSUP;
    if (w_dtype != HG_F32 && w_dtype != HG_F64) return HG_EDTYPE;
    if (dx && !dtype_is_float(x_dtype)) return HG_EDTYPE;
    if (batch == 0 || G.ho == 0 || G.wo == 0) {
        // no samples: zero gradients (the reference's empty sums)
        hipStream_t s0 = reinterpret_cast<hipStream_t>(stream);
        const size_t ws = w_dtype == HG_F64 ? 8 : 4;
        if (dkernel && hipMemsetAsync(dkernel, 0, ws * (size_t)(out_channels * (in_channels / groups) * G.K), s0))
            return HG_EINVAL;
        if (dbias && hipMemsetAsync(dbias, 0, ws * (size_t)out_channels, s0)) return HG_EINVAL;
        if (dx && batch > 0 && h * w > 0 &&
            hipMemsetAsync(dx, 0, (size_t)dtype_size(x_dtype) * (size_t)(batch * in_channels * h * w), s0))
            return HG_EINVAL;
        return HG_OK;
    }
    if (!gy || (dx && !kernel) || (dkernel && !x)) return HG_EINVAL;
    if (!dx && !dkernel && !dbias) return HG_OK;
    G.B = batch; G.C = in_channels; G.O = out_channels; G.h = h; G.w = w;
    G.r = radius; G.s = stride; G.p = padding; G.d = dilation;
    G.cg = (int)(in_channels / groups);
    G.og = (int)(out_channels / groups);
    G.op = ((even_odd_offset & 1) + padding) & 1;
    G.pad_mode = pad_mode;
    G.pad_value = pad_value;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (w_dtype == HG_F64) {
        HG_DISPATCH_IN(x_dtype, TX, { return bwd_launch<TX, double>(x, kernel, gy, dx, dkernel, dbias, G, s); });
    } else {
        HG_DISPATCH_IN(x_dtype, TX, { return bwd_launch<TX, float>(x, kernel, gy, dx, dkernel, dbias, G, s); });
    }
    return HG_EDTYPE;
}
