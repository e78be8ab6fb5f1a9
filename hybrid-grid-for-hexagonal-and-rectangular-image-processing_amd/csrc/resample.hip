// resample.hip — gfx950 kernels for rect->hex, hex->rect and hexresize.
//
// Data layout: `planes` contiguous rasters (planes = batch * channels), each
// row-major (h, w) in, (h1, w1) out.  The lattice maps depend only on the
// output sample, never on the plane, so every workgroup owns one output tile
// and walks a chunk of planes with the tile's maps held in registers.
//
// Workgroup = 256 threads = 4 waves; tile = 16 rows x 128 columns.  Thread t
// owns column t%128 and the 8 rows 8*(t/128) .. +7, so each wave-wide store
// covers 64 consecutive output columns (coalesced).  Linear modes stage, per
// plane, the tile's source footprint (its rows/cols bounding box + 1-sample
// halo, zero-filled outside the raster: the reference's masked gathers,
// geometry_np.py:478-486) into LDS with 16-byte row-chunk loads, converted to
// the accumulator type, then blend from LDS.  A footprint that does not fit
// the LDS budget (extreme downsampling) takes the direct-gather path.
#include <algorithm>
#include <climits>

#include "common.h"
#include "lattice.h"
#include "stream.h"

namespace hg {

constexpr int RS_THREADS = 256;
constexpr int RS_TC = 128;          // tile columns
constexpr int RS_RPT = 8;           // rows per thread
constexpr int RS_TR = 16;           // tile rows = RS_RPT * RS_THREADS / RS_TC
constexpr int RS_LDS_MAX = 64 * 1024;

enum { OP_R2H = HG_OP_RECT_TO_HEX, OP_H2R = HG_OP_HEX_TO_RECT, OP_RESIZE = HG_OP_HEXRESIZE };

struct LaunchGeom {
    Geom g;
    int64_t planes;
    int ntx;          // tiles along columns
    int pc;           // planes per workgroup
    int cap;          // LDS tile capacity (elements of the accumulator type)
    int vec_ok;       // 16-byte staging loads legal (alignment)
};

// Per-row gather record of one output sample (global tap coordinates):
//  r2h : taps (i,j),(i,j+1),(i+1,j),(i+1,j+1); coef c0 = fi, c1 = 1-fi (column coefs apart)
//  tri : p1 = (i, j1); p2 = flag ? (i+1, j1-e) : (i, j1+1); p3 = (i+1, j1+1-e), where
//        e = s2 - s1 in {0,1} (geometry_np.py:288-295); coef alpha, beta, gamma.
// bits: r2h -> valid mask (4 bits); tri -> flag | e<<1 | vk<<2 (vk: p1,p2,p3 valid).
template <int OP, typename A>
struct RowRec {
    int r, c, bits;
    A c0, c1, c2;
};

template <int OP, typename A>
__device__ __forceinline__ RowRec<OP, A> row_record(const Geom& g, int64_t a, int64_t b) {
    RowRec<OP, A> q;
    if constexpr (OP == OP_R2H) {
        R2HSample s = r2h_sample(g, a, b);
        q.r = (int)s.i_n; q.c = (int)s.j_n; q.bits = s.valid;
        q.c0 = (A)s.i_f; q.c1 = (A)(1.0 - s.i_f); q.c2 = (A)0;
    } else {
        TriSample s = tri_sample(g, a, b);
        const int e = (int)(s.r[2] == s.r[0] ? 0 : (s.c[0] + 1 - s.c[2]));   // s2 - s1
        q.r = (int)s.r[0]; q.c = (int)s.c[0];
        q.bits = s.flag | (e << 1) | (s.vk << 2);
        q.c0 = (A)s.alpha; q.c1 = (A)s.beta; q.c2 = (A)s.gamma;
    }
    return q;
}

// Column coefficients of r2h (separable): fj, 1-fj.
template <typename A>
__device__ __forceinline__ void r2h_colcoef(const Geom& g, int64_t b, A* fj, A* gj) {
    R2HSample s = r2h_sample(g, 0, b);
    *fj = (A)s.j_f;
    *gj = (A)(1.0 - s.j_f);
}

// Blend in the reference's evaluation order (bit-exact when A = double).
template <int OP, typename A>
__device__ __forceinline__ A blend(A v0, A v1, A v2, A v3, A c0, A c1, A c2, A fj, A gj) {
    if constexpr (OP == OP_R2H) {
        A t1 = c0 * v2 + c1 * v0;   // geometry_np.py:515 (v2 = p3, v0 = p1)
        A t2 = c0 * v3 + c1 * v1;   // :516
        return fj * t2 + gj * t1;   // :517
    } else {
        (void)v3; (void)fj; (void)gj;
        return c0 * v0 + c1 * v1 + c2 * v2;   // :354
    }
}

template <typename T> struct VecOf { static constexpr int N = 16 / (int)sizeof(T); };

constexpr int RS_MAXPF = 8;   // 16-byte staging chunks held in registers per thread

// Load this thread's chunks of one plane's footprint (raw bits, zeros outside).
template <typename Tin>
__device__ __forceinline__ void fetch_chunks(const Tin* __restrict__ sp, uint4* regs, int64_t h,
                                             int64_t w, int64_t rlo, int nck, int total,
                                             int64_t ca, int vec_ok) {
    constexpr int V = VecOf<Tin>::N;
#pragma unroll
    for (int i = 0; i < RS_MAXPF; ++i) {
        const int idx = threadIdx.x + i * RS_THREADS;
        uint4 raw = make_uint4(0, 0, 0, 0);
        if (idx < total) {
            const int rr = idx / nck;
            const int64_t r = rlo + rr;
            const int64_t c = ca + (int64_t)(idx - rr * nck) * V;
            if (r >= 0 && r < h) {
                const Tin* rp = sp + r * w;
                if (vec_ok && c >= 0 && c + V <= w) {
                    raw = *reinterpret_cast<const uint4*>(rp + c);
                } else {
                    Tin e[V];
#pragma unroll
                    for (int j = 0; j < V; ++j)
                        e[j] = (c + j >= 0 && c + j < w) ? rp[c + j] : (Tin)0;
                    __builtin_memcpy(&raw, e, 16);
                }
            }
        }
        regs[i] = raw;
    }
}

template <typename Tin, typename A>
__device__ __forceinline__ void store_chunks(const uint4* regs, A* __restrict__ tile, int nck,
                                             int total, int pitch) {
    constexpr int V = VecOf<Tin>::N;
#pragma unroll
    for (int i = 0; i < RS_MAXPF; ++i) {
        const int idx = threadIdx.x + i * RS_THREADS;
        if (idx < total) {
            const int rr = idx / nck;
            const int cc = (idx - rr * nck) * V;
            Tin e[V];
            __builtin_memcpy(e, &regs[i], 16);
            A* d = tile + rr * pitch + cc;
#pragma unroll
            for (int j = 0; j < V; ++j) d[j] = to_acc<A>(e[j]);
        }
    }
}

// Per-thread state: 8 rows of one output column.
template <int OP, typename A>
struct ThreadRows {
    int o0[RS_RPT], o1[RS_RPT], o2[RS_RPT];   // tap offsets (LDS or in-plane; -1 = zero)
    A c0[RS_RPT], c1[RS_RPT], c2[RS_RPT];
    A fj, gj;
};

// Fill row k of the thread state from a record (static register indexing).
template <int OP, typename A>
__device__ __forceinline__ void put_row(ThreadRows<OP, A>& T, int k, const RowRec<OP, A>& q,
                                        int o0, int o1, int o2) {
#pragma unroll
    for (int kk = 0; kk < RS_RPT; ++kk)
        if (kk == k) {
            T.o0[kk] = o0; T.o1[kk] = o1; T.o2[kk] = o2;
            T.c0[kk] = q.c0; T.c1[kk] = q.c1; T.c2[kk] = q.c2;
        }
}

// LDS-staged linear resample.
template <int OP, typename Tin, typename Tout, typename A>
__global__ __launch_bounds__(RS_THREADS, 2) void k_resample_lds(const Tin* __restrict__ src,
                                                               Tout* __restrict__ dst,
                                                               LaunchGeom L) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* red = reinterpret_cast<int*>(smem);                 // 4 ints (16 B)
    A* tile = reinterpret_cast<A*>(smem + 16);
    constexpr int V = VecOf<Tin>::N;

    const Geom& g = L.g;
    const int tid = threadIdx.x;
    unsigned bx, by;
    xcd_swizzle2(&bx, &by);
    const int tx = (int)bx % L.ntx, ty = (int)bx / L.ntx;
    const int64_t b = (int64_t)tx * RS_TC + (tid & (RS_TC - 1));
    const int64_t a0 = (int64_t)ty * RS_TR + (tid / RS_TC) * RS_RPT;
    const int64_t p0 = (int64_t)by * L.pc;
    const int64_t p1 = p0 + L.pc < L.planes ? p0 + L.pc : L.planes;
    const int64_t in_plane = g.h * g.w, out_plane = g.h1 * g.w1;
    const bool bact = b < g.w1;
    const int nact = bact ? (int)max((int64_t)0, min((int64_t)RS_RPT, g.h1 - a0)) : 0;

    if (tid == 0) { red[0] = INT_MAX; red[1] = INT_MIN; red[2] = INT_MAX; red[3] = INT_MIN; }
    __syncthreads();
    // pass 1: footprint of the tile
    int rmin = INT_MAX, rmax = INT_MIN, cmin = INT_MAX, cmax = INT_MIN;
#pragma unroll 1
    for (int k = 0; k < nact; ++k) {
        RowRec<OP, A> q = row_record<OP, A>(g, a0 + k, b);
        rmin = min(rmin, q.r); rmax = max(rmax, q.r + 1);
        if constexpr (OP == OP_R2H) {
            cmin = min(cmin, q.c); cmax = max(cmax, q.c + 1);
        } else {
            const int e = (q.bits >> 1) & 1;
            cmin = min(cmin, q.c - e); cmax = max(cmax, q.c + 1);
        }
    }
    if (nact > 0) {
        atomicMin(&red[0], rmin); atomicMax(&red[1], rmax);
        atomicMin(&red[2], cmin); atomicMax(&red[3], cmax);
    }
    __syncthreads();
    if (red[0] == INT_MAX) return;   // tile entirely outside the output (uniform)
    const int64_t rlo = red[0];
    const int nr = red[1] - red[0] + 1;
    const int64_t ca = (int64_t)(red[2] & ~(V - 1));
    const int64_t cb = ((int64_t)red[3] + V) & ~(int64_t)(V - 1);
    const int pitch = (int)(cb - ca);
    const int nck = pitch / V;
    const int total = nr * nck;
    // The host sized the LDS for the worst tile; a larger footprint cannot happen
    // for the launch plan (k_resample_direct takes such calls), but never overrun.
    if ((int64_t)nr * pitch > L.cap || total > RS_MAXPF * RS_THREADS) return;

    // pass 2: LDS offsets + coefficients into registers
    ThreadRows<OP, A> T;
#pragma unroll
    for (int k = 0; k < RS_RPT; ++k) { T.o0[k] = T.o1[k] = T.o2[k] = 0; T.c0[k] = T.c1[k] = T.c2[k] = (A)0; }
    T.fj = T.gj = (A)0;
    if constexpr (OP == OP_R2H) {
        if (bact) r2h_colcoef<A>(g, b, &T.fj, &T.gj);
    }
#pragma unroll 1
    for (int k = 0; k < nact; ++k) {
        RowRec<OP, A> q = row_record<OP, A>(g, a0 + k, b);
        const int base = (int)((q.r - rlo) * pitch + (q.c - ca));
        if constexpr (OP == OP_R2H) {
            put_row<OP, A>(T, k, q, base, 0, 0);
        } else {
            const int flag = q.bits & 1, e = (q.bits >> 1) & 1;
            const int o2 = flag ? base + pitch - e : base + 1;
            put_row<OP, A>(T, k, q, base, o2, base + pitch + 1 - e);
        }
    }

    uint4 regs[RS_MAXPF];
    fetch_chunks<Tin>(src + p0 * in_plane, regs, g.h, g.w, rlo, nck, total, ca, L.vec_ok);
    for (int64_t p = p0; p < p1; ++p) {
        store_chunks<Tin, A>(regs, tile, nck, total, pitch);
        __syncthreads();
        if (p + 1 < p1)
            fetch_chunks<Tin>(src + (p + 1) * in_plane, regs, g.h, g.w, rlo, nck, total, ca,
                              L.vec_ok);
        Tout* dp = dst + p * out_plane;
#pragma unroll
        for (int k = 0; k < RS_RPT; ++k) {
            if (k < nact) {
                A v0, v1, v2, v3 = (A)0;
                if constexpr (OP == OP_R2H) {
                    v0 = tile[T.o0[k]]; v1 = tile[T.o0[k] + 1];
                    v2 = tile[T.o0[k] + pitch]; v3 = tile[T.o0[k] + pitch + 1];
                } else {
                    v0 = tile[T.o0[k]]; v1 = tile[T.o1[k]]; v2 = tile[T.o2[k]];
                }
                dp[(a0 + k) * g.w1 + b] = from_acc<Tout>(
                    blend<OP, A>(v0, v1, v2, v3, T.c0[k], T.c1[k], T.c2[k], T.fj, T.gj));
            }
        }
        __syncthreads();
    }
}

// Direct-gather linear resample (footprint too large for LDS: strong downsampling).
template <int OP, typename Tin, typename Tout, typename A>
__global__ __launch_bounds__(RS_THREADS, 2) void k_resample_direct(const Tin* __restrict__ src,
                                                                  Tout* __restrict__ dst,
                                                                  LaunchGeom L) {
    const Geom& g = L.g;
    const int tid = threadIdx.x;
    unsigned bx, by;
    xcd_swizzle2(&bx, &by);
    const int tx = (int)bx % L.ntx, ty = (int)bx / L.ntx;
    const int64_t b = (int64_t)tx * RS_TC + (tid & (RS_TC - 1));
    const int64_t a0 = (int64_t)ty * RS_TR + (tid / RS_TC) * RS_RPT;
    const int64_t p0 = (int64_t)by * L.pc;
    const int64_t p1 = p0 + L.pc < L.planes ? p0 + L.pc : L.planes;
    const int64_t in_plane = g.h * g.w, out_plane = g.h1 * g.w1;
    if (b >= g.w1) return;
    const int nact = (int)max((int64_t)0, min((int64_t)RS_RPT, g.h1 - a0));
    ThreadRows<OP, A> T;
    int o3[RS_RPT];
#pragma unroll
    for (int k = 0; k < RS_RPT; ++k) {
        T.o0[k] = T.o1[k] = T.o2[k] = o3[k] = -1;
        T.c0[k] = T.c1[k] = T.c2[k] = (A)0;
    }
    T.fj = T.gj = (A)0;
    if constexpr (OP == OP_R2H) r2h_colcoef<A>(g, b, &T.fj, &T.gj);
#pragma unroll 1
    for (int k = 0; k < nact; ++k) {
        RowRec<OP, A> q = row_record<OP, A>(g, a0 + k, b);
        const int base = (int)(q.r * g.w + q.c);
        int x0, x1, x2, x3 = -1;
        if constexpr (OP == OP_R2H) {
            x0 = (q.bits & 1) ? base : -1;
            x1 = (q.bits & 2) ? base + 1 : -1;
            x2 = (q.bits & 4) ? base + (int)g.w : -1;
            x3 = (q.bits & 8) ? base + (int)g.w + 1 : -1;
        } else {
            const int flag = q.bits & 1, e = (q.bits >> 1) & 1, vk = q.bits >> 2;
            x0 = (vk & 1) ? base : -1;
            x1 = (vk & 2) ? (flag ? base + (int)g.w - e : base + 1) : -1;
            x2 = (vk & 4) ? base + (int)g.w + 1 - e : -1;
        }
        put_row<OP, A>(T, k, q, x0, x1, x2);
#pragma unroll
        for (int kk = 0; kk < RS_RPT; ++kk) if (kk == k) o3[kk] = x3;
    }
    for (int64_t p = p0; p < p1; ++p) {
        const Tin* sp = src + p * in_plane;
        Tout* dp = dst + p * out_plane;
#pragma unroll
        for (int k = 0; k < RS_RPT; ++k) {
            if (k < nact) {
                const A v0 = T.o0[k] >= 0 ? to_acc<A>(sp[T.o0[k]]) : (A)0;
                const A v1 = T.o1[k] >= 0 ? to_acc<A>(sp[T.o1[k]]) : (A)0;
                const A v2 = T.o2[k] >= 0 ? to_acc<A>(sp[T.o2[k]]) : (A)0;
                const A v3 = (OP == OP_R2H && o3[k] >= 0) ? to_acc<A>(sp[o3[k]]) : (A)0;
                dp[(a0 + k) * g.w1 + b] = from_acc<Tout>(
                    blend<OP, A>(v0, v1, v2, v3, T.c0[k], T.c1[k], T.c2[k], T.fj, T.gj));
            }
        }
    }
}

// Nearest mode: copy the chosen source element bit for bit (or 0 outside).
template <int OP, typename E>
__global__ __launch_bounds__(RS_THREADS) void k_resample_nearest(const E* __restrict__ src,
                                                                 E* __restrict__ dst,
                                                                 LaunchGeom L) {
    const Geom& g = L.g;
    const int tid = threadIdx.x;
    unsigned bx, by;
    xcd_swizzle2(&bx, &by);
    const int tx = (int)bx % L.ntx, ty = (int)bx / L.ntx;
    const int64_t b = (int64_t)tx * RS_TC + (tid & (RS_TC - 1));
    const int64_t a0 = (int64_t)ty * RS_TR + (tid / RS_TC) * RS_RPT;
    const int64_t p0 = (int64_t)by * L.pc;
    const int64_t p1 = p0 + L.pc < L.planes ? p0 + L.pc : L.planes;
    if (b >= g.w1) return;
    int off[RS_RPT];
#pragma unroll
    for (int k = 0; k < RS_RPT; ++k) {
        const int64_t a = a0 + k;
        off[k] = -2;   // -2: not an output sample; -1: zero
        if (a >= g.h1) continue;
        if constexpr (OP == OP_R2H) {
            R2HSample s = r2h_sample(g, a, b);
            const int m = s.argmin;
            off[k] = ((s.valid >> m) & 1) ? (int)((s.i_n + (m >> 1)) * g.w + s.j_n + (m & 1))
                                          : -1;
        } else {
            TriSample s = tri_sample(g, a, b);
            const int m = s.argmin;
            off[k] = ((s.vk >> m) & 1) ? (int)(tri_pick_r(s, m) * g.w + tri_pick_c(s, m)) : -1;
        }
    }
    for (int64_t p = p0; p < p1; ++p) {
        const E* sp = src + p * g.h * g.w;
        E* dp = dst + p * g.h1 * g.w1;
#pragma unroll
        for (int k = 0; k < RS_RPT; ++k) {
            if (off[k] == -2) continue;
            dp[(a0 + k) * g.w1 + b] = off[k] >= 0 ? sp[off[k]] : (E)0;
        }
    }
}

// Integer maps + fp64 coefficients for parity tests (one thread per sample).
template <int OP>
__global__ void k_lattice_maps(Geom g, int32_t* __restrict__ im, double* __restrict__ fm) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = g.h1 * g.w1;
    if (q >= n) return;
    const int64_t a = q / g.w1, b = q - a * g.w1;
    if constexpr (OP == OP_R2H) {
        R2HSample s = r2h_sample(g, a, b);
        if (im) {
            im[q] = (int32_t)s.i_n; im[n + q] = (int32_t)s.j_n; im[2 * n + q] = 0;
            im[3 * n + q] = s.valid; im[4 * n + q] = s.argmin;
        }
        if (fm) {
            fm[q] = s.i_f; fm[n + q] = s.j_f;
            fm[2 * n + q] = 0.0; fm[3 * n + q] = 0.0; fm[4 * n + q] = 0.0;
        }
    } else {
        TriSample s = tri_sample(g, a, b);
        if (im) {
            im[q] = (int32_t)s.i_n; im[n + q] = (int32_t)s.j_n; im[2 * n + q] = s.flag;
            im[3 * n + q] = s.valid; im[4 * n + q] = s.argmin;
        }
        if (fm) {
            fm[q] = s.i_f; fm[n + q] = s.j_f;
            fm[2 * n + q] = s.alpha; fm[3 * n + q] = s.beta; fm[4 * n + q] = s.gamma;
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static Geom geom_for(int op, int64_t h, int64_t w, int64_t h1, int64_t w1) {
    if (op == OP_R2H) return make_r2h(h, w, h1, w1);
    return make_tri(h, w, h1, w1, op == OP_H2R ? 0.75 : 0.5);
}

static int check_sizes(int64_t planes, int64_t h, int64_t w, int64_t h1, int64_t w1) {
    if (planes < 0 || h < 0 || w < 0 || h1 < 0 || w1 < 0) return HG_EINVAL;
    if (h * w >= INT_MAX / 2 || h1 * w1 >= INT_MAX / 2) return HG_ESHAPE;
    if (h1 > INT_MAX / 2 || w1 > INT_MAX / 2) return HG_ESHAPE;
    return HG_OK;
}

static LaunchGeom plan(const Geom& g, int64_t planes) {
    LaunchGeom L;
    L.g = g;
    L.planes = planes;
    L.ntx = (int)((g.w1 + RS_TC - 1) / RS_TC);
    const int64_t nty = (g.h1 + RS_TR - 1) / RS_TR;
    const int64_t tiles = (int64_t)L.ntx * nty;
    // enough workgroups to fill 256 CUs several times over, and as many planes
    // per workgroup as that allows (the tile's maps are reused per plane)
    int64_t nchunk = (4096 + tiles - 1) / tiles;
    nchunk = std::max<int64_t>(1, std::min<int64_t>(nchunk, planes));
    nchunk = std::min<int64_t>(nchunk, 65535);
    L.pc = (int)((planes + nchunk - 1) / nchunk);
    L.cap = 0;
    L.vec_ok = 0;
    return L;
}

template <int OP, typename Tin, typename Tout, typename A>
static int launch_linear(const void* src, void* dst, int64_t planes, const Geom& g,
                         hipStream_t st) {
    if (planes == 0 || g.h1 == 0 || g.w1 == 0) return HG_OK;
    LaunchGeom L = plan(g, planes);
    constexpr int V = VecOf<Tin>::N;
    // LDS footprint bound of a 16x128 tile (rows (TR-1)*di + 2 + slack, cols
    // (TC-1)*dj + tap spread + chunk alignment on both ends)
    const double di = std::fabs(g.xs.step), dj = std::fabs(g.ys.step);
    const double rows = std::floor((RS_TR - 1) * di) + 4.0;
    const double cols = std::floor((RS_TC - 1) * dj) + 6.0 + 2.0 * V;
    const double cap = rows * cols;
    const bool use_lds = cap * sizeof(A) + 16 <= RS_LDS_MAX &&
                         rows * std::ceil(cols / V) <= RS_MAXPF * RS_THREADS;
    const uintptr_t base = reinterpret_cast<uintptr_t>(src);
    L.vec_ok = (base % 16 == 0) && ((g.w * (int64_t)sizeof(Tin)) % 16 == 0) ? 1 : 0;
    const int64_t nty = (g.h1 + RS_TR - 1) / RS_TR;
    dim3 grid((unsigned)(L.ntx * nty), (unsigned)((planes + L.pc - 1) / L.pc));
    if (use_lds) {
        L.cap = (int)cap;
        const size_t shmem = 16 + (size_t)L.cap * sizeof(A);
        hipLaunchKernelGGL((k_resample_lds<OP, Tin, Tout, A>), grid, dim3(RS_THREADS), shmem, st,
                           (const Tin*)src, (Tout*)dst, L);
    } else {
        hipLaunchKernelGGL((k_resample_direct<OP, Tin, Tout, A>), grid, dim3(RS_THREADS), 0, st,
                           (const Tin*)src, (Tout*)dst, L);
    }
    return launch_status();
}

template <int OP, typename E>
static int launch_nearest(const void* src, void* dst, int64_t planes, const Geom& g,
                          hipStream_t st) {
    if (planes == 0 || g.h1 == 0 || g.w1 == 0) return HG_OK;
    LaunchGeom L = plan(g, planes);
    const int64_t nty = (g.h1 + RS_TR - 1) / RS_TR;
    dim3 grid((unsigned)(L.ntx * nty), (unsigned)((planes + L.pc - 1) / L.pc));
    hipLaunchKernelGGL((k_resample_nearest<OP, E>), grid, dim3(RS_THREADS), 0, st,
                       (const E*)src, (E*)dst, L);
    return launch_status();
}

template <int OP>
static int resample(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                    int64_t w, int64_t h1, int64_t w1, int interp, void* stream) {
    int st = check_sizes(planes, h, w, h1, w1);
    if (st) return st;
    if (planes * h1 * w1 > 0 && (!dst || (h * w > 0 && !src))) return HG_EINVAL;
    const Geom g = geom_for(OP, h, w, h1, w1);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (OP == OP_R2H && (interp == HG_NEAREST || (interp == HG_LINEAR && !acc_is_double(sdt, ddt)))) {
        // ~2x downsampling lattices (ConvertToHexagon, the demo): row-streaming kernel
        const int rc = down_try(src, dst, sdt, ddt, planes, h, w, h1, w1, interp, s);
        if (rc != HG_EUNSUP) return rc;
    }
    if (OP != OP_R2H && interp == HG_NEAREST) {   // upsampling lattices (ConvertToHexagon^-1)
        const int rc = triup_try(OP, src, dst, sdt, ddt, planes, h, w, h1, w1, interp, s, false);
        if (rc != HG_EUNSUP) return rc;
    }
    if (interp == HG_NEAREST) {
        if (sdt != ddt) return HG_EDTYPE;
        switch (dtype_size(sdt)) {
        case 1: return launch_nearest<OP, uint8_t>(src, dst, planes, g, s);
        case 2: return launch_nearest<OP, uint16_t>(src, dst, planes, g, s);
        case 4: return launch_nearest<OP, uint32_t>(src, dst, planes, g, s);
        case 8: return launch_nearest<OP, uint64_t>(src, dst, planes, g, s);
        default: return HG_EDTYPE;
        }
    }
    if (interp != HG_LINEAR) return HG_EINVAL;
    if (!dtype_is_float(ddt)) return HG_EDTYPE;
    const bool dbl = acc_is_double(sdt, ddt);
    if (!dbl && OP != OP_RESIZE) {   // near-identity lattices: row-streaming kernels
        const int rc = stream_try(OP, src, dst, sdt, ddt, planes, h, w, h1, w1, s);
        if (rc != HG_EUNSUP) return rc;
    }
    if (!dbl && OP != OP_R2H) {      // upsampling lattices: hex (h/2, w/2) -> rect (h, w)
        const int rc = triup_try(OP, src, dst, sdt, ddt, planes, h, w, h1, w1, interp, s, false);
        if (rc != HG_EUNSUP) return rc;
    }
    if (!dbl && OP != OP_R2H) {      // ~2x hexresize (pyramid levels)
        const int rc = tristream_try(OP, src, dst, sdt, ddt, planes, h, w, h1, w1, s, false);
        if (rc != HG_EUNSUP) return rc;
    }
    HG_DISPATCH_IN(sdt, TIN, HG_DISPATCH_FLOAT_OUT(ddt, TOUT, {
        if (dbl) return launch_linear<OP, TIN, TOUT, double>(src, dst, planes, g, s);
        return launch_linear<OP, TIN, TOUT, float>(src, dst, planes, g, s);
    }));
    return HG_EDTYPE;
}

}  // namespace hg

extern "C" {

int hg_rect_to_hex(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                   int64_t w, int64_t h1, int64_t w1, int interp, void* stream) {
    return hg::resample<hg::OP_R2H>(src, dst, sdt, ddt, planes, h, w, h1, w1, interp, stream);
}

int hg_hex_to_rect(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                   int64_t w, int64_t h1, int64_t w1, int interp, void* stream) {
    return hg::resample<hg::OP_H2R>(src, dst, sdt, ddt, planes, h, w, h1, w1, interp, stream);
}

int hg_hexresize(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                 int64_t w, int64_t h1, int64_t w1, int interp, void* stream) {
    return hg::resample<hg::OP_RESIZE>(src, dst, sdt, ddt, planes, h, w, h1, w1, interp,
                                       stream);
}

int hg_resample_kernel(int op, int sdt, int ddt, int64_t planes, int64_t h, int64_t w,
                       int64_t h1, int64_t w1, int interp) {
    // the dispatch of hg::resample, without launching
    int st = hg::check_sizes(planes, h, w, h1, w1);
    if (st) return st;
    if (op != HG_OP_RECT_TO_HEX && op != HG_OP_HEX_TO_RECT && op != HG_OP_HEXRESIZE) return HG_EINVAL;
    if (interp == HG_NEAREST && sdt != ddt) return HG_EDTYPE;
    if (interp != HG_NEAREST && interp != HG_LINEAR) return HG_EINVAL;
    // resample() returns HG_EDTYPE for a non-float linear output (no kernel takes one: the
    // down kernel's dtype checks decline it first)
    if (interp == HG_LINEAR && !hg::dtype_is_float(ddt)) return HG_EDTYPE;
    const bool dbl = interp == HG_LINEAR && hg::acc_is_double(sdt, ddt);
    if (op == HG_OP_RECT_TO_HEX && !dbl &&
        hg::down_try(nullptr, nullptr, sdt, ddt, planes, h, w, h1, w1, interp, nullptr, true) == HG_OK)
        return HG_KERNEL_DOWN;
    if (interp == HG_NEAREST && op != HG_OP_RECT_TO_HEX &&
        hg::triup_try(op, nullptr, nullptr, sdt, ddt, planes, h, w, h1, w1, interp, nullptr, true) == HG_OK)
        return HG_KERNEL_UP;
    if (interp == HG_NEAREST) return HG_KERNEL_NEAREST;
    if (!dbl && op != HG_OP_HEXRESIZE &&
        hg::stream_try(op, nullptr, nullptr, sdt, ddt, planes, h, w, h1, w1, nullptr, true) == HG_OK)
        return HG_KERNEL_STREAM;
    if (!dbl && op != HG_OP_RECT_TO_HEX &&
        hg::triup_try(op, nullptr, nullptr, sdt, ddt, planes, h, w, h1, w1, interp, nullptr, true) == HG_OK)
        return HG_KERNEL_UP;
    if (!dbl && op != HG_OP_RECT_TO_HEX && interp == HG_LINEAR &&
        hg::tristream_try(op, nullptr, nullptr, sdt, ddt, planes, h, w, h1, w1, nullptr, true) == HG_OK)
        return HG_KERNEL_DOWN;
    return HG_KERNEL_GENERAL;
}

int hg_lattice_maps(int op, int64_t h, int64_t w, int64_t h1, int64_t w1, int32_t* imaps,
                    double* fmaps, void* stream) {
    int st = hg::check_sizes(1, h, w, h1, w1);
    if (st) return st;
    const int64_t n = h1 * w1;
    if (n == 0) return HG_OK;
    if (!imaps && !fmaps) return HG_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const unsigned blocks = (unsigned)((n + 255) / 256);
    switch (op) {
    case HG_OP_RECT_TO_HEX:
        hipLaunchKernelGGL(hg::k_lattice_maps<hg::OP_R2H>, dim3(blocks), dim3(256), 0, s,
                           hg::make_r2h(h, w, h1, w1), imaps, fmaps);
        break;
    case HG_OP_HEX_TO_RECT:
        hipLaunchKernelGGL(hg::k_lattice_maps<hg::OP_H2R>, dim3(blocks), dim3(256), 0, s,
                           hg::make_tri(h, w, h1, w1, 0.75), imaps, fmaps);
        break;
    case HG_OP_HEXRESIZE:
        hipLaunchKernelGGL(hg::k_lattice_maps<hg::OP_RESIZE>, dim3(blocks), dim3(256), 0, s,
                           hg::make_tri(h, w, h1, w1, 0.5), imaps, fmaps);
        break;
    default:
        return HG_EINVAL;
    }
    return hg::launch_status();
}

}  // extern "C"
