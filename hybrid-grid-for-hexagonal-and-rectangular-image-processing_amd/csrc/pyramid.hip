// pyramid.hip — one level of the hex Gaussian pyramid (BASELINE config 5) in one pass:
//     Z = hexresize(HexConv2d_depthwise(X), (h1, w1))          (from_rect = 0)
//     Z = hexresize(HexConv2d_depthwise(rect_to_hex(R)), ...)  (from_rect = 1, level 0)
// The reference runs the stages as separate calls: rect_to_hex_resample
// (geometry_np.py:358-519, bilinear), HexConv2d(C, C, off, 2, padding=1, groups=C)
// (HexFrames.py:96-169) and hexresize (geometry_np.py:520-681, linear).  Here the
// intermediates stay in LDS in fp32 (one read of the level's input, one write of its
// output), so a level costs its compulsory bytes instead of 2-3 HBM round trips.
//
// Workgroup = 256 threads, one output tile of TZR x TZC samples of one plane chunk.
// Per tile (once, fp64 lattice, reused for every plane of the chunk):
//   * the tile's hexresize triangle records (geometry_np.py:551-681 via lattice.h):
//     3 taps + alpha/beta/gamma per output sample, and their footprint in the conv
//     output Y (rows ry0.., cols cy0..): at most YR_MAX x YC_MAX for a 2x downsample;
//   * from_rect: the r2h row / column records of the X footprint (separable,
//     geometry_np.py:440-449).
// Per plane:
//   1. stage the input footprint in LDS as fp32, zeros outside the raster (the conv's
//      constant-0 padding, and r2h's masked taps, geometry_np.py:478-486);
//      from_rect: blend the rect tile into the X tile (geometry_np.py:514-517, fp32);
//   2. Y = bias + 7-tap hex stencil of X (radius 2, padding 1; tap columns by row
//      parity as in fused_kernel.h), one column per thread with a sliding 3x3 window;
//   3. Z = alpha*Y[p1] + beta*Y[p2] + gamma*Y[p3] (geometry_np.py:347-354), stored.
// The next plane's input is loaded into registers while steps 2-3 run.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "lattice.h"

namespace hg {

// pyramid_stream.hip: the register-streaming level for 2x downsamples (HG_EUNSUP otherwise)
int pyr_stream_try(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                   int64_t C, int64_t h, int64_t w, int64_t h1, int64_t w1, const float* taps,
                   const float* bias, int even_odd_offset, int from_rect, hipStream_t st,
                   bool dry);
// pyramid_fused.hip: the same level on the streaming fused kernel (tried first)
int pyr_fused_try(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                  int64_t C, int64_t h, int64_t w, int64_t h1, int64_t w1, const float* taps,
                  const float* bias, int even_odd_offset, int from_rect, hipStream_t st,
                  bool dry);

constexpr int PY_THREADS = 256;
constexpr int PY_TZR = 16;                 // output tile rows
constexpr int PY_TZC = 60;                 // output tile columns (Y footprint <= 124 cols,
                                           // X tile <= 128: one column per thread and band)
constexpr int PY_NZ = (PY_TZR * PY_TZC + PY_THREADS - 1) / PY_THREADS;   // samples / thread
constexpr int PY_YR = 34;                  // Y footprint capacity (rows, cols)
constexpr int PY_YC = 124;
constexpr int PY_CB = 2;                   // row bands of the column stages (128 x 2 threads)
constexpr int PY_CT = PY_THREADS / PY_CB;  // threads (columns) per band
// X tile: Y footprint + 1 row above / below, 1 column left, 2 right (tap shifts -1..2),
// origin at an even column (dword-aligned staging), so up to one more column on the left
constexpr int PY_XR = PY_YR + 2, PY_XC = PY_YC + 4, PY_XP = PY_XC + 2;
// rect tile (from_rect): X tile + 1 row / column on each side, even origin
constexpr int PY_RR = PY_XR + 2, PY_RP = PY_XP + 4;
constexpr int PY_ABUF = (PY_RR * PY_RP > PY_YR * PY_YC ? PY_RR * PY_RP : PY_YR * PY_YC) + 1;
// prefetched input dwords per thread: a 16-bit staging window of <= PY_RR rows x
// (PY_RP / 2) dwords, an fp32 one PY_RR x PY_RP
template <typename T> struct PyPf {
    static constexpr int N = (PY_RR * (sizeof(T) == 2 ? PY_RP / 2 : PY_RP) + PY_THREADS - 1) / PY_THREADS;
};

struct PyrGeom {
    int64_t planes;
    int C, h, w, h1, w1;       // X (= conv in/out, = rect when from_rect) and Z sizes
    int ntx, nty, pc;          // tiles along Z columns / rows, planes per workgroup
    const float* taps;         // [C][7]
    const float* bias;         // [C] or null
    Geom tri;                  // hexresize lattice (h, w) -> (h1, w1)
    Geom r2h;                  // rect_to_hex lattice (h, w) -> (h, w) (from_rect)
    int cap_yr, cap_yc;        // Y footprint capacity (PY_YR, PY_YC; smaller only in tests)
    int* fault;                // set to 1 by a workgroup whose footprint overflows its tile
                               // (null unless forced_cap: the host bound is exact)
    int forced_cap;            // HYGRID_PYR_LDS_FORCE_CAP (tests): a tile below the bound
};

// r=2, padding-1 tap geometry (fused_kernel.h): tap t of an output row of parity `par`
// reads row +(ii-1) and column +shift (shift in -1..2).
__host__ __device__ constexpr int py_tap_ii(int t) { return t < 2 ? 0 : (t < 5 ? 1 : 2); }
__host__ __device__ constexpr int py_tap_col(int t) {
    return t < 2 ? 1 + 2 * t : (t < 5 ? 2 * (t - 2) : 1 + 2 * (t - 5));
}
__host__ __device__ constexpr int py_tap_shift(int t, int par, int op) {
    return ((1 + par + py_tap_col(t) - ((((par + py_tap_ii(t)) & 1) + op) & 1)) >> 1) - 1;
}

template <typename T> struct Epd { static constexpr int N = sizeof(T) == 2 ? 2 : 1; };
__host__ __device__ inline int floor_even(int c) { return c >= 0 ? c & ~1 : -((-c + 1) & ~1); }

// A staging window: nr rows from r0, dwords from element column ga (dword aligned), nd
// dwords per row.  Per thread and slot: element offset in the plane (-1: outside the
// raster -> zeros) and the LDS offset of the dword's first element.
template <typename T, int NPF>
struct Stage {
    int go[NPF], lo[NPF];
    __device__ __forceinline__ void plan(int r0, int ga, int nr, int nd, int h, int w, int pitch) {
        constexpr int EPD = Epd<T>::N;
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            const int idx = threadIdx.x + i * PY_THREADS;
            const int rr = idx / nd, j = idx - rr * nd;
            const int r = r0 + rr, c = ga + EPD * j;
            const bool in = idx < nr * nd;
            // w even (16-bit types) and c even: a dword is all inside or all outside
            go[i] = (in && r >= 0 && r < h && c >= 0 && c < w) ? r * w + c : -1;
            lo[i] = in ? rr * pitch + EPD * j : -1;
        }
    }
    __device__ __forceinline__ void fetch(const T* __restrict__ plane, unsigned* pf) const {
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            const unsigned v = *reinterpret_cast<const unsigned*>(plane + (go[i] >= 0 ? go[i] : 0));
            pf[i] = go[i] >= 0 ? v : 0u;
        }
    }
    __device__ __forceinline__ void store(const unsigned* pf, float* tile) const {
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
            if (lo[i] >= 0) {
                if constexpr (sizeof(T) == 2) {   // lo even (even pitch): one 8-byte write
                    *reinterpret_cast<float2*>(tile + lo[i]) =
                        make_float2((float)__builtin_bit_cast(T, (unsigned short)(pf[i] & 0xffffu)),
                                    (float)__builtin_bit_cast(T, (unsigned short)(pf[i] >> 16)));
                } else {
                    tile[lo[i]] = __builtin_bit_cast(float, pf[i]);
                }
            }
        }
    }
};

template <int FROM_RECT, int OP, typename Tin, typename Tout>
__global__ __launch_bounds__(PY_THREADS) void k_pyr_level(const Tin* __restrict__ src,
                                                          Tout* __restrict__ dst, PyrGeom G) {
    // from_rect: abuf = rect tile, then Y tile; bbuf = X tile.  Otherwise abuf = X tile,
    // bbuf = Y tile.  The last element of the Y tile's buffer is a constant 0: the tap
    // of a masked (outside the raster) triangle vertex.
    __shared__ float abuf[PY_ABUF];
    __shared__ float bbuf[FROM_RECT ? PY_XR * PY_XP : PY_YR * PY_YC + 1];
    __shared__ int red[8];
    // r2h records of the X footprint (from_rect): fractional part (fp32), first rect
    // index, validity bits (bit 0: index inside the raster, bit 1: index + 1 inside)
    // (rows packed as {index - sr0, validity, fraction} for one broadcast 8-byte read)
    __shared__ int2 rrow[FROM_RECT ? PY_XR : 1];
    __shared__ float rcol_f[FROM_RECT ? PY_XC : 1];
    __shared__ int rcol_j[FROM_RECT ? PY_XC : 1], rcol_v[FROM_RECT ? PY_XC : 1];
    __shared__ int rrow_i[FROM_RECT ? PY_XR : 1], rrow_v[FROM_RECT ? PY_XR : 1];
    __shared__ float rrow_f[FROM_RECT ? PY_XR : 1];
    float* const xt = FROM_RECT ? bbuf : abuf;       // X tile, pitch PY_XP
    float* const yt = FROM_RECT ? abuf : bbuf;       // Y tile, pitch PY_YC
    const int zero_slot = FROM_RECT ? PY_ABUF - 1 : PY_YR * PY_YC;

    const int tid = threadIdx.x;
    unsigned bx, by;
    xcd_swizzle2(&bx, &by);
    const int tx = (int)bx % G.ntx, ty = (int)bx / G.ntx;
    const int a0 = ty * PY_TZR, b0 = tx * PY_TZC;
    const int64_t p0 = (int64_t)by * G.pc;
    const int64_t p1 = p0 + G.pc < G.planes ? p0 + G.pc : G.planes;

    // ---- per tile: hexresize triangle records (fp64), footprint in Y -------------
    if (tid < 8) red[tid] = (tid & 1) ? INT_MIN : INT_MAX;
    if (tid == 0) yt[zero_slot] = 0.f;
    __syncthreads();
    int tr[PY_NZ][3], tc[PY_NZ][3], tv[PY_NZ];
    float tw[PY_NZ][3];
    {
        int rmin = INT_MAX, rmax = INT_MIN, cmin = INT_MAX, cmax = INT_MIN;
#pragma unroll
        for (int i = 0; i < PY_NZ; ++i) {
            const int k = tid + i * PY_THREADS;
            const int a = a0 + k / PY_TZC, b = b0 + k % PY_TZC;
            tv[i] = 0;
            tw[i][0] = tw[i][1] = tw[i][2] = 0.f;
            tr[i][0] = tr[i][1] = tr[i][2] = 0;
            tc[i][0] = tc[i][1] = tc[i][2] = 0;
            if (k < PY_TZR * PY_TZC && a < G.h1 && b < G.w1) {
                const TriSample s = tri_sample(G.tri, a, b);
                tv[i] = 8 | s.vk;                                   // bit 3: an output sample
                tw[i][0] = (float)s.alpha; tw[i][1] = (float)s.beta; tw[i][2] = (float)s.gamma;
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    tr[i][m] = (int)s.r[m];
                    tc[i][m] = (int)s.c[m];
                    if ((s.vk >> m) & 1) {
                        rmin = min(rmin, tr[i][m]); rmax = max(rmax, tr[i][m]);
                        cmin = min(cmin, tc[i][m]); cmax = max(cmax, tc[i][m]);
                    }
                }
            }
        }
        if (rmin != INT_MAX) {
            atomicMin(&red[0], rmin); atomicMax(&red[1], rmax);
            atomicMin(&red[2], cmin); atomicMax(&red[3], cmax);
        }
    }
    __syncthreads();
    const bool any_valid = red[0] != INT_MAX;
    // a tile whose samples all fall outside the raster still stores its zeros
    const int ry0 = any_valid ? red[0] : 0, cy0 = any_valid ? red[2] : 0;
    const int yr = any_valid ? red[1] - red[0] + 1 : 1, yc = any_valid ? red[3] - red[2] + 1 : 1;
    // Footprint larger than the LDS tile: the host bound (pyr_footprint_ok) is exact, so
    // this cannot happen for a launch it admitted; if it does (a test drives it with a
    // smaller cap), the workgroup raises the call's fault flag -- hg_hex_pyramid_level then
    // returns HG_EOVERFLOW -- and writes its outputs as NaN instead of leaving them unset.
    auto poison = [&]() {
        if (tid == 0 && G.fault) atomicOr(G.fault, 1);
        for (int64_t p = p0; p < p1; ++p)
            for (int k = tid; k < PY_TZR * PY_TZC; k += PY_THREADS) {
                const int a = a0 + k / PY_TZC, b = b0 + k % PY_TZC;
                if (a < G.h1 && b < G.w1)
                    dst[(p * G.h1 + a) * (int64_t)G.w1 + b] = (Tout)__builtin_nanf("");
            }
    };
    if (yr > G.cap_yr || yc > G.cap_yc) { poison(); return; }
    int zo[PY_NZ][3];
#pragma unroll
    for (int i = 0; i < PY_NZ; ++i)
#pragma unroll
        for (int m = 0; m < 3; ++m)
            zo[i][m] = ((tv[i] >> m) & 1) ? (tr[i][m] - ry0) * PY_YC + (tc[i][m] - cy0) : zero_slot;

    // X footprint: rows ry0-1 .. ry0+yr, columns cy0-1 .. cy0+yc+1; tile origin at the
    // even column xa, so Y column c reads X tile columns xs + c + (0..3)
    const int xr0 = ry0 - 1, xa = floor_even(cy0 - 1), xs = cy0 - 1 - xa;
    const int xr = yr + 2, xc = xs + yc + 3;                    // X tile extent (<= PY_XP)
    constexpr int EPD = Epd<Tin>::N;
    constexpr int NPF = PyPf<Tin>::N;
    Stage<Tin, NPF> stg;
    const int64_t in_plane = (int64_t)G.h * G.w, out_plane = (int64_t)G.h1 * G.w1;
    // column stages: thread -> column cc_t of row band cb_t
    const int cc_t = tid % PY_CT, cb_t = tid / PY_CT;

    int sr0, sa;                                                // staged window origin
    if constexpr (FROM_RECT) {
        // ---- from_rect: r2h records of the X tile, rect footprint ----------------
        for (int e = tid; e < xr + xc; e += PY_THREADS) {
            if (e < xr) {                                    // X row r: rect rows in, in+1
                const int r = xr0 + e;
                float f = 0.f;
                int in = 0, v = 0;
                if (r >= 0 && r < G.h) {
                    const R2HSample q = r2h_sample(G.r2h, r, 0);   // row part only
                    in = (int)q.i_n;
                    f = (float)q.i_f;
                    v = (in >= 0 && in < G.h ? 1 : 0) | (in + 1 >= 0 && in + 1 < G.h ? 2 : 0);
                    if (v) { atomicMin(&red[4], in); atomicMax(&red[5], in + 1); }
                }
                rrow_i[e] = in; rrow_f[e] = f; rrow_v[e] = v;
            } else {                                         // X col c: rect cols jn, jn+1
                const int g = e - xr, c = xa + g;
                float f = 0.f;
                int jn = 0, v = 0;
                if (c >= 0 && c < G.w) {
                    const R2HSample q = r2h_sample(G.r2h, 0, c);
                    jn = (int)q.j_n;
                    f = (float)q.j_f;
                    v = (jn >= 0 && jn < G.w ? 1 : 0) | (jn + 1 >= 0 && jn + 1 < G.w ? 2 : 0);
                    if (v) { atomicMin(&red[6], jn); atomicMax(&red[7], jn + 1); }
                }
                rcol_j[g] = jn; rcol_f[g] = f; rcol_v[g] = v;
            }
        }
        __syncthreads();
        const bool rin = red[4] != INT_MAX && red[6] != INT_MAX;
        sr0 = rin ? red[4] : 0;
        sa = rin ? floor_even(red[6]) : 0;
        const int sr = rin ? red[5] - red[4] + 1 : 1;
        const int sd = rin ? (red[7] - sa) / EPD + 1 : 1;
        if (sr > PY_RR || sd * EPD + 1 > PY_RP) { poison(); return; }   // host-checked
        for (int e = tid; e < xr; e += PY_THREADS)
            // rows outside the raster (validity 0) point at tile row 0: read, never used
            rrow[e] = make_int2((rrow_v[e] ? rrow_i[e] - sr0 : 0) | (rrow_v[e] << 28),
                                __builtin_bit_cast(int, rrow_f[e]));
        __syncthreads();
        stg.plan(sr0, sa, sr, sd, G.h, G.w, PY_RP);
    } else {
        sr0 = xr0;
        sa = xa;
        stg.plan(xr0, xa, xr, (xc + EPD - 1) / EPD, G.h, G.w, PY_XP);
    }
    float* const stile = FROM_RECT ? abuf : xt;

    // two planes of input in flight: plane p's registers are refilled with plane p + 2
    // right after they are staged
    unsigned pfa[NPF], pfb[NPF];
    if (p0 < p1) stg.fetch(src + p0 * in_plane, pfa);
    if (p0 + 1 < p1) stg.fetch(src + (p0 + 1) * in_plane, pfb);
    auto plane = [&](int64_t p, unsigned* pf) {
        const int ch = (int)(p % G.C);
        // ---- 1. stage the input window (zeros outside the raster) --------------------
        stg.store(pf, stile);
        __syncthreads();
        if (p + 2 < p1) stg.fetch(src + (p + 2) * in_plane, pf);
        if constexpr (FROM_RECT) {
            // X = r2h(rect) on the hex raster, 0 outside it (the conv's padding).  One X
            // column per thread walks down its band; the two rect taps of the column stay
            // in registers, so a row reads only the rect row it newly needs.
            if (cc_t < xc) {
                const int cc = cc_t, c = xa + cc;
                const int vc = rcol_v[cc], jo = vc ? rcol_j[cc] - sa : 0;   // masked: col 0
                const float fj = rcol_f[cc];
                const bool cin = c >= 0 && c < G.w;
                constexpr int XRB = (PY_XR + PY_CB - 1) / PY_CB;
                const int rb = cb_t * XRB, re = min(rb + XRB, xr);
                int cur = -2;                         // rect tile row held in (q0, q1): none
                float q0 = 0.f, q1 = 0.f, n0 = 0.f, n1 = 0.f;   // rows cur, cur + 1
                for (int rr = rb; rr < re; ++rr) {
                    const int r = xr0 + rr;
                    const int2 rec = rrow[rr];
                    const int ri = rec.x & 0x0fffffff, vr = rec.x >> 28;
                    const float fi = __builtin_bit_cast(float, rec.y);
                    if (ri != cur) {                  // slide: row ri + 1 is new
                        if (ri == cur + 1) { q0 = n0; q1 = n1; }
                        else { q0 = abuf[ri * PY_RP + jo]; q1 = abuf[ri * PY_RP + jo + 1]; }
                        n0 = abuf[(ri + 1) * PY_RP + jo];
                        n1 = abuf[(ri + 1) * PY_RP + jo + 1];
                        cur = ri;
                    }
                    float v = 0.f;
                    if (cin && r >= 0 && r < G.h) {
                        // masked gathers read 0 (geometry_np.py:465-486): a tap is valid iff
                        // its row and its column are inside the raster
                        const float p1_ = (vr & 1) && (vc & 1) ? q0 : 0.f;
                        const float p2_ = (vr & 1) && (vc & 2) ? q1 : 0.f;
                        const float p3_ = (vr & 2) && (vc & 1) ? n0 : 0.f;
                        const float p4_ = (vr & 2) && (vc & 2) ? n1 : 0.f;
                        // geometry_np.py:514-517 in fp32
                        const float t1 = fi * p3_ + (1.f - fi) * p1_;
                        const float t2 = fi * p4_ + (1.f - fi) * p2_;
                        v = fj * t2 + (1.f - fj) * t1;
                    }
                    xt[rr * PY_XP + cc] = v;
                }
            }
            __syncthreads();
        }
        // ---- 2. Y = depthwise hex conv of X (sliding 3x4 window down one column) ------
        if (cc_t < yc) {
            float k[7];
#pragma unroll
            for (int t = 0; t < 7; ++t) k[t] = G.taps[ch * 7 + t];
            const float bv = G.bias ? G.bias[ch] : 0.f;
            const float* xcol = xt + xs + cc_t;     // X tile column of tap shift -1
            constexpr int YRB = (PY_YR + PY_CB - 1) / PY_CB;
            const int rb = cb_t * YRB, re = min(rb + YRB, yr);
            float wm[4], w0[4], wp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                wm[j] = xcol[rb * PY_XP + j];
                w0[j] = xcol[(rb + 1) * PY_XP + j];
            }
            // one Y row of parity PAR (tap columns as in fused_kernel.h), then slide (a
            // 3-row register ring unrolled by 6 instead needs ~25 more VGPRs: 3 waves per
            // SIMD instead of 4, and ran slower)
            auto yrow = [&](int rr, auto PARc) {
                constexpr int PAR = decltype(PARc)::value;
#pragma unroll
                for (int j = 0; j < 4; ++j) wp[j] = xcol[(rr + 2) * PY_XP + j];
                float y = bv;
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int ii = py_tap_ii(t), sh = 1 + py_tap_shift(t, PAR, OP);
                    const float* row = ii == 0 ? wm : (ii == 1 ? w0 : wp);
                    y = fmaf(k[t], row[sh], y);
                }
                yt[rr * PY_YC + cc_t] = y;
#pragma unroll
                for (int j = 0; j < 4; ++j) { wm[j] = w0[j]; w0[j] = wp[j]; }
            };
            auto rows = [&](auto P0c) {
                constexpr int P0 = decltype(P0c)::value;
                int rr = rb;
                for (; rr + 2 <= re; rr += 2) {
                    yrow(rr, std::integral_constant<int, P0>{});
                    yrow(rr + 1, std::integral_constant<int, 1 - P0>{});
                }
                if (rr < re) yrow(rr, std::integral_constant<int, P0>{});
            };
            if (((ry0 + rb) & 1) == 0) rows(std::integral_constant<int, 0>{});
            else rows(std::integral_constant<int, 1>{});
        }
        __syncthreads();
        // ---- 3. Z = triangle blend of Y (geometry_np.py:347-354) -------------------
        Tout* dp = dst + p * out_plane;
#pragma unroll
        for (int i = 0; i < PY_NZ; ++i) {
            if (tv[i] & 8) {
                const int kk = tid + i * PY_THREADS;
                const int a = a0 + kk / PY_TZC, b = b0 + kk % PY_TZC;
                const float v = tw[i][0] * yt[zo[i][0]] + tw[i][1] * yt[zo[i][1]] +
                                tw[i][2] * yt[zo[i][2]];
                dp[(int64_t)a * G.w1 + b] = (Tout)v;
            }
        }
        // Without from_rect no barrier here: the next plane's staging writes only the X
        // tile (last read by this plane's Y stage, before the barrier above), and its
        // first barrier orders this Z stage's Y reads before the next Y stage's writes.
        // from_rect stages the rect tile into the Y tile's buffer: wait for every Z read.
        if constexpr (FROM_RECT) __syncthreads();
    };
    for (int64_t p = p0; p < p1; p += 2) {
        plane(p, pfa);
        if (p + 1 < p1) plane(p + 1, pfb);
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// rect -> hex taps of every live sample (one of its two indices inside the raster) sit
// at hex index - 1 or + 0, so a hex footprint of n rows / columns reads at most n + 1
// rect rows / columns (the rect tile's +1 halo).
static bool r2h_near_identity(const Geom& g) {
    for (int64_t q = 0; q < g.w1; ++q) {
        const int64_t jn = (int64_t)(axis_at(g.ys, q) + (double)(g.w - 1) * 0.5);
        const bool live = (jn >= 0 && jn < g.w) || (jn + 1 >= 0 && jn + 1 < g.w);
        if (live && (jn - q < -1 || jn - q > 0)) return false;
    }
    for (int64_t r = 0; r < g.h1; ++r) {
        const int64_t in = (int64_t)(axis_at(g.xs, r) + (double)(g.h - 1) * 0.5);
        const bool live = (in >= 0 && in < g.h) || (in + 1 >= 0 && in + 1 < g.h);
        if (live && (in - r < -1 || in - r > 0)) return false;
    }
    return true;
}

// Does the Y footprint of every output tile fit cap_r x cap_c?  A sample's triangle
// vertices lie in rows i_n, i_n + 1 and columns j_n - s2 .. j_n + 1 - s1 (s1 = (i_n + 1) / 2,
// s2 = (i_n + 2) / 2; geometry_np.py:289-322, lattice.h tri_sample_xy).  i_n depends on the row
// a only and grows with it; j_n grows with the column b for a fixed row.  So per tile column
// [b0, b1] and row a the columns span [j_n(a, b0) - s2(a), j_n(a, b1) + 1 - s1(a)], and a
// tile's footprint is the union over its rows: an exact bound on the kernel's reduction
// (which counts only the vertices inside the raster), O(h1) per tile column.
static bool pyr_footprint_ok(const Geom& g, int cap_r, int cap_c) {
    // i_n(a) and j_n(a, b) exactly as tri_sample_xy computes them (the same fp64 expressions in
    // the same order), without the rest of the sample: the row terms once per row, the y_ of
    // every tile column's two end columns once per call, then two adds and a trunc per
    // (row, tile column).
    const double ch = (double)(g.h - 1) * 0.5, cw = (g.ww - 0.5) * 0.5;
    const int64_t nty = (g.h1 + PY_TZR - 1) / PY_TZR, ntx = (g.w1 + PY_TZC - 1) / PY_TZC;
    std::vector<double> y0(ntx), y1(ntx);
    std::vector<int64_t> lo(ntx), hi(ntx);
    for (int64_t tx = 0; tx < ntx; ++tx) {
        y0[tx] = axis_at(g.ys, tx * PY_TZC);
        y1[tx] = axis_at(g.ys, std::min<int64_t>(tx * PY_TZC + PY_TZC, g.w1) - 1);
    }
    for (int64_t ty = 0; ty < nty; ++ty) {
        const int64_t a0 = ty * PY_TZR, a1 = std::min<int64_t>(a0 + PY_TZR, g.h1);
        std::fill(lo.begin(), lo.end(), INT64_MAX);
        std::fill(hi.begin(), hi.end(), INT64_MIN);
        int64_t in0 = 0, in1 = 0;
        for (int64_t a = a0; a < a1; ++a) {
            const double i_ = axis_at(g.xs, a) + ch;                              // :276
            const int64_t in = (int64_t)i_;                                       // :280
            if (a == a0) in0 = in;
            in1 = in;
            const int64_t q1 = (int64_t)((double)(in + 1) / 2.0), q2 = (int64_t)((double)(in + 2) / 2.0);
            const double hi_ = 0.5 * i_;
            for (int64_t tx = 0; tx < ntx; ++tx) {
                lo[tx] = std::min(lo[tx], (int64_t)(hi_ + y0[tx] + cw) - q2);     // :277, :281
                hi[tx] = std::max(hi[tx], (int64_t)(hi_ + y1[tx] + cw) + 1 - q1);
            }
        }
        if (in1 + 1 - in0 + 1 > cap_r) return false;       // i_n grows with the row
        for (int64_t tx = 0; tx < ntx; ++tx)
            if (hi[tx] - lo[tx] + 1 > cap_c) return false;
    }
    return true;
}

template <int FR, int OP, typename Tin, typename Tout>
static int pyr_launch(const void* src, void* dst, PyrGeom& G, hipStream_t st) {
    const int64_t tiles = (int64_t)G.ntx * G.nty;
    int64_t nchunk = std::max<int64_t>(1, std::min<int64_t>((2048 + tiles - 1) / tiles, G.planes));
    nchunk = std::min<int64_t>(nchunk, 65535);
    G.pc = (int)((G.planes + nchunk - 1) / nchunk);
    const dim3 grid((unsigned)tiles, (unsigned)((G.planes + G.pc - 1) / G.pc));
    // The host bound (pyr_footprint_ok) is exact, so a launch it admitted never overflows its
    // tile: production launches carry no fault word and never synchronise (a workgroup that
    // overflowed anyway would still write NaN, never stale data).  Only under the test-only
    // HYGRID_PYR_LDS_FORCE_CAP (a tile smaller than the bound) does the call allocate a fault
    // word, read it back and return HG_EOVERFLOW.
    if (!G.forced_cap) {
        G.fault = nullptr;
        hipLaunchKernelGGL((k_pyr_level<FR, OP, Tin, Tout>), grid, dim3(PY_THREADS), 0, st,
                           (const Tin*)src, (Tout*)dst, G);
        return launch_status();
    }
    int* fault = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&fault), sizeof(int), st);
    if (e != hipSuccess) return (int)e;
    G.fault = fault;
    int rc = (int)hipMemsetAsync(fault, 0, sizeof(int), st);
    if (rc == HG_OK) {
        hipLaunchKernelGGL((k_pyr_level<FR, OP, Tin, Tout>), grid, dim3(PY_THREADS), 0, st,
                           (const Tin*)src, (Tout*)dst, G);
        rc = launch_status();
    }
    int hf = 0;
    if (rc == HG_OK) rc = (int)hipMemcpyAsync(&hf, fault, sizeof(int), hipMemcpyDeviceToHost, st);
    if (rc == HG_OK) rc = (int)hipStreamSynchronize(st);
    (void)hipFreeAsync(fault, st);
    if (rc == HG_OK && hf) rc = HG_EOVERFLOW;
    return rc;
}

template <typename Tin, typename Tout>
static int pyr_dispatch(const void* src, void* dst, PyrGeom& G, int from_rect, int op,
                        hipStream_t st) {
    if (from_rect)
        return op ? pyr_launch<1, 1, Tin, Tout>(src, dst, G, st) : pyr_launch<1, 0, Tin, Tout>(src, dst, G, st);
    return op ? pyr_launch<0, 1, Tin, Tout>(src, dst, G, st) : pyr_launch<0, 0, Tin, Tout>(src, dst, G, st);
}

static bool pyr_dtypes_ok(int src_dtype, int dst_dtype) {
    switch (src_dtype) {
    case HG_F16: return dst_dtype == HG_F16 || dst_dtype == HG_F32;
    case HG_BF16: return dst_dtype == HG_BF16 || dst_dtype == HG_F32;
    case HG_F32: return dst_dtype == HG_F32 || dst_dtype == HG_F16 || dst_dtype == HG_BF16;
    default: return false;
    }
}

// One level: the fused kernel, else k_pyr_stream, else k_pyr_level (each declines with
// HG_EUNSUP outside its domain).  dry: return the kernel that would run, launch nothing.
// HYGRID_PYR_KERNEL = "fused" | "stream" | "lds" restricts the choice to one kernel (tests,
// A/B).  HYGRID_PYR_LDS_FORCE_CAP = <rows> (tests only): skip the host footprint bound and
// give k_pyr_level a tile of that many rows, to drive its overflow branch.
static int pyr_level(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                     int64_t channels, int64_t h, int64_t w, int64_t h1, int64_t w1,
                     const float* taps, const float* bias, int even_odd_offset, int from_rect,
                     hipStream_t st, bool dry) {
    if (batch < 0 || channels < 1 || h < 1 || w < 1 || h1 < 1 || w1 < 1) return HG_EINVAL;
    if (!dry && (!taps || (batch > 0 && (!src || !dst)))) return HG_EINVAL;
    if (even_odd_offset != 0 && even_odd_offset != 1) return HG_EINVAL;
    if (h * w >= INT_MAX / 2 || h1 * w1 >= INT_MAX / 2) return HG_ESHAPE;
    if (!pyr_dtypes_ok(src_dtype, dst_dtype)) return HG_EDTYPE;
    if (batch == 0) return dry ? HG_PYR_LDS : HG_OK;
    // a restriction to one kernel, or null (unset, "auto" or any other value: no restriction)
    const char* force = nullptr;
    for (const char* k : {"fused", "stream", "lds"})
        if (env_is("HYGRID_PYR_KERNEL", k)) force = k;
    if (!force || !strcmp(force, "fused")) {
        const int rc = pyr_fused_try(src, dst, src_dtype, dst_dtype, batch, channels, h, w, h1, w1,
                                     taps, bias, even_odd_offset, from_rect, st, dry);
        if (rc != HG_EUNSUP) return rc;
    }
    if (!force || !strcmp(force, "stream")) {
        const int rc = pyr_stream_try(src, dst, src_dtype, dst_dtype, batch, channels, h, w, h1,
                                      w1, taps, bias, even_odd_offset, from_rect, st, dry);
        if (rc != HG_EUNSUP) return rc;
    }
    if (force && strcmp(force, "lds")) return HG_EUNSUP;
    PyrGeom G = {};
    G.planes = batch * channels;
    G.C = (int)channels;
    G.h = (int)h; G.w = (int)w; G.h1 = (int)h1; G.w1 = (int)w1;
    G.ntx = (int)((w1 + PY_TZC - 1) / PY_TZC);
    G.nty = (int)((h1 + PY_TZR - 1) / PY_TZR);
    const int op = (even_odd_offset + 1) & 1;  // tap column class at padding 1
    G.taps = taps;
    G.bias = bias;
    G.tri = make_tri(h, w, h1, w1, 0.5);
    G.r2h = make_r2h(h, w, h, w);
    G.cap_yr = PY_YR;
    G.cap_yc = PY_YC;
    if ((int64_t)G.ntx * G.nty > INT_MAX) return HG_ESHAPE;
    // dword staging of 16-bit rasters: rows must start on a dword (even width, 4-B base)
    if (dtype_size(src_dtype) == 2 && ((w & 1) || (reinterpret_cast<uintptr_t>(src) & 3)))
        return HG_EUNSUP;
    if (from_rect && !r2h_near_identity(G.r2h)) return HG_EUNSUP;
    const char* cap = getenv("HYGRID_PYR_LDS_FORCE_CAP");   // tests only
    if (cap && atoi(cap) > 0) {
        G.cap_yr = std::min(PY_YR, atoi(cap));
        G.forced_cap = 1;
    } else if (!pyr_footprint_ok(G.tri, PY_YR, PY_YC)) {
        return HG_EUNSUP;
    }
    if (dry) return HG_PYR_LDS;
    switch (src_dtype) {
    case HG_F16:
        if (dst_dtype == HG_F16) return pyr_dispatch<_Float16, _Float16>(src, dst, G, from_rect, op, st);
        return pyr_dispatch<_Float16, float>(src, dst, G, from_rect, op, st);
    case HG_BF16:
        if (dst_dtype == HG_BF16) return pyr_dispatch<__bf16, __bf16>(src, dst, G, from_rect, op, st);
        return pyr_dispatch<__bf16, float>(src, dst, G, from_rect, op, st);
    default:
        if (dst_dtype == HG_F32) return pyr_dispatch<float, float>(src, dst, G, from_rect, op, st);
        if (dst_dtype == HG_F16) return pyr_dispatch<float, _Float16>(src, dst, G, from_rect, op, st);
        return pyr_dispatch<float, __bf16>(src, dst, G, from_rect, op, st);
    }
}

}  // namespace hg

extern "C" int hg_hex_pyramid_level(const void* src, void* dst, int src_dtype, int dst_dtype,
                                    int64_t batch, int64_t channels, int64_t h, int64_t w,
                                    int64_t h1, int64_t w1, const float* taps,
                                    const float* bias, int even_odd_offset, int from_rect,
                                    void* stream) {
    return hg::pyr_level(src, dst, src_dtype, dst_dtype, batch, channels, h, w, h1, w1, taps, bias,
                         even_odd_offset, from_rect, reinterpret_cast<hipStream_t>(stream), false);
}

extern "C" int hg_hex_pyramid_level_kernel(int x_dtype, int y_dtype, int64_t batch,
                                           int64_t channels, int64_t h, int64_t w, int64_t h1,
                                           int64_t w1, int even_odd_offset, int from_rect) {
    return hg::pyr_level(nullptr, nullptr, x_dtype, y_dtype, batch, channels, h, w, h1, w1, nullptr,
                         nullptr, even_odd_offset, from_rect, nullptr, true);
}
