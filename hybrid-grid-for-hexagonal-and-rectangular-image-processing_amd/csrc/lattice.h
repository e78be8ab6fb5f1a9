// lattice.h — per-sample lattice geometry of the three resamplers.
//
// Everything here is evaluated in IEEE fp64 in the reference's NumPy order and
// the library is built with -ffp-contract=off, so the integer maps (i_n, j_n,
// the triangle flag, validity, nearest choice) and the fp64 coefficients are the
// reference's bit for bit.  The functions run once per output sample per
// workgroup and are reused for every plane the workgroup walks, so their fp64
// cost is amortised over the whole batch.
//
// Citations: /root/reference/HyGrid/geometry_np.py, geometry_torch.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hg {

// One numpy.linspace(start, stop, n) axis (geometry_np.py:415-422, :251-258).
struct Axis {
    double start, stop, delta, div, step;
    int64_t n;
};

inline Axis make_axis(double start, double stop, int64_t n) {
    Axis a;
    a.start = start;
    a.stop = stop;
    a.n = n;
    a.delta = stop - start;
    a.div = n > 1 ? (double)(n - 1) : 0.0;
    a.step = n > 1 ? a.delta / a.div : 0.0;
    return a;
}

// numpy 2.2 linspace: y = k*step (or (k/div)*delta if step == 0); y += start;
// y[-1] = stop.
__host__ __device__ __forceinline__ double axis_at(const Axis& a, int64_t k) {
    if (a.n > 1 && k == a.n - 1) return a.stop;
    if (a.n > 1) {
        double y = (a.step == 0.0) ? ((double)k / a.div) * a.delta : (double)k * a.step;
        return y + a.start;
    }
    return (double)k * a.delta + a.start;
}

// Geometry of one resample call.
struct Geom {
    int64_t h, w, h1, w1;
    Axis xs, ys;
    double hh, ww;   // (double)h, (double)w
};

// rect -> hex: corners geometry_np.py:401-413.
inline Geom make_r2h(int64_t h, int64_t w, int64_t h1, int64_t w1) {
    Geom g;
    g.h = h; g.w = w; g.h1 = h1; g.w1 = w1;
    g.hh = (double)h; g.ww = (double)w;
    g.xs = make_axis(-(g.hh / 2.0), g.hh / 2.0, h1);
    g.ys = make_axis(-(g.ww / 2.0 + 0.5), g.ww / 2.0 + 0.5, w1);
    return g;
}

// hex -> rect (margin .75, geometry_np.py:236-239) and hexresize (margin .5, :560-563).
inline Geom make_tri(int64_t h, int64_t w, int64_t h1, int64_t w1, double margin) {
    Geom g;
    g.h = h; g.w = w; g.h1 = h1; g.w1 = w1;
    g.hh = (double)h; g.ww = (double)w;
    g.xs = make_axis(-(g.hh / 2.0 - 0.5), g.hh / 2.0 - 0.5, h1);
    g.ys = make_axis(-((g.ww + 0.5) / 2.0 - margin), (g.ww + 0.5) / 2.0 - margin, w1);
    return g;
}

// ---- rect -> hex sample (geometry_np.py:440-506) ----------------------------
struct R2HSample {
    int64_t i_n, j_n;
    double i_f, j_f;
    int valid;    // bit k: neighbour k+1 inside the raster (:465-476)
    int argmin;   // nearest neighbour, first minimum (:499-506)
};

__host__ __device__ __forceinline__ R2HSample r2h_sample(const Geom& g, int64_t a, int64_t b) {
    R2HSample s;
    double x_ = axis_at(g.xs, a), y_ = axis_at(g.ys, b);
    double i_ = x_ + (double)(g.h - 1) * 0.5;   // :440
    double j_ = y_ + (double)(g.w - 1) * 0.5;   // :441
    s.i_n = (int64_t)i_;                        // astype(int): toward zero
    s.j_n = (int64_t)j_;
    s.i_f = i_ - (double)(float)s.i_n;          // :448 i_n.astype(np.float32)
    s.j_f = j_ - (double)(float)s.j_n;
    s.valid = 0;
    s.argmin = 0;
    double best = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {               // 1=(i,j) 2=(i,j+1) 3=(i+1,j) 4=(i+1,j+1)
        int64_t ii = s.i_n + (k >> 1), jj = s.j_n + (k & 1);
        if (ii >= 0 && jj >= 0 && ii < g.h && jj < g.w) s.valid |= 1 << k;
        double dx = x_ - (double)ii, dy = y_ - (double)jj;   // :499-502 (centred vs not)
        double d = dx * dx + dy * dy;
        if (k == 0 || d < best) { best = d; s.argmin = k; }
    }
    return s;
}

// ---- hex -> rect / hexresize sample (geometry_np.py:276-354) ----------------
struct TriSample {
    int64_t i_n, j_n;
    int64_t r[3], c[3];   // p1, p2 (chosen by the flag), p3
    int vk;               // validity bits of p1, p2, p3
    int flag, valid, argmin;
    double i_f, j_f, alpha, beta, gamma;
};

// The triangle sample at the Cartesian hex-frame point (x_, y_) of a source hex raster
// (h, w) = (g.h, g.w).  Shared by hex->rect / hexresize (x_, y_ from linspace axes) and
// image_geometric_transformation (x_, y_ from an inverse homography, geometry_np.py:107-187,
// whose i_f = i_ - i_n equals the (float) cast below for |i_n| < 2^24).
// I: the integer type of the lattice indices.  int64_t is the reference's astype(int);
// int gives the same values whenever |i_|, |j_| < 2^31 (and the float casts below are exact
// for |i_n|, |j_n| < 2^24 either way): tri_sample_fast, for the callers that check tri_fast_ok.
template <typename I>
__host__ __device__ __forceinline__ TriSample tri_sample_xy_t(const Geom& g, double x_, double y_) {
    TriSample s;
    const double hh = g.hh, ww = g.ww;
    double i_ = x_ + (double)(g.h - 1) * 0.5;            // :276
    double j_ = 0.5 * i_ + y_ + (ww - 0.5) * 0.5;        // :277
    const I in_ = (I)i_, jn_ = (I)j_;
    s.i_n = in_;
    s.j_n = jn_;
    s.i_f = i_ - (double)(float)in_;                     // :284-285
    s.j_f = j_ - (double)(float)jn_;
    I s1 = (I)((double)(in_ + 1) / 2.0);                 // :289 true div, then trunc
    I s2 = (I)((double)(in_ + 2) / 2.0);
    I ii[4] = {in_, in_ + 1, in_, in_ + 1};
    I jj[4] = {jn_ - s1, jn_ - s2, jn_ + 1 - s1, jn_ + 1 - s2};
    s.flag = s.i_f > s.j_f;                              // :298
    s.valid = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (ii[k] >= 0 && jj[k] >= 0 && ii[k] < g.h && jj[k] < g.w) s.valid |= 1 << k;
    int k2 = s.flag ? 1 : 2;                             // :321-322
    s.r[0] = ii[0]; s.c[0] = jj[0];
    s.r[1] = s.flag ? ii[1] : ii[2]; s.c[1] = s.flag ? jj[1] : jj[2];   // ii[k2] (selects: no scratch)
    s.r[2] = ii[3]; s.c[2] = jj[3];
    s.vk = (s.valid & 1) | (((s.valid >> k2) & 1) << 1) | (((s.valid >> 3) & 1) << 2);
    // cartesian vertices :326-331
    double fl = (double)s.flag, in = (double)s.i_n, jn = (double)s.j_n;
    double p1_x = in - (hh - 1.0) / 2.0;
    double p1_y = jn - in / 2.0 - (ww - 0.5) / 2.0;
    double p2_x = (in + fl) - (hh - 1.0) / 2.0;
    double p2_y = (jn + 1.0 - fl) - (in + fl) / 2.0 - (ww - 0.5) / 2.0;
    double p3_x = (in + 1.0) - (hh - 1.0) / 2.0;
    double p3_y = (jn + 1.0) - (in + 1.0) / 2.0 - (ww - 0.5) / 2.0;
    // nearest (geometry_torch.py:336-341): first minimum of d1, d2, d3
    double d1 = (x_ - p1_x) * (x_ - p1_x) + (y_ - p1_y) * (y_ - p1_y);
    double d2 = (x_ - p2_x) * (x_ - p2_x) + (y_ - p2_y) * (y_ - p2_y);
    double d3 = (x_ - p3_x) * (x_ - p3_x) + (y_ - p3_y) * (y_ - p3_y);
    s.argmin = 0;
    double best = d1;
    if (d2 < best) { best = d2; s.argmin = 1; }
    if (d3 < best) { s.argmin = 2; }
    // barycentric weights :348-353
    double S1 = 0.5 * fabs((x_ - p2_x) * (y_ - p3_y) - (y_ - p2_y) * (x_ - p3_x));
    double S2 = 0.5 * fabs((x_ - p1_x) * (y_ - p3_y) - (y_ - p1_y) * (x_ - p3_x));
    double S3 = 0.5 * fabs((x_ - p1_x) * (y_ - p2_y) - (y_ - p1_y) * (x_ - p2_x));
    double S = S1 + S2 + S3;
    s.alpha = S1 / S;
    s.beta = S2 / S;
    s.gamma = S3 / S;
    return s;
}

__host__ __device__ __forceinline__ TriSample tri_sample_xy(const Geom& g, double x_, double y_) {
    return tri_sample_xy_t<int64_t>(g, x_, y_);
}

// Vertex m of a sample by selects: s.r[m] with a run-time m puts the sample in scratch.
__host__ __device__ __forceinline__ int64_t tri_pick_r(const TriSample& s, int m) {
    return m == 0 ? s.r[0] : m == 1 ? s.r[1] : s.r[2];
}
__host__ __device__ __forceinline__ int64_t tri_pick_c(const TriSample& s, int m) {
    return m == 0 ? s.c[0] : m == 1 ? s.c[1] : s.c[2];
}

__host__ __device__ __forceinline__ TriSample tri_sample(const Geom& g, int64_t a, int64_t b) {
    return tri_sample_xy(g, axis_at(g.xs, a), axis_at(g.ys, b));
}

// axis_at for an axis with n > 1 and step != 0: the same value without the (k / div) * delta
// branch, whose fp64 division the compiler otherwise evaluates for every sample and selects away.
__host__ __device__ __forceinline__ double axis_at_step(const Axis& a, int64_t k) {
    if (k == a.n - 1) return a.stop;
    const double y = (double)k * a.step;
    return y + a.start;
}

// tri_sample bit for bit, cheaper (32-bit lattice indices, no speculated division) when
// tri_fast_ok(g) holds (host-checked by the streaming kernels that compute per-sample records).
// (Both axes need n > 1: h1 == 1 or w1 == 1 calls -- one output row or column -- run on the
// general kernels, which evaluate axis_at's n == 1 case; the streaming callers rely on it.)
inline bool tri_fast_ok(const Geom& g) {
    const int64_t lim = (int64_t)1 << 22;   // |i_|, |j_| < 2^23 << 2^24
    return g.xs.n > 1 && g.ys.n > 1 && g.xs.step != 0.0 && g.ys.step != 0.0 && g.h < lim &&
           g.w < lim && g.h1 < lim && g.w1 < lim;
}
__host__ __device__ __forceinline__ TriSample tri_sample_fast(const Geom& g, int64_t a, int64_t b) {
    return tri_sample_xy_t<int>(g, axis_at_step(g.xs, a), axis_at_step(g.ys, b));
}

}  // namespace hg
