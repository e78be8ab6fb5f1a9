// tri_window.h — host checks shared by the row-streaming triangle-blend kernels
// (hexresize_down.hip: downsampling; tri_up.hip: upsampling): does a window of output
// columns keep every triangle vertex inside the input columns its wave loads, and does a band
// of output rows read only the input rows it loads?  The kernels evaluate the same window
// origin (tsk_window_x0) on the device.
//
// With s1(a) = trunc((i_n + 1) / 2) (geometry_np.py:289) and j_ = 0.5 i_ + y_(b) + (w - 0.5) / 2
// (:277), c0 = j_n - s1 = floor(q(a) + f(b)) for q(a) = 0.5 i_(a) - s1(a) and f(b) = y_(b) +
// (w - 0.5) / 2 (f increasing), and every vertex lies in c0 - 1 .. c0 + 1.
#pragma once
#include <algorithm>
#include <cmath>
#include <stdint.h>

#include "lattice.h"

namespace hg {

// First input column of the window starting at output column b0: the lowest vertex column
// of its outputs (c0 - 1, with c0 >= floor(qmin + f(b0))) rounded down to a multiple of al
// (the columns of one lane's load piece, so a piece clamped at the left edge holds only
// columns outside the raster).
__host__ __device__ inline int tsk_window_x0(const Geom& g, double qmin, int b0, int al) {
    const double cw = ((double)g.w - 0.5) * 0.5;
    const double f = axis_at(g.ys, b0) + cw;
    const int lo = (int)floor(qmin + f - 1e-6) - 1;
    return lo >= 0 ? lo - lo % al : -(((-lo) + al - 1) / al * al);
}

// Every output row's i_n inside the input; qmin / qmax = the extremes of q(a).  O(h1).
inline bool tsk_rows_ok(const Geom& g, double* qmin, double* qmax) {
    *qmin = 1e300;
    *qmax = -1e300;
    const double ch = (double)(g.h - 1) * 0.5;
    for (int64_t a = 0; a < g.h1; ++a) {
        const double i_ = axis_at(g.xs, a) + ch;
        const int64_t in = (int64_t)i_;
        if (in < 0 || in >= g.h) return false;
        const int64_t s1 = (int64_t)((double)(in + 1) / 2.0);
        const double q = 0.5 * i_ - (double)s1;
        *qmin = std::min(*qmin, q);
        *qmax = std::max(*qmax, q);
    }
    return true;
}

// Do the RB output rows of every band read at most NR input rows (i_n(a) .. i_n(a') + 1 for
// the band's first / last row a, a'; i_n is monotone in a)?  O(h1).
inline bool tsk_bands_ok(const Geom& g, int RB, int NR) {
    const double ch = (double)(g.h - 1) * 0.5;
    for (int64_t a0 = 0; a0 < g.h1; a0 += RB) {
        const int64_t a1 = std::min<int64_t>(a0 + RB, g.h1) - 1;
        const int64_t i0 = (int64_t)(axis_at(g.xs, a0) + ch), i1 = (int64_t)(axis_at(g.xs, a1) + ch);
        if (i1 - i0 + 2 > NR) return false;
    }
    return true;
}

// Every window of nout output columns: its vertices lie in [floor(qmin + f(b0)) - 1,
// floor(qmax + f(b1)) + 1], checked against the window origin the kernel computes, with a
// margin for the fp64 rounding of j_ and one column for a j_ truncated towards 0 at the left
// edge.  O(w1 / nout).
inline bool tsk_lattice_ok(const Geom& g, int nout, int wc, int al, double qmin, double qmax) {
    const double cw = ((double)g.w - 0.5) * 0.5;
    const int64_t nwin = (g.w1 + nout - 1) / nout;
    for (int64_t wi = 0; wi < nwin; ++wi) {
        const int b0 = (int)(wi * nout);
        const int b1 = (int)std::min<int64_t>(b0 + nout, g.w1) - 1;
        const int x0 = tsk_window_x0(g, qmin, b0, al);
        const int hi = (int)floor(qmax + axis_at(g.ys, b1) + cw + 1e-6) + 2;
        if (hi - x0 > wc - 1) return false;
    }
    return true;
}

}  // namespace hg
