/*
 * hg_oracle.c — CPU restatement of the HyGrid hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path links, loads or calls
 * this file: it is the checker used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Parity is PINNED: tests/test_oracle_golden.py
 * checks every function below against the golden vectors that
 * tests/golden/make_golden.py captured from the reference itself (outputs and
 * the reference's own integer index maps).
 *
 * All citations are /root/reference/<path>:<line>.  The arithmetic follows the
 * reference's NumPy evaluation order exactly, in IEEE fp64, and must be built
 * with -ffp-contract=off (no FMA contraction): the integer lattice maps, the
 * triangle choice and nearest-neighbour ties depend on the last bit.
 *
 * Images are planar, row-major (planes, h, w) float64 — every reference dtype
 * (u8, f16, f32, f64) is exactly representable in fp64, and the reference itself
 * blends in fp64 (geometry_np.py:515-517, :351-354).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_ABI 1
int or_abi_version(void) { return OR_ABI; }

/* numpy.linspace(start, stop, n)[k] (numpy/_core/function_base.py, numpy 2.2):
 * step = (stop-start)/(n-1); y = k*step (or (k/div)*delta when step == 0);
 * y += start; y[-1] = stop.  Two roundings, no FMA. */
double or_linspace(double start, double stop, int64_t n, int64_t k) {
    if (n > 1 && k == n - 1) return stop;
    double delta = stop - start;
    if (n > 1) {
        double div = (double)(n - 1);
        double step = delta / div;
        double y;
        if (step == 0.0) y = ((double)k / div) * delta;
        else y = (double)k * step;
        return y + start;
    }
    return (double)k * delta + start;
}

/* ---------------------------------------------------------------------------
 * rect -> hex (geometry_np.rect_to_hex_resample, geometry_np.py:358-519)
 * ------------------------------------------------------------------------- */
typedef struct {
    int32_t i_n, j_n;      /* :444-445  astype(int) truncates toward zero */
    double i_f, j_f;       /* :448-449  i_ - float32(i_n) */
    int32_t valid;         /* bit k-1 = valid_indices_k, :465-476 */
    int32_t argmin;        /* :499-506 nearest choice (first minimum) */
} r2h_px;

static void r2h_pixel(int64_t h, int64_t w, int64_t h1, int64_t w1, int64_t a, int64_t b,
                      r2h_px* o) {
    /* corners :401-413 */
    double h_inf = -((double)h / 2.0), h_sup = (double)h / 2.0;
    double w_inf = -((double)w / 2.0 + 0.5), w_sup = (double)w / 2.0 + 0.5;
    double x_ = or_linspace(h_inf, h_sup, h1, a);          /* :415-422 */
    double y_ = or_linspace(w_inf, w_sup, w1, b);
    double i_ = x_ + (double)(h - 1) * 0.5;                 /* :440 */
    double j_ = y_ + (double)(w - 1) * 0.5;                 /* :441 */
    int64_t i_n = (int64_t)i_, j_n = (int64_t)j_;
    o->i_n = (int32_t)i_n;
    o->j_n = (int32_t)j_n;
    o->i_f = i_ - (double)(float)i_n;
    o->j_f = j_ - (double)(float)j_n;
    /* neighbours :452-459: 1=(i,j) 2=(i,j+1) 3=(i+1,j) 4=(i+1,j+1) */
    int64_t ii[4] = {i_n, i_n, i_n + 1, i_n + 1};
    int64_t jj[4] = {j_n, j_n + 1, j_n, j_n + 1};
    int32_t v = 0;
    double best = 0.0;
    int32_t arg = 0;
    for (int k = 0; k < 4; ++k) {
        if (ii[k] >= 0 && jj[k] >= 0 && ii[k] < h && jj[k] < w) v |= 1 << k;
        /* :499-502 distance between the CENTRED sample and UN-centred indices */
        double dx = x_ - (double)ii[k], dy = y_ - (double)jj[k];
        double d = dx * dx + dy * dy;
        if (k == 0 || d < best) { best = d; arg = k; }
    }
    o->valid = v;
    o->argmin = arg;
}

void or_r2h_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, int32_t* imaps, double* fmaps) {
    int64_t n = h1 * w1;
    for (int64_t a = 0; a < h1; ++a)
        for (int64_t b = 0; b < w1; ++b) {
            r2h_px p;
            r2h_pixel(h, w, h1, w1, a, b, &p);
            int64_t q = a * w1 + b;
            if (imaps) {
                imaps[0 * n + q] = p.i_n;
                imaps[1 * n + q] = p.j_n;
                imaps[2 * n + q] = 0;
                imaps[3 * n + q] = p.valid;
                imaps[4 * n + q] = p.argmin;
            }
            if (fmaps) {
                fmaps[0 * n + q] = p.i_f;
                fmaps[1 * n + q] = p.j_f;
            }
        }
}

static inline double tap(const double* img, int64_t w, int64_t r, int64_t c, int valid) {
    return valid ? img[r * w + c] : 0.0;   /* :478-486 masked gathers into zeros */
}

void or_rect_to_hex(const double* src, double* dst, int64_t planes, int64_t h, int64_t w,
                    int64_t h1, int64_t w1, int interp) {
#pragma omp parallel for schedule(static)
    for (int64_t a = 0; a < h1; ++a) {
        for (int64_t b = 0; b < w1; ++b) {
            r2h_px p;
            r2h_pixel(h, w, h1, w1, a, b, &p);
            int64_t i = p.i_n, j = p.j_n;
            for (int64_t pl = 0; pl < planes; ++pl) {
                const double* img = src + pl * h * w;
                double p1 = tap(img, w, i, j, p.valid & 1);
                double p2 = tap(img, w, i, j + 1, p.valid & 2);
                double p3 = tap(img, w, i + 1, j, p.valid & 4);
                double p4 = tap(img, w, i + 1, j + 1, p.valid & 8);
                double out;
                if (interp == 0) {            /* :508-512 */
                    double pk[4] = {p1, p2, p3, p4};
                    out = pk[p.argmin];
                } else {                      /* :514-517 */
                    double t1 = p.i_f * p3 + (1.0 - p.i_f) * p1;
                    double t2 = p.i_f * p4 + (1.0 - p.i_f) * p2;
                    out = p.j_f * t2 + (1.0 - p.j_f) * t1;
                }
                dst[pl * h1 * w1 + a * w1 + b] = out;
            }
        }
    }
}

/* ---------------------------------------------------------------------------
 * hex -> rect (geometry_np.hex_to_rect_resample, :191-356) and hex -> hex
 * (geometry_np.hexresize, :520-681).  The two differ only in the column bound
 * of the sample lattice: -((w+.5)/2 - .75) (:236-239) vs -((w+.5)/2 - .5)
 * (:560-563).  The nearest rule is geometry_torch.hex_to_square_resample's
 * (geometry_torch.py:335-347): argmin over the 3 triangle vertices, first min.
 * ------------------------------------------------------------------------- */
typedef struct {
    int32_t i_n, j_n, flag, valid, argmin;
    int64_t r[3], c[3];          /* p1, p2 (chosen), p3 */
    int32_t vk[3];               /* validity of p1, p2, p3 */
    double i_f, j_f, alpha, beta, gamma;
} tri_px;

static void tri_pixel(int64_t h, int64_t w, int64_t h1, int64_t w1, int64_t a, int64_t b,
                      double w_margin, tri_px* o) {
    double hh = (double)h, ww = (double)w;
    double h_inf = -(hh / 2.0 - 0.5), h_sup = hh / 2.0 - 0.5;
    double w_inf = -((ww + 0.5) / 2.0 - w_margin), w_sup = (ww + 0.5) / 2.0 - w_margin;
    double x_ = or_linspace(h_inf, h_sup, h1, a);           /* :251-258 */
    double y_ = or_linspace(w_inf, w_sup, w1, b);
    double i_ = x_ + (double)(h - 1) * 0.5;                  /* :276 */
    double j_ = 0.5 * i_ + y_ + (ww - 0.5) * 0.5;            /* :277 */
    int64_t i_n = (int64_t)i_, j_n = (int64_t)j_;            /* :280-281 */
    double i_f = i_ - (double)(float)i_n;                    /* :284-285 */
    double j_f = j_ - (double)(float)j_n;
    /* :288-295 — ((i_n+1)/2).astype(int): true division then truncation */
    int64_t s1 = (int64_t)((double)(i_n + 1) / 2.0);
    int64_t s2 = (int64_t)((double)(i_n + 2) / 2.0);
    int64_t ii[4] = {i_n, i_n + 1, i_n, i_n + 1};
    int64_t jj[4] = {j_n - s1, j_n - s2, j_n + 1 - s1, j_n + 1 - s2};
    int flag = i_f > j_f;                                    /* :298 */
    int32_t v = 0;
    for (int k = 0; k < 4; ++k)
        if (ii[k] >= 0 && jj[k] >= 0 && ii[k] < h && jj[k] < w) v |= 1 << k;
    o->i_n = (int32_t)i_n;
    o->j_n = (int32_t)j_n;
    o->flag = flag;
    o->valid = v;
    o->i_f = i_f;
    o->j_f = j_f;
    /* p1 = 1, p2 = flag ? 2 : 3, p3 = 4   (:320-323) */
    int k2 = flag ? 1 : 2;
    o->r[0] = ii[0]; o->c[0] = jj[0]; o->vk[0] = (v >> 0) & 1;
    o->r[1] = ii[k2]; o->c[1] = jj[k2]; o->vk[1] = (v >> k2) & 1;
    o->r[2] = ii[3]; o->c[2] = jj[3]; o->vk[2] = (v >> 3) & 1;
    /* cartesian vertices :326-331 */
    double fl = (double)flag, in = (double)i_n, jn = (double)j_n;
    double p1_x = in - (hh - 1.0) / 2.0;
    double p1_y = jn - in / 2.0 - (ww - 0.5) / 2.0;
    double p2_x = (in + fl) - (hh - 1.0) / 2.0;
    double p2_y = (jn + 1.0 - fl) - (in + fl) / 2.0 - (ww - 0.5) / 2.0;
    double p3_x = (in + 1.0) - (hh - 1.0) / 2.0;
    double p3_y = (jn + 1.0) - (in + 1.0) / 2.0 - (ww - 0.5) / 2.0;
    /* nearest :334-339 (torch twin :336-341) */
    double d1 = (x_ - p1_x) * (x_ - p1_x) + (y_ - p1_y) * (y_ - p1_y);
    double d2 = (x_ - p2_x) * (x_ - p2_x) + (y_ - p2_y) * (y_ - p2_y);
    double d3 = (x_ - p3_x) * (x_ - p3_x) + (y_ - p3_y) * (y_ - p3_y);
    int arg = 0;
    double best = d1;
    if (d2 < best) { best = d2; arg = 1; }
    if (d3 < best) { best = d3; arg = 2; }
    o->argmin = arg;
    /* barycentric :348-353 */
    double S1 = 0.5 * fabs((x_ - p2_x) * (y_ - p3_y) - (y_ - p2_y) * (x_ - p3_x));
    double S2 = 0.5 * fabs((x_ - p1_x) * (y_ - p3_y) - (y_ - p1_y) * (x_ - p3_x));
    double S3 = 0.5 * fabs((x_ - p1_x) * (y_ - p2_y) - (y_ - p1_y) * (x_ - p2_x));
    double S = S1 + S2 + S3;
    o->alpha = S1 / S;
    o->beta = S2 / S;
    o->gamma = S3 / S;
}

static void tri_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, double margin,
                     int32_t* imaps, double* fmaps) {
    int64_t n = h1 * w1;
    for (int64_t a = 0; a < h1; ++a)
        for (int64_t b = 0; b < w1; ++b) {
            tri_px p;
            tri_pixel(h, w, h1, w1, a, b, margin, &p);
            int64_t q = a * w1 + b;
            if (imaps) {
                imaps[0 * n + q] = p.i_n;
                imaps[1 * n + q] = p.j_n;
                imaps[2 * n + q] = p.flag;
                imaps[3 * n + q] = p.valid;
                imaps[4 * n + q] = p.argmin;
            }
            if (fmaps) {
                fmaps[0 * n + q] = p.i_f;
                fmaps[1 * n + q] = p.j_f;
                fmaps[2 * n + q] = p.alpha;
                fmaps[3 * n + q] = p.beta;
                fmaps[4 * n + q] = p.gamma;
            }
        }
}

void or_h2r_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, int32_t* imaps, double* fmaps) {
    tri_maps(h, w, h1, w1, 0.75, imaps, fmaps);
}
void or_hexresize_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, int32_t* imaps,
                       double* fmaps) {
    tri_maps(h, w, h1, w1, 0.5, imaps, fmaps);
}

static void tri_resample(const double* src, double* dst, int64_t planes, int64_t h, int64_t w,
                         int64_t h1, int64_t w1, int interp, double margin) {
#pragma omp parallel for schedule(static)
    for (int64_t a = 0; a < h1; ++a) {
        for (int64_t b = 0; b < w1; ++b) {
            tri_px p;
            tri_pixel(h, w, h1, w1, a, b, margin, &p);
            for (int64_t pl = 0; pl < planes; ++pl) {
                const double* img = src + pl * h * w;
                double v[3];
                for (int k = 0; k < 3; ++k) v[k] = tap(img, w, p.r[k], p.c[k], p.vk[k]);
                double out;
                if (interp == 0) out = v[p.argmin];
                else out = p.alpha * v[0] + p.beta * v[1] + p.gamma * v[2];   /* :354 */
                dst[pl * h1 * w1 + a * w1 + b] = out;
            }
        }
    }
}

void or_hex_to_rect(const double* src, double* dst, int64_t planes, int64_t h, int64_t w,
                    int64_t h1, int64_t w1, int interp) {
    tri_resample(src, dst, planes, h, w, h1, w1, interp, 0.75);
}
void or_hexresize(const double* src, double* dst, int64_t planes, int64_t h, int64_t w,
                  int64_t h1, int64_t w1, int interp) {
    tri_resample(src, dst, planes, h, w, h1, w1, interp, 0.5);
}

/* ---------------------------------------------------------------------------
 * Adjoints of the three resamplers (the reference gets them from torch autograd
 * through the indexing of geometry_torch.py:322-325; geometry_np.py:514-517 and
 * :347-354 give the weights): gx = R^T gy.  Every output sample scatters its
 * gradient onto the taps it read, with the forward's fp64 weights (bilinear:
 * (1-fi)(1-fj), (1-fi)fj, fi(1-fj), fi*fj as products of the two blend stages;
 * triangle: alpha, beta, gamma; nearest: 1 on the chosen tap).  Invalid taps
 * (zero in the forward) receive nothing.  Planes are independent, so the plane
 * loop is the parallel one and the scatter order inside a plane is sequential
 * (deterministic).
 * ------------------------------------------------------------------------- */
static inline void add_tap(double* g, int64_t w, int64_t r, int64_t c, int valid, double v) {
    if (valid) g[r * w + c] += v;
}

void or_rect_to_hex_backward(const double* gy, double* gx, int64_t planes, int64_t h, int64_t w,
                             int64_t h1, int64_t w1, int interp) {
#pragma omp parallel for schedule(static)
    for (int64_t pl = 0; pl < planes; ++pl) {
        double* g = gx + pl * h * w;
        const double* gp = gy + pl * h1 * w1;
        memset(g, 0, (size_t)(h * w) * sizeof(double));
        for (int64_t a = 0; a < h1; ++a)
            for (int64_t b = 0; b < w1; ++b) {
                r2h_px p;
                r2h_pixel(h, w, h1, w1, a, b, &p);
                const int64_t i = p.i_n, j = p.j_n;
                const double go = gp[a * w1 + b];
                if (interp == 0) {                 /* :508-512: the chosen neighbour */
                    const int k = p.argmin;
                    add_tap(g, w, i + (k >> 1), j + (k & 1), (p.valid >> k) & 1, go);
                } else {                           /* :514-517: out = fj*t2 + (1-fj)*t1 */
                    const double gt1 = (1.0 - p.j_f) * go, gt2 = p.j_f * go;
                    add_tap(g, w, i, j, p.valid & 1, (1.0 - p.i_f) * gt1);
                    add_tap(g, w, i, j + 1, p.valid & 2, (1.0 - p.i_f) * gt2);
                    add_tap(g, w, i + 1, j, p.valid & 4, p.i_f * gt1);
                    add_tap(g, w, i + 1, j + 1, p.valid & 8, p.i_f * gt2);
                }
            }
    }
}

static void tri_backward(const double* gy, double* gx, int64_t planes, int64_t h, int64_t w,
                         int64_t h1, int64_t w1, int interp, double margin) {
#pragma omp parallel for schedule(static)
    for (int64_t pl = 0; pl < planes; ++pl) {
        double* g = gx + pl * h * w;
        const double* gp = gy + pl * h1 * w1;
        memset(g, 0, (size_t)(h * w) * sizeof(double));
        for (int64_t a = 0; a < h1; ++a)
            for (int64_t b = 0; b < w1; ++b) {
                tri_px p;
                tri_pixel(h, w, h1, w1, a, b, margin, &p);
                const double go = gp[a * w1 + b];
                if (interp == 0) {
                    const int k = p.argmin;
                    add_tap(g, w, p.r[k], p.c[k], p.vk[k], go);
                } else {                           /* :354 */
                    const double wt[3] = {p.alpha, p.beta, p.gamma};
                    for (int k = 0; k < 3; ++k) add_tap(g, w, p.r[k], p.c[k], p.vk[k], wt[k] * go);
                }
            }
    }
}

void or_hex_to_rect_backward(const double* gy, double* gx, int64_t planes, int64_t h, int64_t w,
                             int64_t h1, int64_t w1, int interp) {
    tri_backward(gy, gx, planes, h, w, h1, w1, interp, 0.75);
}
void or_hexresize_backward(const double* gy, double* gx, int64_t planes, int64_t h, int64_t w,
                           int64_t h1, int64_t w1, int interp) {
    tri_backward(gy, gx, planes, h, w, h1, w1, interp, 0.5);
}

/* ---------------------------------------------------------------------------
 * HexConv2d (HexFrames.py:22-185, heximage_to_type1 :417-445, pad :13-21)
 *
 * Restated without materialising the type1 image.  With P = pad(x, p), H' = H+2p,
 * W' = W+2p, o' = (off+p)%2 (:44), type1 row y holds P[y,k] at columns
 * 2k+L(y) and 2k+1+L(y), L(y) = (y%2 + o')%2 (:429-438), zero elsewhere.  The
 * dense kernel (:108-118) puts tap m of kernel row ii at column t*d + 2*d*m,
 * t = |ii-r+1|, row ii*d.  The even/odd strided convs (:127-146) interleaved
 * (:157-162) give, for output row ro and column q:
 *     y   = s*ro + ii*d
 *     x   = 1 + (ro odd ? s : 0) + 2*s*q + t*d + 2*d*m     (type1 column)
 *     val = (x - L(y) <= 2W'-1) ? P[y, (x-L(y))>>1] : 0
 * Output rows: floor((H'-k_h)/s)+1; cols: floor((2W'-s-k_w)/(2s))+1.
 * ------------------------------------------------------------------------- */
enum { OR_PAD_CONSTANT = 0, OR_PAD_REFLECT = 1, OR_PAD_REPLICATE = 2, OR_PAD_CIRCULAR = 3 };

int or_hexconv2d_out_shape(int64_t h, int64_t w, int r, int s, int p, int d, int64_t* ho,
                           int64_t* wo) {
    if (r < 1 || s < 1 || d < 1 || p < 0) return -1;
    int64_t kh = (int64_t)(2 * r - 2) * d + 1;
    int64_t kw = (int64_t)2 * d * (2 * r - 2) + 1;
    int64_t H = h + 2 * p, W = w + 2 * p;
    /* both strided convs need >= k_h rows and >= k_w cols (:127-146);
     * with only the even conv valid the result is its single row (:163-164) */
    if (H < kh || 2 * W - s < kw) return -3;
    *ho = (H - kh) / s + 1;
    *wo = (2 * W - s - kw) / (2 * s) + 1;
    return 0;
}

static inline int64_t pad_index(int64_t i, int64_t n, int mode) {
    if (i >= 0 && i < n) return i;
    switch (mode) {
    case OR_PAD_REFLECT:   /* torch 'reflect': mirror without repeating the edge */
        while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * (n - 1) - i; }
        return i;
    case OR_PAD_REPLICATE:
        return i < 0 ? 0 : n - 1;
    case OR_PAD_CIRCULAR:
        return ((i % n) + n) % n;
    default:
        return -1;
    }
}

/* torch F.pad's rules for the non-constant modes (the reference pads with F.pad,
 * HexFrames.py:13-21): reflect needs padding < size, circular padding <= size.  Outside
 * them torch raises; the mirror loop of pad_index would not terminate. */
static int pad_args_ok(int64_t h, int64_t w, int p, int mode) {
    if (mode == OR_PAD_REFLECT && p > 0 && (p >= h || p >= w)) return 0;
    if (mode != OR_PAD_CONSTANT && p > 0 && (h == 0 || w == 0)) return 0;
    if (mode == OR_PAD_CIRCULAR && (p > h || p > w)) return 0;
    return 1;
}

int or_hexconv2d(const double* x, const double* kern, const double* bias, double* y,
                 int64_t B, int64_t C, int64_t O, int64_t h, int64_t w, int r, int s, int p,
                 int d, int groups, int off, int pad_mode, double pad_value) {
    int64_t ho, wo;
    int st = or_hexconv2d_out_shape(h, w, r, s, p, d, &ho, &wo);
    if (st == 0 && !pad_args_ok(h, w, p, pad_mode)) st = -2;
    if (st) return st;
    if (groups < 1 || C % groups || O % groups) return -1;
    int K = 3 * r * r - 3 * r + 1;                    /* :52 */
    int64_t cg = C / groups, og = O / groups;
    int64_t Wp = w + 2 * p;
    int op = (off + p) % 2;
    /* tap table: (ii, t*d + 2*d*m) in kernel flattening order (:114-118) */
    int* tii = (int*)malloc(sizeof(int) * K);
    int* tcol = (int*)malloc(sizeof(int) * K);
    int n = 0;
    for (int ii = 0; ii < 2 * r - 1; ++ii) {
        int t = abs(ii - r + 1), ln = 2 * r - 1 - t;
        for (int m = 0; m < ln; ++m) { tii[n] = ii; tcol[n] = t * d + 2 * d * m; ++n; }
    }
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t bo = 0; bo < B * O; ++bo) {
        for (int64_t ro = 0; ro < ho; ++ro) {
            int64_t b = bo / O, o = bo % O, g = o / og;
            for (int64_t q = 0; q < wo; ++q) {
                double acc = 0.0;
                for (int64_t ci = 0; ci < cg; ++ci) {
                    int64_t c = g * cg + ci;
                    const double* xin = x + (b * C + c) * h * w;
                    const double* kk = kern + (o * cg + ci) * K;
                    for (int t = 0; t < K; ++t) {
                        int64_t yy = s * ro + (int64_t)tii[t] * d;
                        int64_t xx = 1 + ((ro & 1) ? s : 0) + 2 * s * q + tcol[t];
                        int64_t L = ((yy & 1) + op) & 1;
                        int64_t u = xx - L;
                        if (u > 2 * Wp - 1) continue;          /* type1 structural zero */
                        int64_t k = u >> 1;
                        int64_t yi = yy - p, xi = k - p;       /* un-padded coordinates */
                        double v;
                        int64_t ry = pad_index(yi, h, pad_mode), rx = pad_index(xi, w, pad_mode);
                        if (pad_mode == OR_PAD_CONSTANT && (ry < 0 || rx < 0)) v = pad_value;
                        else v = xin[ry * w + rx];
                        acc += kk[t] * v;
                    }
                }
                if (bias) acc += bias[o];
                y[((b * O + o) * ho + ro) * wo + q] = acc;
            }
        }
    }
    free(tii);
    free(tcol);
    return 0;
}

/* HexConv2d backward: the exact adjoint of or_hexconv2d's index map (the reference
 * gets it from torch autograd through pad -> heximage_to_type1 -> two strided
 * F.conv2d -> interleave, HexFrames.py:96-169).  For every output sample and tap
 * the forward reads one padded sample P[yy][k]; its input pixel (after the padding
 * mode's index map, pad_index) receives kern*gy, the tap's weight receives
 * gy*value, the bias receives gy.  Constant-mode padding samples have no input
 * pixel (their value is the constant).  Serial in (b, o) so the accumulation order
 * is fixed.  dx / dk / db may be NULL; they are overwritten (not accumulated). */
int or_hexconv2d_backward(const double* x, const double* kern, const double* gy, double* dx,
                          double* dk, double* db, int64_t B, int64_t C, int64_t O, int64_t h,
                          int64_t w, int r, int s, int p, int d, int groups, int off,
                          int pad_mode, double pad_value) {
    int64_t ho, wo;
    int st = or_hexconv2d_out_shape(h, w, r, s, p, d, &ho, &wo);
    if (st == 0 && !pad_args_ok(h, w, p, pad_mode)) st = -2;
    if (st) return st;
    if (groups < 1 || C % groups || O % groups) return -1;
    int K = 3 * r * r - 3 * r + 1;
    int64_t cg = C / groups, og = O / groups;
    int64_t Wp = w + 2 * p;
    int op = (off + p) % 2;
    int* tii = (int*)malloc(sizeof(int) * K);
    int* tcol = (int*)malloc(sizeof(int) * K);
    int n = 0;
    for (int ii = 0; ii < 2 * r - 1; ++ii) {
        int t = abs(ii - r + 1), ln = 2 * r - 1 - t;
        for (int m = 0; m < ln; ++m) { tii[n] = ii; tcol[n] = t * d + 2 * d * m; ++n; }
    }
    if (dx) memset(dx, 0, sizeof(double) * (size_t)(B * C * h * w));
    if (dk) memset(dk, 0, sizeof(double) * (size_t)(O * cg * K));
    if (db) memset(db, 0, sizeof(double) * (size_t)O);
    for (int64_t b = 0; b < B; ++b)
        for (int64_t o = 0; o < O; ++o) {
            int64_t g = o / og;
            for (int64_t ro = 0; ro < ho; ++ro)
                for (int64_t q = 0; q < wo; ++q) {
                    double gv = gy[((b * O + o) * ho + ro) * wo + q];
                    if (db) db[o] += gv;
                    for (int64_t ci = 0; ci < cg; ++ci) {
                        int64_t c = g * cg + ci;
                        const double* xin = x + (b * C + c) * h * w;
                        for (int t = 0; t < K; ++t) {
                            int64_t yy = s * ro + (int64_t)tii[t] * d;
                            int64_t xx = 1 + ((ro & 1) ? s : 0) + 2 * s * q + tcol[t];
                            int64_t L = ((yy & 1) + op) & 1;
                            int64_t u = xx - L;
                            if (u > 2 * Wp - 1) continue;      /* type1 structural zero */
                            int64_t k = u >> 1;
                            int64_t ry = pad_index(yy - p, h, pad_mode);
                            int64_t rx = pad_index(k - p, w, pad_mode);
                            int inside = !(pad_mode == OR_PAD_CONSTANT && (ry < 0 || rx < 0));
                            double v = inside ? xin[ry * w + rx] : pad_value;
                            if (dk) dk[(o * cg + ci) * K + t] += gv * v;
                            if (dx && inside)
                                dx[(b * C + c) * h * w + ry * w + rx] += kern[(o * cg + ci) * K + t] * gv;
                        }
                    }
                }
        }
    free(tii);
    free(tcol);
    return 0;
}

/* heximage_to_type1 (HexFrames.py:417-445): (planes,h,w) -> (planes,h,2w+1) */
void or_heximage_to_type1(const double* x, double* t, int64_t planes, int64_t h, int64_t w,
                          int off) {
    int64_t W2 = 2 * w + 1;
    for (int64_t pl = 0; pl < planes; ++pl)
        for (int64_t yy = 0; yy < h; ++yy) {
            int L = (int)(((yy & 1) + off) & 1);
            double* row = t + (pl * h + yy) * W2;
            for (int64_t u = 0; u < W2; ++u) row[u] = 0.0;
            for (int64_t k = 0; k < w; ++k)
                row[2 * k + L] = row[2 * k + 1 + L] = x[(pl * h + yy) * w + k];
        }
}

int or_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void or_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
