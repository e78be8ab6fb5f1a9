/*
 * selftest.c — memory-safety and identity checks of the CPU restatement (hg_oracle.c),
 * built with -fsanitize=address,undefined by `make -C oracle asan` and run by
 * tests/test_oracle_asan.py.  TEST INFRASTRUCTURE ONLY (see hg_oracle.c's header).
 *
 * Every entry point runs on the edge shapes the reference's callers reach: 1x1 and
 * 1xN rasters, odd and even sizes, strong down- and up-sampling (tiles whose taps
 * fall off the raster), zero planes, every HexConv2d radius / stride / dilation /
 * padding mode the goldens cover.  Besides "no out-of-bounds access, no UB", each
 * resampler's adjoint is checked against its forward: <R x, g> == <x, R^T g> in fp64
 * (relative 1e-12), which ties or_*_backward to the pinned forwards.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void or_rect_to_hex(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_hex_to_rect(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_hexresize(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_rect_to_hex_backward(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_hex_to_rect_backward(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_hexresize_backward(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);
void or_r2h_maps(int64_t, int64_t, int64_t, int64_t, int32_t*, double*);
void or_h2r_maps(int64_t, int64_t, int64_t, int64_t, int32_t*, double*);
void or_hexresize_maps(int64_t, int64_t, int64_t, int64_t, int32_t*, double*);
int or_hexconv2d_out_shape(int64_t, int64_t, int, int, int, int, int64_t*, int64_t*);
int or_hexconv2d(const double*, const double*, const double*, double*, int64_t, int64_t, int64_t,
                 int64_t, int64_t, int, int, int, int, int, int, int, double);
int or_hexconv2d_backward(const double*, const double*, const double*, double*, double*, double*,
                          int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int, int, int, int,
                          int, double);
void or_heximage_to_type1(const double*, double*, int64_t, int64_t, int64_t, int);

typedef void (*resample_fn)(const double*, double*, int64_t, int64_t, int64_t, int64_t, int64_t, int);

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static double urand(void) {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (double)(rng >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}
static double* fresh(int64_t n) {
    double* p = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int64_t i = 0; i < n; ++i) p[i] = urand();
    return p;
}
static double dot(const double* a, const double* b, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

static int fails = 0;

static void adjoint(const char* name, resample_fn fwd, resample_fn bwd, int64_t planes, int64_t h,
                    int64_t w, int64_t h1, int64_t w1, int interp) {
    double* x = fresh(planes * h * w);
    double* y = fresh(planes * h1 * w1);
    double* g = fresh(planes * h1 * w1);
    double* gx = fresh(planes * h * w);
    fwd(x, y, planes, h, w, h1, w1, interp);
    bwd(g, gx, planes, h, w, h1, w1, interp);
    const double lhs = dot(y, g, planes * h1 * w1), rhs = dot(x, gx, planes * h * w);
    const double scale = fabs(lhs) > 1e-300 ? fabs(lhs) : 1.0;
    if (!(fabs(lhs - rhs) <= 1e-12 * scale + 1e-300)) {
        printf("FAIL %s adjoint %lldx%lld -> %lldx%lld interp %d: %.17g vs %.17g\n", name,
               (long long)h, (long long)w, (long long)h1, (long long)w1, interp, lhs, rhs);
        ++fails;
    }
    free(x); free(y); free(g); free(gx);
}

static void maps(int64_t h, int64_t w, int64_t h1, int64_t w1) {
    const int64_t n = h1 * w1;
    int32_t* im = (int32_t*)malloc((size_t)(5 * n + 1) * sizeof(int32_t));
    double* fm = (double*)malloc((size_t)(5 * n + 1) * sizeof(double));
    or_r2h_maps(h, w, h1, w1, im, fm);
    or_h2r_maps(h, w, h1, w1, im, fm);
    or_hexresize_maps(h, w, h1, w1, im, fm);
    free(im); free(fm);
}

static void conv(int64_t B, int64_t C, int64_t O, int64_t h, int64_t w, int r, int s, int p,
                 int d, int groups, int off, int mode) {
    int64_t ho, wo;
    if (or_hexconv2d_out_shape(h, w, r, s, p, d, &ho, &wo) != 0 || ho <= 0 || wo <= 0) return;
    if (getenv("ST_TRACE")) printf("conv %lldx%lld r%d s%d p%d d%d g%d off%d mode%d -> %lldx%lld\n", (long long)h, (long long)w, r, s, p, d, groups, off, mode, (long long)ho, (long long)wo);
    const int64_t K = 3 * r * r - 3 * r + 1;
    double* x = fresh(B * C * h * w);
    double* k = fresh(O * (C / groups) * K);
    double* b = fresh(O);
    double* y = fresh(B * O * ho * wo);
    double* gy = fresh(B * O * ho * wo);
    double* dx = fresh(B * C * h * w);
    double* dk = fresh(O * (C / groups) * K);
    double* db = fresh(O);
    const int bad_pad = (mode == 1 && p > 0 && (p >= h || p >= w)) || (mode == 3 && (p > h || p > w));
    if (bad_pad) {   /* torch raises for these pads: the restatement must refuse, not loop */
        if (or_hexconv2d(x, k, b, y, B, C, O, h, w, r, s, p, d, groups, off, mode, 0.25) == 0 ||
            or_hexconv2d_backward(x, k, gy, dx, dk, db, B, C, O, h, w, r, s, p, d, groups, off,
                                  mode, 0.25) == 0) {
            printf("FAIL conv accepted an invalid pad: mode %d p%d on %lldx%lld\n", mode, p,
                   (long long)h, (long long)w);
            ++fails;
        }
        free(x); free(k); free(b); free(y); free(gy); free(dx); free(dk); free(db);
        return;
    }
    if (or_hexconv2d(x, k, b, y, B, C, O, h, w, r, s, p, d, groups, off, mode, 0.25) != 0) {
        printf("FAIL conv r%d s%d p%d d%d g%d mode %d on %lldx%lld\n", r, s, p, d, groups, mode,
               (long long)h, (long long)w);
        ++fails;
    }
    or_hexconv2d_backward(x, k, gy, dx, dk, db, B, C, O, h, w, r, s, p, d, groups, off, mode, 0.25);
    /* constant padding with value 0 is linear in x: <conv0(x), gy> == <x, dx> */
    if (mode == 0) {
        double* y0 = fresh(B * O * ho * wo);
        or_hexconv2d(x, k, NULL, y0, B, C, O, h, w, r, s, p, d, groups, off, 0, 0.0);
        or_hexconv2d_backward(x, k, gy, dx, NULL, NULL, B, C, O, h, w, r, s, p, d, groups, off, 0, 0.0);
        const double lhs = dot(y0, gy, B * O * ho * wo), rhs = dot(x, dx, B * C * h * w);
        if (!(fabs(lhs - rhs) <= 1e-12 * (fabs(lhs) + 1e-300))) {
            printf("FAIL conv adjoint r%d s%d p%d d%d g%d: %.17g vs %.17g\n", r, s, p, d, groups,
                   lhs, rhs);
            ++fails;
        }
        free(y0);
    }
    free(x); free(k); free(b); free(y); free(gy); free(dx); free(dk); free(db);
}

int main(void) {
    setvbuf(stdout, NULL, _IONBF, 0);
    static const int64_t shapes[][4] = {
        {1, 1, 1, 1}, {1, 7, 1, 7}, {7, 1, 7, 1}, {2, 2, 2, 2}, {16, 20, 8, 10}, {15, 17, 15, 17},
        {9, 12, 20, 25}, {33, 64, 5, 3}, {5, 3, 33, 64}, {64, 96, 64, 96}, {40, 70, 20, 35},
        {43, 77, 21, 38}, {3, 200, 60, 9}};
    const int ns = (int)(sizeof shapes / sizeof shapes[0]);
    for (int i = 0; i < ns; ++i) {
        const int64_t h = shapes[i][0], w = shapes[i][1], h1 = shapes[i][2], w1 = shapes[i][3];
        maps(h, w, h1, w1);
        for (int interp = 0; interp < 2; ++interp) {
            adjoint("rect_to_hex", or_rect_to_hex, or_rect_to_hex_backward, 2, h, w, h1, w1, interp);
            adjoint("hex_to_rect", or_hex_to_rect, or_hex_to_rect_backward, 2, h, w, h1, w1, interp);
            adjoint("hexresize", or_hexresize, or_hexresize_backward, 2, h, w, h1, w1, interp);
        }
        /* zero planes: nothing read or written */
        or_rect_to_hex(NULL, NULL, 0, h, w, h1, w1, 1);
        or_hex_to_rect_backward(NULL, NULL, 0, h, w, h1, w1, 1);
    }
    static const int64_t cshapes[][2] = {{1, 1}, {2, 3}, {7, 9}, {8, 10}, {13, 6}};
    for (int i = 0; i < 5; ++i)
        for (int r = 2; r <= 4; ++r)
            for (int s = 1; s <= 2; ++s)
                for (int p = 0; p <= 2; ++p)
                    for (int d = 1; d <= 2; ++d)
                        for (int mode = 0; mode < 4; ++mode)
                            for (int off = 0; off < 2; ++off) {
                                conv(2, 3, 3, cshapes[i][0], cshapes[i][1], r, s, p, d, 1, off, mode);
                                conv(1, 3, 6, cshapes[i][0], cshapes[i][1], r, s, p, d, 3, off, mode);
                            }
    double* x = fresh(2 * 5 * 7);
    double* t = fresh(2 * 5 * 15);
    or_heximage_to_type1(x, t, 2, 5, 7, 1);
    free(x); free(t);
    printf(fails ? "selftest: %d FAILURES\n" : "selftest: ok\n", fails);
    return fails ? 1 : 0;
}
