// Host check: tri_sample_fast (32-bit lattice indices, no speculated division) returns the
// same triangle samples as tri_sample, field for field, for every output sample of a set of
// hex->rect / hexresize geometries (lattice.h; used by k_tri_up and k_hexresize_down).
#include "lattice.h"
#include <cstdio>
#include <cstring>
using namespace hg;
int main() {
    const int shapes[][4] = {{60, 100, 120, 200}, {2, 2, 4, 4},       {5, 10, 10, 19},
                             {100, 1000, 200, 2000}, {40, 96, 41, 97}, {33, 260, 65, 520},
                             {1080, 1920, 2160, 3840}, {2160, 3840, 1080, 1920}, {17, 40, 34, 80}};
    long total = 0, bad = 0;
    for (const auto& sh : shapes)
        for (double m : {0.5, 0.75}) {
            const Geom g = make_tri(sh[0], sh[1], sh[2], sh[3], m);
            if (!tri_fast_ok(g)) { printf("not fast_ok: %d %d %d %d\n", sh[0], sh[1], sh[2], sh[3]); return 2; }
            for (int a = 0; a < sh[2]; ++a)
                for (int b = 0; b < sh[3]; ++b) {
                    const TriSample s = tri_sample(g, a, b), f = tri_sample_fast(g, a, b);
                    ++total;
                    if (s.i_n != f.i_n || s.j_n != f.j_n || memcmp(s.r, f.r, sizeof s.r) ||
                        memcmp(s.c, f.c, sizeof s.c) || s.vk != f.vk || s.flag != f.flag ||
                        s.valid != f.valid || s.argmin != f.argmin ||
                        memcmp(&s.i_f, &f.i_f, 8) || memcmp(&s.j_f, &f.j_f, 8) ||
                        memcmp(&s.alpha, &f.alpha, 8) || memcmp(&s.beta, &f.beta, 8) ||
                        memcmp(&s.gamma, &f.gamma, 8))
                        ++bad;
                }
        }
    printf("%ld samples, %ld differ\n", total, bad);
    return bad ? 1 : 0;
}
