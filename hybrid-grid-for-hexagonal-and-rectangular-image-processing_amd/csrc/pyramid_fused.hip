// pyramid_fused.hip — one hex-pyramid level (BASELINE config 5) on the streaming fused
// kernel (fused_kernel.h, MD 3 from the rect image, MD 4 from a hex image):
//     Z = hexresize(HexConv2d_depthwise(X), (h2, w2))      for a 2x downsample
// The reference chains HexConv2d(C, C, off, 2, padding=1, groups=C) (HexFrames.py:96-169)
// and hexresize (geometry_np.py:520-681, 'linear'), after rect_to_hex (geometry_np.py:
// 358-519, bilinear, same size) for the first level.  The kernel is the headline pipeline's
// row walk — u rows from the rect image (r2h) or the input rows, the 7-tap stencil as packed
// FMAs into three conv-row accumulators — with the hexresize triangle as its output stage:
// every second step completes the two conv rows one output row reads.  Tried first by
// hg_hex_pyramid_level (pyramid.hip); returns HG_EUNSUP outside its domain (then
// k_pyr_stream, then k_pyr_level).  With `dry` nothing is launched and the kernel that
// would run (HG_PYR_FUSED / HG_PYR_FUSED_SHORT) is returned.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "fused_kernel.h"

namespace hg {

template <typename Tin, typename Tout, int C, int MD>
static int pf_launch(const void* x, const float* taps, const float* bias, void* y,
                     const FusedGeom& F, int op, hipStream_t st) {
    const int64_t blocks = F.B * (int64_t)F.nband * ((F.nwin + FU_GW - 1) / FU_GW);
    if (blocks > INT_MAX) return HG_ESHAPE;
    const dim3 grid((unsigned)blocks), blk(FU_THREADS);
    if (op)
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, C, C, 1, MD>), grid, blk, 0, st, (const Tin*)x,
                           taps, bias, (Tout*)y, F);
    else
        hipLaunchKernelGGL((k_fused<Tin, Tout, C, C, C, 0, MD>), grid, blk, 0, st, (const Tin*)x,
                           taps, bias, (Tout*)y, F);
    return launch_status();
}

template <typename Tin, typename Tout>
static int pf_channels(const void* x, const float* taps, const float* bias, void* y,
                       const FusedGeom& F, int C, int md, int op, hipStream_t st) {
#define HG_PF_MD(CC)                                                                          \
    switch (md) {                                                                             \
    case 3: return pf_launch<Tin, Tout, CC, 3>(x, taps, bias, y, F, op, st);                  \
    case 4: return pf_launch<Tin, Tout, CC, 4>(x, taps, bias, y, F, op, st);                  \
    default: return pf_launch<Tin, Tout, CC, 5>(x, taps, bias, y, F, op, st);                 \
    }
    if (C == 3) { HG_PF_MD(3) }
    if (C == 1) { HG_PF_MD(1) }
#undef HG_PF_MD
    return HG_EUNSUP;
}

// The hexresize lattice class the output stage assumes, checked on the lattice itself
// (O(h2 + w2)): i_n(a) - 2a in {0, 1} for every output row, and 1 only where conv row
// i_n(a) + 1 is outside the raster (the kernel has conv row 2a + 2 only one step later);
// 2a + 1 < h1 (the step that outputs row a exists); c0 - 2b in {-1, 0, 1} and
// c1 - 2b in {-2 .. 1} (bounded by the extreme row and column terms plus a margin for the
// fp64 rounding of j_, as k_pyr_stream's check).
static bool pf_lattice_ok(const Geom& g) {
    double qmin = 1e300, qmax = -1e300, gmin = 1e300, gmax = -1e300;
    const double ch = (double)(g.h - 1) * 0.5, cw = ((double)g.w - 0.5) * 0.5;
    for (int64_t a = 0; a < g.h1; ++a) {
        const double i_ = axis_at(g.xs, a) + ch;
        const int64_t in = (int64_t)i_;
        const int64_t e = in - 2 * a;
        if (e < 0 || e > 1 || in < 0 || in >= g.h || 2 * a + 1 >= g.h) return false;
        if (e == 1 && in + 1 < g.h) return false;
        const double q = 0.5 * (i_ - (double)in) - 0.5 * (double)e;
        qmin = std::min(qmin, q);
        qmax = std::max(qmax, q);
    }
    for (int64_t b = 0; b < g.w1; ++b) {
        const double gb = axis_at(g.ys, b) + cw - 2.0 * (double)b;
        gmin = std::min(gmin, gb);
        gmax = std::max(gmax, gb);
    }
    const double eps = 1e-6;
    return qmin + gmin - eps >= -1.0 && qmax + gmax + eps < 2.0;
}

// FR: the same-size rect -> hex lattice is the near-identity one the fused kernel's u rows
// assume (every live tap within one row / column below the sample: in - r, jn - q in {-1, 0})
static bool pf_r2h_ok(const Geom& g) {
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

// The level's geometry and mode (MD 3 from the rect image, MD 4 / 5 from a hex image), or
// HG_EUNSUP outside the kernel's domain.  Shared by the one-level launch and the chain.
static int pf_prepare(const void* src, int src_dtype, int dst_dtype, int64_t batch, int64_t C,
                      int64_t h, int64_t w, int64_t h1, int64_t w1, int from_rect, FusedGeom& F,
                      int& md) {
    if (C != 1 && C != 3) return HG_EUNSUP;
    if ((w & 1) || w < 2 || h < 2 || h1 < 1 || w1 < 1 || batch < 1) return HG_EUNSUP;
    if (src_dtype != HG_F16 && src_dtype != HG_BF16) return HG_EUNSUP;
    if (dst_dtype != src_dtype && dst_dtype != HG_F32) return HG_EUNSUP;
    if (reinterpret_cast<uintptr_t>(src) & 3) return HG_EUNSUP;   // dword loads
    // 32-bit buffer offsets, including the past-the-range loads and stores
    if (C * h * w * 2 >= ((int64_t)1 << 31) || C * h1 * w1 * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;
    const Geom g = make_tri(h, w, h1, w1, 0.5);
    if (!pf_lattice_ok(g)) return HG_EUNSUP;
    F = {};
    F.B = batch;
    F.h = (int)h; F.w = (int)w;           // input (rect for MD 3, hex for MD 4)
    F.h1 = (int)h; F.w1 = (int)w;         // hex / conv image: same size
    F.h2 = (int)h1; F.w2 = (int)w1;       // level output
    F.txs = g.xs;
    F.tys = g.ys;
    if (from_rect) {
        const Geom r = make_r2h(h, w, h, w);
        if (!pf_r2h_ok(r)) return HG_EUNSUP;
        F.rxs = r.xs;
        F.rys = r.ys;
    }
    F.nwin = (int)((w1 + FU_OWN / 2 - 1) / (FU_OWN / 2));
    // From a hex image: a level whose 60-row bands give fewer than six rounds of waves over
    // the chip (256 CUs x 4 SIMDs x 4 waves) runs on short bands (MD 5): the last round of a
    // launch that is only a few rounds long is mostly idle.  A/B switch HYGRID_PYR_SHORT=0/1
    // (exactly "0" or "1"; anything else: the rule above).
    md = from_rect ? 3 : 4;
    if (!from_rect) {
        const int64_t waves = batch * ((h + fu_rb(4) - 1) / fu_rb(4)) * (int64_t)F.nwin;
        bool shrt = waves < 6 * 4096;
        if (env_is("HYGRID_PYR_SHORT", "1")) shrt = true;
        if (env_is("HYGRID_PYR_SHORT", "0")) shrt = false;
        if (shrt) md = 5;
    }
    F.nband = (int)((h + fu_rb(md) - 1) / fu_rb(md));
    return HG_OK;
}

int pyr_fused_try(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t batch,
                  int64_t C, int64_t h, int64_t w, int64_t h1, int64_t w1, const float* taps,
                  const float* bias, int even_odd_offset, int from_rect, hipStream_t st,
                  bool dry) {
    FusedGeom F;
    int md = 0;
    const int rc = pf_prepare(src, src_dtype, dst_dtype, batch, C, h, w, h1, w1, from_rect, F, md);
    if (rc != HG_OK) return rc;
    if (dry) return md == 5 ? HG_PYR_FUSED_SHORT : HG_PYR_FUSED;
    const int op = (even_odd_offset + 1) & 1;   // tap column class at padding 1
    if (src_dtype == HG_F16)
        return dst_dtype == HG_F32 ? pf_channels<_Float16, float>(src, taps, bias, dst, F, (int)C, md, op, st)
                                   : pf_channels<_Float16, _Float16>(src, taps, bias, dst, F, (int)C, md, op, st);
    return dst_dtype == HG_F32 ? pf_channels<__bf16, float>(src, taps, bias, dst, F, (int)C, md, op, st)
                               : pf_channels<__bf16, __bf16>(src, taps, bias, dst, F, (int)C, md, op, st);
}

// ---- the pyramid chain: every level in one launch (round 6) ---------------------------------
// One level per launch pays each launch's ramp and tail (profiles/r06/launch_edges.txt: 50-65,
// 12-16 and 20-22 us of fixed cost for the three config-5 levels, 0.61 ms in all).  The chain
// runs the levels' workgroups in one grid and a workgroup of level l >= 1 starts its band once
// the bands of level l - 1 that wrote its input rows are complete: per (image, band) of every
// producing level a counter of finished window groups.  The hand-off follows the agent-scope
// release / acquire protocol of cdna_hip_programming.md Guideline 16 (no dispatch-order, timing
// or placement assumption):
//   * Work order by ticket: each workgroup draws a ticket (agent atomic) when it starts; tickets
//     0 .. n0 - 1 are level 0's units, then level 1's, then level 2's.  A unit waits only on units
//     of the level before, whose tickets are lower, so their workgroups have started (they are
//     resident or done) and level 0 never waits: no deadlock whatever the dispatch order.  A wait
//     past PC_SPIN polls (~1 s) sets the fault word and goes on (wrong output, never a hang; the
//     tests assert the word is 0).  Within a level the ticket maps through the XCD swizzle (for
//     L2 locality only, as in the one-level launch).
//   * Producer: plain stores; every wave s_waitcnt vmcnt(0); barrier; one lane releases at agent
//     scope (L2 write-back), waits, adds 1 to its band's counter (relaxed, agent).
//   * Consumer: wave 0 polls the counters it needs (relaxed, s_sleep between polls), one lane
//     acquires at agent scope and waits; barrier; then the band's plain loads.
//   * The workspace words (ticket, fault, counters) are zeroed by a memset on the stream before
//     every launch (Guideline 16: re-initialise every call).
constexpr int PC_MAXLEV = 3;
constexpr int PC_SPIN = 1 << 20;
struct PyrChain {
    FusedGeom F[PC_MAXLEV];
    const void* x[PC_MAXLEV];
    void* y[PC_MAXLEV];
    unsigned first[PC_MAXLEV];    // first ticket of each level
    unsigned nblk[PC_MAXLEV];     // units (workgroups) of each level
    int* cnt[PC_MAXLEV];          // level l's (image, band) counters, read by level l + 1
    int* ws;                      // [0] ticket, [1] fault, [2 ...] the counters
    int levels;
};

// workspace ints: ticket, fault, and B x nband counters of every level but the last; padded to
// a multiple of 4 ints (the per-call memset zeroes whole 16-byte blocks)
static int64_t pc_ws_ints(int levels, int64_t batch, int64_t h) {
    int64_t n = 2, hl = h;
    for (int l = 0; l + 1 < levels; ++l) {
        n += batch * ((hl + fu_rb(l == 0 ? 3 : 5) - 1) / fu_rb(l == 0 ? 3 : 5));
        hl /= 2;
    }
    return (n + 3) / 4 * 4;
}

template <typename T, int C, int OP>
__global__ __launch_bounds__(FU_THREADS) __attribute__((amdgpu_waves_per_eu(FU_WPE)))
void k_pyr_chain(const float* __restrict__ kern, const float* __restrict__ bias, PyrChain P) {
    __shared__ FuShared<true, C> sh;
    __shared__ unsigned tk;
    if (threadIdx.x == 0)
        tk = __hip_atomic_fetch_add((unsigned*)P.ws, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned t = tk;
    const int L = (P.levels > 2 && t >= P.first[2]) ? 2 : (t >= P.first[1] ? 1 : 0);   // uniform
    const unsigned n = L == 2 ? P.nblk[2] : L == 1 ? P.nblk[1] : P.nblk[0];
    const int64_t blk = (int64_t)xcd_swizzle(t - (L == 2 ? P.first[2] : L == 1 ? P.first[1] : 0u), n);
    if (L == 0) {
        fu_band<T, T, C, C, C, OP, 3>((const T*)P.x[0], kern, bias, (T*)P.y[0], P.F[0], blk, sh);
    } else {
        // level L's geometry and buffers (selects on kernel arguments, no private copy)
        const FusedGeom& F = L == 2 ? P.F[2] : P.F[1];
        const FusedGeom& Fp = L == 2 ? P.F[1] : P.F[0];    // the producing level
        int* const cnt = L == 2 ? P.cnt[1] : P.cnt[0];
        const int ngrp = (F.nwin + FU_GW - 1) / FU_GW;
        const int64_t rest = blk / ngrp;
        const int band = (int)(rest % F.nband);
        const int64_t b = rest / F.nband;
        if (b < F.B) {
            // input rows the band reads: row(-2) .. row(n + 1), clamped to the raster
            const int s0 = band * fu_rb(5), s1 = min(s0 + fu_rb(5), F.h1);
            const int lo = max(s0 - 2, 0), hi = min(s1 + 1, F.h - 1);
            const int half = (L == 1 ? fu_rb(3) : fu_rb(5)) / 2;   // output rows per producer band
            const int j0 = lo / half, j1 = min(hi / half, Fp.nband - 1);
            const int pgrp = (Fp.nwin + FU_GW - 1) / FU_GW;
            if (threadIdx.x < 64) {                               // wave 0 polls, one lane per band
                if ((int)threadIdx.x <= j1 - j0) {
                    int* const c = cnt + b * Fp.nband + j0 + threadIdx.x;
                    int it = 0;
                    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < pgrp) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++it >= PC_SPIN) {
                            __hip_atomic_store(P.ws + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // this CU's L1 invalidated
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        }
        const T* x = (const T*)(L == 2 ? P.x[2] : P.x[1]);
        T* y = (T*)(L == 2 ? P.y[2] : P.y[1]);
        fu_band<T, T, C, C, C, OP, 5>(x, kern, bias, y, F, blk, sh);
    }
    // this workgroup's band is complete: publish it to the next level
    if (L + 1 < P.levels) {
        const FusedGeom& F = L == 1 ? P.F[1] : P.F[0];
        const int ngrp = (F.nwin + FU_GW - 1) / FU_GW;
        const int64_t rest = blk / ngrp;
        const int64_t b = rest / F.nband;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every wave: its stores done
        __syncthreads();
        if (threadIdx.x == 0 && b < F.B) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // the XCD's L2 written back
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int* const cnt = L == 1 ? P.cnt[1] : P.cnt[0];
            __hip_atomic_fetch_add(cnt + b * F.nband + (int)(rest % F.nband), 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

static int pc_run(const void* src, void* const* dsts, int levels, int dtype, int64_t batch,
                  int64_t C, int64_t h, int64_t w, const float* taps, const float* bias,
                  int even_odd_offset, void* workspace, int64_t ws_bytes, hipStream_t st) {
    if (levels < 1 || batch < 0 || C < 1 || h < 1 || w < 1 || ws_bytes < 0) return HG_EINVAL;
    if (even_odd_offset != 0 && even_odd_offset != 1) return HG_EINVAL;
    if (dtype != HG_F16 && dtype != HG_BF16 && dtype != HG_F32) return HG_EDTYPE;
    if (batch == 0) return HG_OK;
    if (!src || !dsts || !taps) return HG_EINVAL;
    for (int l = 0; l < levels; ++l)
        if (!dsts[l]) return HG_EINVAL;
    if (levels < 2 || levels > PC_MAXLEV || C != 3 || dtype == HG_F32) return HG_EUNSUP;
    PyrChain P = {};
    P.levels = levels;
    int64_t hl = h, wl = w, total = 0;
    for (int l = 0; l < levels; ++l) {
        int md = 0;
        const int rc = pf_prepare(l ? dsts[l - 1] : src, dtype, dtype, batch, C, hl, wl, hl / 2,
                                  wl / 2, l == 0, P.F[l], md);
        if (rc != HG_OK) return rc;
        if (md != (l == 0 ? 3 : 5)) return HG_EUNSUP;
        P.x[l] = l ? dsts[l - 1] : src;
        P.y[l] = dsts[l];
        const int64_t nb = batch * (int64_t)P.F[l].nband * ((P.F[l].nwin + FU_GW - 1) / FU_GW);
        P.first[l] = (unsigned)total;
        P.nblk[l] = (unsigned)nb;
        total += P.nblk[l];
        if (total > INT_MAX) return HG_ESHAPE;
        hl /= 2;
        wl /= 2;
    }
    if (levels == 2) P.first[2] = UINT_MAX;
    const int64_t need = pc_ws_ints(levels, batch, h);
    if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 15) || ws_bytes < need * 4)
        return HG_EINVAL;
    P.ws = (int*)workspace;
    int* c = P.ws + 2;
    for (int l = 0; l + 1 < levels; ++l) {
        P.cnt[l] = c;
        c += batch * P.F[l].nband;
    }
    const int op = (even_odd_offset + 1) & 1;   // tap column class at padding 1
    const int ms = hip_status(hipMemsetAsync(workspace, 0, (size_t)need * 4, st));
    if (ms != HG_OK) return ms;
    const dim3 grid((unsigned)total), blk(FU_THREADS);
    if (dtype == HG_F16) {
        if (op) hipLaunchKernelGGL((k_pyr_chain<_Float16, 3, 1>), grid, blk, 0, st, taps, bias, P);
        else hipLaunchKernelGGL((k_pyr_chain<_Float16, 3, 0>), grid, blk, 0, st, taps, bias, P);
    } else {
        if (op) hipLaunchKernelGGL((k_pyr_chain<__bf16, 3, 1>), grid, blk, 0, st, taps, bias, P);
        else hipLaunchKernelGGL((k_pyr_chain<__bf16, 3, 0>), grid, blk, 0, st, taps, bias, P);
    }
    return launch_status();
}

}  // namespace hg

extern "C" int64_t hg_hex_pyramid_chain_workspace(int levels, int64_t batch, int64_t h) {
    if (levels < 1 || batch < 0 || h < 1) return HG_EINVAL;
    return hg::pc_ws_ints(levels, batch, h) * 4;
}

extern "C" int hg_hex_pyramid_chain(const void* x, void* const* ys, int levels, int dtype,
                                    int64_t batch, int64_t channels, int64_t h, int64_t w,
                                    const float* taps, const float* bias, int even_odd_offset,
                                    void* workspace, int64_t workspace_bytes, void* stream) {
    return hg::pc_run(x, ys, levels, dtype, batch, channels, h, w, taps, bias, even_odd_offset,
                      workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}
