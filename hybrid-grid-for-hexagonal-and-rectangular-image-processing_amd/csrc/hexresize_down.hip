// hexresize_down.hip — triangle-blend resamples (hexresize, geometry_np.py:520-681, and
// hex_to_rect_resample, :191-356, 'linear') on a row-streaming kernel, for the lattices whose
// triangle vertices for a run of output columns fit one 128-column window of input columns:
// every pyramid level's ~2x hexresize (BASELINE config 5's operator chain, one output column
// per lane) and the inverse of ConvertToHexagon's lattice, hex (h/2, w/2) -> rect (h, w)
// (Image.py:111-116 read backwards; two output columns per lane).  Bit-identical to
// k_resample_lds (resample.hip) for the same call: the same fp64 triangle records (lattice.h
// tri_sample, the reference's expression order) cast to the accumulator type, the same blend
// order alpha*p1 + beta*p2 + gamma*p3 (:354) and 0 for a vertex outside the raster (the
// reference's masked gather, :336-346), NaN / Inf included.
//
// Work unit = (window of nout output columns, band of RB output rows, chunk of planes), one
// wave each, independent of the other waves of its workgroup:
//   * lane l owns K consecutive output columns b = window * nout + K * l + k; the window's input
//     columns xb .. xb + WC - 1 (WC = 32 * DB: one DB-byte piece of 16-bit samples per lane; xb
//     from the lattice, host-checked to hold every vertex of the window: tsk_lattice_ok);
//   * the band's triangle records are computed once (fp64, per lane, row and column) and kept
//     in registers for every plane of the chunk: 3 weights + one packed word of vertex
//     columns / rows / validity;
//   * per (plane, output row) the two input rows i_n, i_n + 1 arrive in a per-wave LDS ring by
//     LDS-DMA (buffer_load_dword[x4] ... lds: one 256-B or 1-KiB row piece per instruction) PDP
//     planes ahead, so the loads hold no VGPRs; each lane gathers its vertices with
//     ds_read_u16 and stores its K output samples as one 4-16 B piece.
// Downsampling (ratio >= 0.75 input columns per output column) uses DB = 16 (512-column
// windows: ~2x hexresize takes 252 output columns per wave, 4 per lane); upsampling DB = 4
// (128-column windows: 2x up takes 244 output columns per wave, 4 per lane).
// Waves stride over the units (a grid sized to the resident waves), so a launch has no
// partial last round.
#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>

#include "common.h"
#include "lattice.h"
#include "stream.h"
#include "tri_window.h"

namespace hg {

template <int N, int I = 0, typename F>
__device__ __forceinline__ void fu_static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        fu_static_for<N, I + 1>(f);
    }
}

// tuning knobs (A/B variants: tools/build_ovariant.sh)
#ifndef HD_RB16
#define HD_RB16 2           // 16-B pieces: output rows per unit
#endif
#ifndef HD_PDP16
#define HD_PDP16 1          // 16-B pieces: planes in flight ahead of the one blended
#endif
#ifndef HD_RB4
#define HD_RB4 2            // (4 spilled 277 VGPRs: r04 ISA; up-lattices now run tri_up.hip)
#endif
#ifndef HD_NR16
#define HD_NR16 4           // 16-B pieces: input rows loaded per (unit, plane) (host-checked)
#endif
#ifndef HD_NR4
#define HD_NR4 4
#endif
#ifndef HD_PDP4
#define HD_PDP4 2
#endif
#ifndef HD_P16
#define HD_P16 1            // 16-B pieces: adjacent output columns per lane and store
#endif
#ifndef HD_P4
#define HD_P4 2
#endif
// waves per SIMD asked of the register allocator: 4 capped the K = 4 kernels at 128 VGPRs
// and spilled 124-180 B per lane; 3 waves without spills are 7-18 % faster (r05 A/B)
#ifndef HD_WPE
#define HD_WPE 3
#endif
#ifndef HD_RING
#define HD_RING 8576        // LDS ring bytes per wave
#endif
constexpr int HD_THREADS = 256;

// (DB: bytes of an input-row piece per lane) -> window columns (64 lanes x DB bytes + one
// 32-B piece of 8 lanes), rows per unit, planes ahead; a ring row holds the window's WC
// samples and a 16-B zero slot (the vertices outside the raster read it)
template <int DB> struct TsCfg;
template <> struct TsCfg<4> { static constexpr int WC = 144, RB = HD_RB4, NR = HD_NR4, PDP = HD_PDP4; };
template <> struct TsCfg<16> { static constexpr int WC = 528, RB = HD_RB16, NR = HD_NR16, PDP = HD_PDP16; };

struct HexDownGeom {
    Geom g;                       // make_tri(h, w, h1, w1, margin)
    int64_t planes;
    int h, w, h1, w1;
    int nout;                     // output columns per window (<= 64 * K)
    int nwin, nband, nchunk, pc;  // units = nwin x nband x nchunk; planes per chunk
    int64_t units;
    double qmin;                  // min over output rows of 0.5 i_(a) - s1(a) (window origin)
};

// packed vertex record of one (row, lane, column): the ring index (16-bit samples) of p1 in
// row i_n (bits 0-9), of p2 from row i_n's start (bits 10-20: + the row pitch when the
// triangle flag puts it in row i_n + 1) and of p3 in row i_n + 1 (bits 21-30); a vertex
// outside the raster indexes its row's zero slot (the reference's masked gather reads 0)
__device__ __forceinline__ unsigned hd_pack(int o1, int o2, int o3) {
    return (unsigned)o1 | ((unsigned)o2 << 10) | ((unsigned)o3 << 21);
}

template <typename Tin, typename Tout, int K, int DB, int P, bool SEP>
__global__ __launch_bounds__(HD_THREADS, HD_WPE) void k_hexresize_down(const Tin* __restrict__ x,
                                                               Tout* __restrict__ y,
                                                               HexDownGeom D) {
    static_assert(sizeof(Tin) == 2, "16-bit inputs");
    // SEP: every output row loads its own two input rows (strong downsampling: the band's
    // rows share none), else the band's NR consecutive rows are loaded once per plane
    constexpr int WC = TsCfg<DB>::WC, RB = TsCfg<DB>::RB, PDP = TsCfg<DB>::PDP;
    constexpr int NR = SEP ? 2 * RB : TsCfg<DB>::NR;
    constexpr int NP = PDP + 1;
    constexpr int ROWB = WC * 2 + 16;                         // ring bytes of one input row
    constexpr int RW = ROWB / 2;                              // the same in samples
    static_assert(NP * NR * ROWB <= HD_RING && WC < 1024 && 2 * RW < 2048, "ring");
    __shared__ __attribute__((aligned(16))) unsigned char ring_all[HD_THREADS / 64][HD_RING];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned char* const ring = ring_all[wslot];
    if (lane < NP * NR) {                                     // the zero slots (never DMA'd)
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        *reinterpret_cast<u4v*>(ring + lane * ROWB + 2 * WC) = u4v{0u, 0u, 0u, 0u};
    }
    const int64_t nwaves = (int64_t)gridDim.x * (HD_THREADS / 64);
    const int64_t wid = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (HD_THREADS / 64) + wslot;
    const unsigned rowb = (unsigned)D.w * 2u, planeb = (unsigned)D.h * rowb;
    const unsigned oplane = (unsigned)D.h1 * (unsigned)D.w1 * (unsigned)sizeof(Tout);
    const unsigned orow = (unsigned)D.w1 * (unsigned)sizeof(Tout);

    for (int64_t u = wid; u < D.units; u += nwaves) {        // uniform per wave
        const int win = (int)(u % D.nwin);
        const int64_t r_ = u / D.nwin;
        const int band = (int)(r_ % D.nband);
        const int chunk = (int)(r_ / D.nband);
        const int64_t p0 = (int64_t)chunk * D.pc;
        const int np = (int)std::min<int64_t>(D.pc, D.planes - p0);
        const int a0 = band * RB, nr = min(RB, D.h1 - a0);
        const int b0 = win * D.nout;
        const int xb = __builtin_amdgcn_readfirstlane(tsk_window_x0(D.g, D.qmin, b0, DB / 2));
        // the chunk's planes as one buffer each way (host: < 2^31 bytes); a plane >= np
        // reads past the range (zeros)
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(x + p0 * (int64_t)D.h * D.w), (short)0, (int)(np * planeb), 0x00020000);
        const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((char*)y + p0 * (int64_t)oplane), (short)0, (int)(np * oplane), 0x00020000);

        // ---- the band's triangle records (fp64, geometry_np.py:276-354 via lattice.h) ----
        // lane l owns the columns b0 + P l + 64 P j + p (j < K / P, p < P) of its window: P
        // adjacent columns per store, the lanes of one store consecutive (so the gathers of
        // one ds_read hit consecutive LDS dwords, and one store covers 64 P columns)
        static_assert(K % P == 0, "K");
        constexpr int NJ = K / P;
        float wt[RB][K][3];
        unsigned pk[RB][K], yo[RB];
        int r0[RB];
        const int bend = min(b0 + D.nout, D.w1);            // the window's end column
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            // rows past the band's last (k >= nr) repeat its records, so they store the same
            // values to the same row: every store has in-range lanes (a store whose lanes are
            // all out of range can retire ahead of older loads and break the counted waits)
            const int a = a0 + min(k, nr - 1);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
                // one sample's fp64 temporaries at a time (interleaved samples spill)
                __builtin_amdgcn_sched_barrier(0);
                const int bb = b0 + P * lane + 64 * P * (kk / P) + kk % P;
                const TriSample s = tri_sample_fast(D.g, a, bb < bend ? bb : b0);   // (tri_fast_ok: host)
                if (kk == 0) r0[k] = __builtin_amdgcn_readfirstlane((int)s.i_n);   // i_n: row only
                auto ix = [&](int v) {                           // vertex v's ring index
                    return (s.vk >> v) & 1 ? min(max((int)s.c[v] - xb, 0), WC - 1) : WC;
                };
                wt[k][kk][0] = (float)s.alpha;
                wt[k][kk][1] = (float)s.beta;
                wt[k][kk][2] = (float)s.gamma;
                pk[k][kk] = hd_pack(ix(0), (s.r[1] != s.r[0] && ((s.vk >> 1) & 1) ? RW : 0) + ix(1), ix(2));
            }
            yo[k] = (unsigned)a * orow;
        }
        __builtin_amdgcn_sched_barrier(0);
        // per store j: the lane's byte offset in the row when all its P columns are in the
        // window; else lane 0 (whose column b0 always is, and b0 + 1 for P = 2: host) repeats
        // store 0, so no store has all its lanes out of range; a lane with only its first
        // column inside stores that one separately (pc1)
        unsigned co[NJ];
        bool pc1[NJ], rep[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = b0 + P * lane + 64 * P * j;
            const bool all = c + P - 1 < bend;
            rep[j] = !all && lane == 0;
            co[j] = all ? (unsigned)c * (unsigned)sizeof(Tout)
                        : lane == 0 ? (unsigned)b0 * (unsigned)sizeof(Tout) : 0x80000000u;
            pc1[j] = P == 2 && !all && c < bend;
        }

        // ---- per plane: LDS-DMA of the NR input rows rlo .. rlo + NR - 1 the band's output
        // rows read (rows i_n, i_n + 1 of each; host-checked to fit), PDP planes ahead ------
        // (columns left of the raster: the lane's piece is clamped to column 0 and every
        // vertex there is outside the raster, read from the zero slot)
        const int rlo = r0[0];
        const unsigned voff = (unsigned)max(xb + (DB / 2) * lane, 0) * 2u;
        const unsigned voff2 = (unsigned)max(xb + 32 * DB + 2 * lane, 0) * 2u;
        auto slots = [&](int pi) { return ring + (pi % NP) * (NR * ROWB); };
        auto dma = [&](int pi) {
            unsigned char* const sl = slots(pi);
            const unsigned po = pi < np ? (unsigned)pi * planeb : (unsigned)np * planeb;
#pragma unroll
            for (int q = 0; q < NR; ++q) {
                const unsigned so = po + (unsigned)(SEP ? r0[q / 2] + q % 2 : rlo + q) * rowb;
                auto* const ld = (__attribute__((address_space(3))) void*)(sl + q * ROWB);
                if constexpr (DB == 16)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, ld, 16, voff, so, 0, 0);
                else
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, ld, 4, voff, so, 0, 0);
                // the window's last 16 columns: one dword each from lanes 0-7
                auto* const le = (__attribute__((address_space(3))) void*)(sl + q * ROWB + 64 * DB);
                if (lane < 8) __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, le, 4, voff2, so, 0, 0);
            }
        };
        for (int pi = 0; pi < PDP; ++pi) dma(pi);              // prologue: planes 0 .. PDP - 1
        for (int pi = 0; pi < np; ++pi) {
            const unsigned short* const base = reinterpret_cast<const unsigned short*>(slots(pi));
            const unsigned yp = (unsigned)pi * oplane;
            dma(pi + PDP);
            {
                // plane pi's 2 NR pieces are done once at most the operations issued after
                // them are outstanding (vmcnt counts loads, stores and LDS-DMA together, in
                // issue order): the pieces of the PDP planes after it and the RB NJ stores of
                // each plane since -- 2 NR PDP + RB NJ min(pi, PDP)
                constexpr int NPC = 2 * NR * PDP, NST = RB * NJ;
                static_assert(NPC + PDP * NST < 64, "vmcnt");
                auto wait = [](auto Nc) {
                    constexpr int N = decltype(Nc)::value;
                    __builtin_amdgcn_s_waitcnt((0x0f70 & ~0xf) | (N & 0xf) | ((N >> 4) << 14));
                };
                if (pi >= PDP) {
                    wait(std::integral_constant<int, NPC + PDP * NST>{});
                } else {
                    fu_static_for<PDP>([&](auto Pc) {
                        constexpr int P_ = decltype(Pc)::value;
                        if (pi == P_) wait(std::integral_constant<int, NPC + P_ * NST>{});
                    });
                }
            }
            fu_static_for<RB>([&](auto Kc) {
                constexpr int k = decltype(Kc)::value;
                asm volatile("" ::: "memory");                    // LDS reads after the wait
                const unsigned short* const s0 = base + (SEP ? 2 * k : r0[k] - rlo) * RW;
                const unsigned short* const s1 = s0 + RW;
                float v[K];
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    const unsigned q = pk[k][kk];
                    const float v0 = to_acc<float>(__builtin_bit_cast(Tin, s0[q & 1023]));
                    const float v1 = to_acc<float>(__builtin_bit_cast(Tin, s0[(q >> 10) & 2047]));
                    const float v2 = to_acc<float>(__builtin_bit_cast(Tin, s1[q >> 21]));
                    v[kk] = wt[k][kk][0] * v0 + wt[k][kk][1] * v1 + wt[k][kk][2] * v2;   // :354
                }
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    // lane 0 out of the window repeats store 0 (co[j] = b0): its values too
                    const float v0 = rep[j] ? v[0] : v[P * j];
                    const unsigned o = yo[k] + co[j];
                    if constexpr (P == 1) {
                        if constexpr (sizeof(Tout) == 2)
                            __builtin_amdgcn_raw_buffer_store_b16(
                                __builtin_bit_cast(unsigned short, from_acc<Tout>(v0)), yr, o, yp, 0);
                        else
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v0), yr, o, yp, 0);
                    } else {
                        const float v1 = rep[j] ? v[1] : v[P * j + 1];
                        if constexpr (sizeof(Tout) == 2) {
                            typedef Tout t2v __attribute__((ext_vector_type(2)));
                            __builtin_amdgcn_raw_buffer_store_b32(
                                __builtin_bit_cast(unsigned, t2v{from_acc<Tout>(v0), from_acc<Tout>(v1)}), yr, o, yp, 0);
                        } else {
                            typedef unsigned u2v __attribute__((ext_vector_type(2)));
                            __builtin_amdgcn_raw_buffer_store_b64(
                                u2v{__builtin_bit_cast(unsigned, v0), __builtin_bit_cast(unsigned, v1)}, yr, o, yp, 0);
                        }
                        if (pc1[j]) {   // the raster's last column alone (extra stores only
                                        // over-count the waits above)
                            const unsigned o1 = yo[k] + (unsigned)(b0 + 2 * lane + 128 * j) * (unsigned)sizeof(Tout);
                            if constexpr (sizeof(Tout) == 2)
                                __builtin_amdgcn_raw_buffer_store_b16(
                                    __builtin_bit_cast(unsigned short, from_acc<Tout>(v[P * j])), yr, o1, yp, 0);
                            else
                                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[P * j]), yr, o1, yp, 0);
                        }
                    }
                }
            });
        }
        // the trailing pieces (zeros past the last plane) land before the ring is reused
        __builtin_amdgcn_s_waitcnt(0x0f70);                   // vmcnt(0)
    }
}

#ifndef HD_CPP
#define HD_CPP 48           // planes per unit in the one-wave-per-unit grid (round 5)
#endif
template <typename Tin, typename Tout, int K, int DB, int P, bool SEP>
static int hd_launch(const void* src, void* dst, HexDownGeom& D, hipStream_t st) {
    // resident waves: 256 CUs x 4 SIMDs x 4 waves; units split into plane chunks until
    // there are >= upw units per resident wave (the records are then recomputed per chunk:
    // fewer, longer units amortise them, more units balance the waves; A/B switch
    // HYGRID_TSK_UPW, default 1)
    constexpr int64_t RESIDENT = 256 * 4 * 4;
    constexpr int PDP = TsCfg<DB>::PDP;
    const char* ue = getenv("HYGRID_TSK_UPW");
    const int64_t upw = ue ? std::max(1, atoi(ue)) : 1;
    const int64_t tiles = (int64_t)D.nwin * D.nband;
    int64_t nchunk = std::max<int64_t>(1, std::min<int64_t>(D.planes, (upw * RESIDENT + tiles - 1) / tiles));
    // Round 5: one wave per unit and ~HD_CPP planes per unit (the records amortised over more
    // planes; fewer, longer-lived units contend less): 4K -> 2K bf16 b32 0.496 -> 0.429 ms, 8K ->
    // 4K fp16 b8 -1.9 % (profiles/r05/hexresize_grid_ab.txt).  HYGRID_TSK_GRID=0: the old rule.
    // (only with >= 2 chunks of planes: below that the old rule's plane chunks fill the
    // resident waves, e.g. a single RGB image's 3 planes, as k_tri_up does)
    const bool grid = !env_is("HYGRID_TSK_GRID", "0") && D.planes >= 2 * HD_CPP;
    if (grid) nchunk = std::max<int64_t>(1, D.planes / HD_CPP);
    if (const char* e = getenv("HYGRID_TSK_CHUNKS"))   // A/B switch: plane chunks per tile
        nchunk = std::max<int64_t>(1, std::min<int64_t>(D.planes, atoi(e)));
    // a chunk's planes are one buffer each way: 32-bit offsets, including the planes past
    // the chunk the prefetch addresses (out of range: zeros)
    const int64_t plane_bytes = std::max<int64_t>((int64_t)D.h * D.w * 2, (int64_t)D.h1 * D.w1 * 4);
    const int64_t max_pc = std::max<int64_t>(1, (((int64_t)1 << 31) - 1) / plane_bytes - PDP - 1);
    nchunk = std::max<int64_t>(nchunk, (D.planes + max_pc - 1) / max_pc);
    D.pc = (int)((D.planes + nchunk - 1) / nchunk);
    D.nchunk = (int)((D.planes + D.pc - 1) / D.pc);
    D.units = tiles * D.nchunk;
    int64_t waves = std::min<int64_t>(D.units, RESIDENT);
    if (grid) waves = std::min<int64_t>(D.units, (int64_t)1 << 30);   // a wave per unit
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    hipLaunchKernelGGL((k_hexresize_down<Tin, Tout, K, DB, P, SEP>), dim3(blocks), dim3(HD_THREADS), 0, st,
                       (const Tin*)src, (Tout*)dst, D);
    return launch_status();
}

// A triangle-blend resample (op: HG_OP_HEXRESIZE or HG_OP_HEX_TO_RECT, linear) on the
// streaming kernel, or HG_EUNSUP (the caller runs k_resample_lds).  dry: check only (HG_OK if
// the kernel would run).
int tristream_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                  int64_t w, int64_t h1, int64_t w1, hipStream_t st, bool dry) {
    if (env_is("HYGRID_DOWN", "0")) return HG_EUNSUP;   // A/B switch: general kernels only
    if (op != HG_OP_HEXRESIZE && op != HG_OP_HEX_TO_RECT) return HG_EUNSUP;
    if (sdt != HG_F16 && sdt != HG_BF16) return HG_EUNSUP;
    if (ddt != HG_F16 && ddt != HG_BF16 && ddt != HG_F32) return HG_EUNSUP;
    if (planes < 1 || h < 2 || w < 2 || h1 < 1 || w1 < 1) return HG_EUNSUP;
    // LDS-DMA moves whole dwords from dword-aligned addresses: every input row must start on
    // one (even width, 4-B aligned base); 16-B pieces want 16-B aligned rows
    if ((w & 1) || (reinterpret_cast<uintptr_t>(src) & 3)) return HG_EUNSUP;
    const bool a16 = (w % 8) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0;
    // one plane (+ the prefetch's out-of-range planes) within 32-bit buffer offsets
    if ((h * w * 2) * 4 >= ((int64_t)1 << 31) || (h1 * w1 * 4) * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;
    const Geom g = make_tri(h, w, h1, w1, op == HG_OP_HEXRESIZE ? 0.5 : 0.75);
    if (!tri_fast_ok(g)) return HG_EUNSUP;
    // input columns per output column: 512-column windows (16-B pieces) when downsampling,
    // 128-column windows (4-B pieces) when upsampling or the rows are not 16-B aligned; a
    // lane owns K output columns of its window in groups of P adjacent ones (K = 4, or
    // fewer for narrow windows)
    const double ratio = (double)(w - 1) / (double)(w1 - 1);   // (tri_fast_ok: w1 > 1)
    const int DB = (ratio >= 0.75 && a16) ? 16 : 4, wc = 32 * DB + 16, al = DB / 2;
    const int P = DB == 16 ? HD_P16 : HD_P4;
    if (P == 2 && w1 < 2) return HG_EUNSUP;
    HexDownGeom D = {};
    double qmax;
    if (!tsk_rows_ok(g, &D.qmin, &qmax)) return HG_EUNSUP;
    const int RB = DB == 16 ? TsCfg<16>::RB : TsCfg<4>::RB, NR = DB == 16 ? TsCfg<16>::NR : TsCfg<4>::NR;
    const bool sep = !tsk_bands_ok(g, RB, NR);       // rows shared by no two output rows
    // output windows of whole 128-B lines when the lattice allows (64 16-bit or 32 fp32
    // columns: partial lines shared by two waves cost ~10-20 %, measured), else the widest
    int nout = std::min(256, (int)std::floor((wc - 6) / std::max(ratio, 1e-3)));
    if (const char* ne = getenv("HYGRID_TSK_NOUT")) nout = std::min(nout, atoi(ne));   // A/B switch
    const int L = ddt == HG_F32 ? 32 : 64;
    int best = 0;
    for (int n = nout / L * L; n >= L && !best; n -= L)
        if (tsk_lattice_ok(g, n, wc, al, D.qmin, qmax) && !(P == 2 && w1 % n == 1)) best = n;
    for (int n = nout; n >= 32 && !best; --n) {
        if (P == 2 && ((n & 1) || w1 % n == 1)) continue;   // >= 2 columns per window
        if (tsk_lattice_ok(g, n, wc, al, D.qmin, qmax)) best = n;
    }
    if (!best) return HG_EUNSUP;                       // > ~15x downsampling: the general kernel
    nout = best;
    const int K = nout > 64 * P ? 4 : P;
    D.g = g;
    D.planes = planes;
    D.h = (int)h; D.w = (int)w; D.h1 = (int)h1; D.w1 = (int)w1;
    D.nout = nout;
    D.nwin = (int)((w1 + nout - 1) / nout);
    D.nband = (int)((h1 + RB - 1) / RB);
    if (dry) return HG_OK;
#define HG_TSK2(TI, TO, S)                                                                     \
    if (DB == 4) return K == 4 ? hd_launch<TI, TO, 4, 4, HD_P4, S>(src, dst, D, st)            \
                               : hd_launch<TI, TO, HD_P4, 4, HD_P4, S>(src, dst, D, st);       \
    return K == 4 ? hd_launch<TI, TO, 4, 16, HD_P16, S>(src, dst, D, st)                        \
                  : hd_launch<TI, TO, HD_P16, 16, HD_P16, S>(src, dst, D, st);
#define HG_TSK(TI, TO)                                                                         \
    if (sep) { HG_TSK2(TI, TO, true) }                                                         \
    HG_TSK2(TI, TO, false)
    if (sdt == HG_BF16) {
        if (ddt == HG_BF16) { HG_TSK(__bf16, __bf16) }
        if (ddt == HG_F16) { HG_TSK(__bf16, _Float16) }
        HG_TSK(__bf16, float)
    }
    if (ddt == HG_BF16) { HG_TSK(_Float16, __bf16) }
    if (ddt == HG_F16) { HG_TSK(_Float16, _Float16) }
    HG_TSK(_Float16, float)
#undef HG_TSK
#undef HG_TSK2
}

}  // namespace hg
