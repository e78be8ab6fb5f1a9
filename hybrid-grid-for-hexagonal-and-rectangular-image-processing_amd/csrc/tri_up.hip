// tri_up.hip — upsampling triangle resamples on a row-streaming kernel: hex_to_rect_resample
// (geometry_np.py:191-356) and hexresize (:520-681) whose output lattice is at least as fine
// as the input's (row and column steps <= 1 input sample), 'linear' (the triangle blend,
// :347-354) and 'nearest' (the first-minimum vertex, geometry_torch.py:335-347).  The case
// that matters is the inverse of ConvertToHexagon's lattice, hex (h/2, w/2) -> rect (h, w)
// (Image.py:111-116 read backwards): 4 output samples per input sample, so the output stores
// are ~80 % of the bytes.
//
// Bit-identical to the general kernels of resample.hip for the same call: the per-sample
// records are the fp64 triangle samples of lattice.h (tri_sample, the reference's expression
// order) — weights cast to fp32, the blend alpha*p1 + beta*p2 + gamma*p3 evaluated in the
// same order (:354) — and a vertex outside the raster reads 0 (the reference's masked gather,
// :336-346); nearest copies the chosen element's bits.
//
// Work unit = (window of 64 K output columns, band of RB output rows, chunk of planes), one
// wave each:
//   * lane l owns the K adjacent output columns b0 + K l .. + K - 1 (one K-sample vector store
//     per row; lanes past the raster's last column repeat the last K-group, identical values
//     to identical addresses, so every store has in-range lanes);
//   * the unit's records are computed once (fp64) and kept in registers for every plane of
//     the chunk: per sample the LDS byte offsets of its vertices (the zero slot for a vertex
//     outside the raster) and, for 'linear', the three fp32 weights — so a gather is one
//     ds_read with no address arithmetic;
//   * per plane, the unit's RB / 2 + 2 input rows (WC = 288 / sizeof(Tin) columns from a dword-
//     aligned window origin) arrive in a per-wave LDS ring by LDS-DMA (buffer_load_dword ...
//     lds: a 256-B piece from all lanes + a 32-B piece from lanes 0-7 per row) several planes
//     ahead, so the loads hold no VGPRs.
// What bounds it (4K b32, r04 sessions K-N): the memory side alone — these stores plus these
// row loads, no arithmetic (tools/microbench/wpat.hip) — takes 0.54 ms of the kernel's
// 0.61 ms, while the stores alone take 0.29 ms (0.70 of 8 TB/s) and the arithmetic alone
// 0.31 ms; deeper prefetch (2 -> 6 planes), 16-B DMA pieces, other unit orders, 4- and 6-row
// bands and narrower windows did not move the mixed pattern below 0.41-0.48 ms.
// Chunks (round 5): ~TU_CPP planes per unit and one wave per unit when the call has enough
// planes (records amortised over >= 24 planes, short-lived waves); otherwise the units about
// fill the resident waves once and waves stride over units.
#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>

#include "common.h"
#include "lattice.h"
#include "stream.h"
#include "tri_window.h"

namespace hg {

#ifndef TU_RB
#define TU_RB 2             // 'linear': output rows per unit (input rows: TU_RB / 2 + 2)
#endif
#ifndef TU_RB_NEAR
#define TU_RB_NEAR 4        // 'nearest': output rows per unit (1 gather per sample: more rows
#endif                      // per unit, fewer loaded rows per output row; r04 session N)
#ifndef TU_PDP
#define TU_PDP 6            // 'linear': planes in flight ahead of the one blended
#endif
#ifndef TU_WPE
#define TU_WPE 4            // waves per SIMD asked of the register allocator
#endif
#ifndef TU_ORDER
#define TU_ORDER 0          // unit index -> (window fastest, band, chunk); 1: band fastest
#endif
#ifndef TU_VLD
#define TU_VLD 1            // 1: input rows by dword loads into VGPRs, PDP planes ahead, written to a
#endif                      // one-plane LDS slot when consumed (instead of LDS-DMA into a ring)
#ifndef TU_PDP_VLD
#define TU_PDP_VLD 3        // with TU_VLD: planes of rows held in VGPRs ahead of the one blended
                            // (4 spilled 24-28 B per lane in the f16-input linear kernels)
#endif
#ifndef TU_CPP
#define TU_CPP 24           // planes per unit when the grid has a wave per unit (round 5)
#endif
constexpr int TU_THREADS = 256;
#ifndef TU_KDIV
#define TU_KDIV 1           // output columns per lane = the natural K / TU_KDIV (A/B variants)
#endif
constexpr int TU_PCB = 288;         // DMA bytes per input row: 64 lanes x 4 B + 8 lanes x 4 B
constexpr int TU_ROWB = TU_PCB + 16;         // ring bytes of one input row (+ a 16-B zero slot)
// per interp: output rows per unit, input rows per unit (i_n(a0) .. i_n(a0 + RB - 1) + 1 of an
// upsampling lattice, host-checked), planes in flight (vmcnt counts DMA pieces and stores:
// < 64 outstanding), ring slots and bytes of one plane slot
template <bool NEAR> struct TuCfg {
    static constexpr int RB = NEAR ? TU_RB_NEAR : TU_RB, NR = RB / 2 + 2;
    static constexpr int PDP_ = TU_VLD ? TU_PDP_VLD : NEAR ? 63 / (2 * NR + RB) : TU_PDP;
    static constexpr int PDP = PDP_ < 6 ? PDP_ : 6, NP = TU_VLD ? 1 : PDP + 1, SLOT = NR * TU_ROWB;
    static_assert(PDP >= 1 && PDP * (2 * NR + RB) < 64, "vmcnt");
};

struct TriUpGeom {
    Geom g;                       // make_tri(h, w, h1, w1, margin)
    int h, w, h1, w1;
    int nwin, nband, pc;          // units = nwin x nband x chunks; planes per chunk
    int64_t planes, units;
    double qmin;                  // min over output rows of 0.5 i_(a) - s1(a) (window origin)
};

template <int N, int I = 0, typename F>
__device__ __forceinline__ void tu_static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        tu_static_for<N, I + 1>(f);
    }
}

template <int N> struct UInt;
template <> struct UInt<1> { using T = uint8_t; };
template <> struct UInt<2> { using T = unsigned short; };
template <> struct UInt<4> { using T = unsigned; };

// One lane's K-sample store of `bytes` = K * sizeof(Tout) bytes from the packed words v
// (16-byte stores: hg_store_b128, soffset 0 — the store-data hazard of round 5, common.h).
template <int BYTES>
__device__ __forceinline__ void tu_store(const unsigned (&v)[4], __amdgpu_buffer_rsrc_t rs, unsigned vo,
                                         unsigned so) {
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    if constexpr (BYTES == 1) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v[0], rs, vo, so, 0);
    else if constexpr (BYTES == 2) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v[0], rs, vo, so, 0);
    else if constexpr (BYTES == 4) __builtin_amdgcn_raw_buffer_store_b32(v[0], rs, vo, so, 0);
    else if constexpr (BYTES == 8) __builtin_amdgcn_raw_buffer_store_b64(u2v{v[0], v[1]}, rs, vo, so, 0);
    else hg_store_b128(hg_u4v{v[0], v[1], v[2], v[3]}, rs, vo, so);
}

template <typename T> __device__ __forceinline__ float tu_f32(unsigned bits) {
    if constexpr (std::is_same<T, __bf16>::value) return __builtin_bit_cast(float, bits << 16);
    else if constexpr (std::is_same<T, _Float16>::value)
        return (float)__builtin_bit_cast(_Float16, (unsigned short)bits);
    else return __builtin_bit_cast(float, bits);
}
template <typename T> __device__ __forceinline__ unsigned tu_bits(float v) {
    if constexpr (sizeof(T) == 4) return __builtin_bit_cast(unsigned, v);
    else return (unsigned)__builtin_bit_cast(unsigned short, (T)v);
}

// NEAR: 'nearest' (Tin == Tout, raw bits); else 'linear' into Tout with fp32 accumulation.
template <typename Tin, typename Tout, int K, bool NEAR>
__global__ __launch_bounds__(TU_THREADS) __attribute__((amdgpu_waves_per_eu(TU_WPE)))
void k_tri_up(const Tin* __restrict__ x, Tout* __restrict__ y, TriUpGeom D) {
    constexpr int E = (int)sizeof(Tin);
    constexpr int WC = TU_PCB / E;                    // window input columns
    constexpr int OB = K * (int)sizeof(Tout);         // bytes of one lane's store
    static_assert(OB <= 16 && (!NEAR || sizeof(Tin) == sizeof(Tout)), "store width");
    static_assert(WC * E == TU_PCB && 4 % E == 0, "a lane's DMA dword holds whole samples");
    constexpr int NV = NEAR ? 1 : 3;                  // gathers per sample
    using UIn = typename UInt<E>::T;
    constexpr int TU_RB_ = TuCfg<NEAR>::RB, TU_NR_ = TuCfg<NEAR>::NR, TU_PDP_ = TuCfg<NEAR>::PDP;
    constexpr int TU_NP_ = TuCfg<NEAR>::NP, TU_SLOT_ = TuCfg<NEAR>::SLOT;
    __shared__ __attribute__((aligned(16))) unsigned char ring_all[TU_THREADS / 64][TU_NP_ * TU_SLOT_];
    const int lane = threadIdx.x & 63;
    const int wslot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned char* const ring = ring_all[wslot];
    if (lane < TU_NP_ * TU_NR_) {                       // the zero slots (never DMA'd)
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        *reinterpret_cast<u4v*>(ring + lane * TU_ROWB + TU_PCB) = u4v{0u, 0u, 0u, 0u};
    }
    const int64_t nwaves = (int64_t)gridDim.x * (TU_THREADS / 64);
    const int64_t wid = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (TU_THREADS / 64) + wslot;
    const unsigned rowb = (unsigned)D.w * (unsigned)E, planeb = (unsigned)D.h * rowb;
    const unsigned orow = (unsigned)D.w1 * (unsigned)sizeof(Tout);
    const unsigned oplane = (unsigned)D.h1 * orow;

    for (int64_t u = wid; u < D.units; u += nwaves) {        // uniform per wave
        const int64_t tile = u % ((int64_t)D.nwin * D.nband);
        const int win = (int)(TU_ORDER ? tile / D.nband : tile % D.nwin);
        const int band = (int)(TU_ORDER ? tile % D.nband : tile / D.nwin);
        const int64_t p0 = (u / ((int64_t)D.nwin * D.nband)) * (int64_t)D.pc;
        const int np = (int)std::min<int64_t>(D.pc, D.planes - p0);
        const int a0 = band * TU_RB_, nr = min(TU_RB_, D.h1 - a0);
        const int b0 = win * 64 * K;
        const int xb = __builtin_amdgcn_readfirstlane(tsk_window_x0(D.g, D.qmin, b0, 4 / E));
        // the chunk's planes as one buffer each way (host: < 2^31 bytes); planes past the
        // chunk (the prefetch's) read as zeros
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(x + p0 * (int64_t)D.h * D.w), (short)0, (int)(np * planeb), 0x00020000);
        const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((char*)y + p0 * (int64_t)oplane), (short)0, (int)(np * oplane), 0x00020000);
        // this lane's K-group (lanes past the raster repeat the last one: w1 % K == 0, host)
        const int cb = min(b0 + K * lane, D.w1 - K);

        // ---- the unit's records (fp64, geometry_np.py:276-354 via lattice.h) --------------
        // rows past the band's last (k >= nr) repeat its records: same values, same addresses
        unsigned off[TU_RB_][K][NV];
        float wt[TU_RB_][K][NEAR ? 1 : 3];
        unsigned yo[TU_RB_];
        int rlo = 0;
#pragma unroll
        for (int k = 0; k < TU_RB_; ++k) {
            const int a = a0 + min(k, nr - 1);
            yo[k] = (unsigned)a * orow;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
                // one sample's fp64 temporaries at a time (the scheduler would otherwise
                // interleave the samples and spill)
                __builtin_amdgcn_sched_barrier(0);
                const TriSample s = tri_sample_fast(D.g, a, cb + kk);   // (tri_fast_ok: host)
                if (k == 0 && kk == 0) rlo = __builtin_amdgcn_readfirstlane((int)s.i_n);
                auto ix = [&](int v) -> unsigned {           // vertex v's LDS byte offset
                    return (s.vk >> v) & 1
                               ? (unsigned)((int)(s.r[v] - rlo) * TU_ROWB + ((int)s.c[v] - xb) * E)
                               : (unsigned)TU_PCB;           // row 0's zero slot
                };
                if constexpr (NEAR) {
                    // selects, not s.r[s.argmin]: a run-time index into the sample's arrays put
                    // them in scratch (128 B per lane for every nearest kernel)
                    const int am = s.argmin;
                    const int rr = (int)(am == 0 ? s.r[0] : am == 1 ? s.r[1] : s.r[2]);
                    const int cc = (int)(am == 0 ? s.c[0] : am == 1 ? s.c[1] : s.c[2]);
                    off[k][kk][0] = (s.vk >> am) & 1 ? (unsigned)((rr - rlo) * TU_ROWB + (cc - xb) * E)
                                                     : (unsigned)TU_PCB;
                    asm volatile("" : "+v"(off[k][kk][0]));   // one sample's temporaries at a time
                } else {
                    off[k][kk][0] = ix(0);
                    off[k][kk][1] = ix(1);
                    off[k][kk][2] = ix(2);
                    wt[k][kk][0] = (float)s.alpha;
                    wt[k][kk][1] = (float)s.beta;
                    wt[k][kk][2] = (float)s.gamma;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        const unsigned vo = (unsigned)cb * (unsigned)sizeof(Tout);

        // ---- per plane: LDS-DMA of the unit's rows rlo .. rlo + 2, PDP planes ahead -------
        // (a lane's dword left of the raster is out of the buffer range: zeros; rows past the
        // raster are clamped to the last one, whose vertices there are outside: zero slot)
        const unsigned voff0 = xb + (4 / E) * lane >= 0 ? (unsigned)(xb * E + 4 * lane) : 0x80000000u;
        const unsigned voff1 = (unsigned)(xb * E + 256 + 4 * lane);   // lanes 0-7
        auto dma = [&](int pi, auto SLc) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned po = pi < np ? (unsigned)pi * planeb : (unsigned)np * planeb;
#pragma unroll
            for (int q = 0; q < TU_NR_; ++q) {
                const unsigned so = po + (unsigned)min(rlo + q, D.h - 1) * rowb;
                auto* const l0 = (__attribute__((address_space(3))) void*)(ring + SL * TU_SLOT_ + q * TU_ROWB);
                auto* const l1 = (__attribute__((address_space(3))) void*)(ring + SL * TU_SLOT_ + q * TU_ROWB + 256);
                const unsigned so_ = so;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, l0, 4, voff0, so_, 0, 0);
                if (lane < 8) __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, l1, 4, voff1, so_, 0, 0);
            }
        };
        // plane pi's pieces are done once at most the operations issued after them are
        // outstanding (vmcnt counts loads, stores and LDS-DMA together, in issue order): the
        // pieces of the PDP planes after it and the RB stores of each plane since
        constexpr int NPC_ = 2 * TU_NR_, NST = TU_RB_;   // (lanes 8+ of the 32-B piece: no-ops, still counted)
        static_assert(TU_PDP_ * (NPC_ + NST) < 64, "vmcnt");
        auto wait = [](auto Nc) {
            constexpr int N = decltype(Nc)::value;
            __builtin_amdgcn_s_waitcnt((0x0f70 & ~0xf) | (N & 0xf) | ((N >> 4) << 14));
        };
        // TU_VLD: the rows of PDP planes in VGPRs, slot pi % PDP; plane pi is written to the one
        // LDS slot when its turn comes (the wave's LDS ops run in order: its gathers of plane
        // pi - 1 are done, its gathers of plane pi see the writes)
        unsigned rv[TU_VLD ? TU_PDP_ : 1][TU_VLD ? TU_NR_ : 1][2];
        const unsigned voff1v = lane < 8 ? voff1 : 0x80000000u;
        auto vld = [&](int pi, auto SLc) {
            constexpr int SL = decltype(SLc)::value;
            const unsigned po = pi < np ? (unsigned)pi * planeb : (unsigned)np * planeb;
#pragma unroll
            for (int q = 0; q < TU_NR_; ++q) {
                const unsigned so = po + (unsigned)min(rlo + q, D.h - 1) * rowb;
                rv[SL][q][0] = __builtin_amdgcn_raw_buffer_load_b32(xr, voff0, so, 0);
                rv[SL][q][1] = __builtin_amdgcn_raw_buffer_load_b32(xr, voff1v, so, 0);
            }
        };
        auto body_v = [&](int pi, auto SLc) {
            constexpr int SL = decltype(SLc)::value;
            // plane pi's loads are done once at most those issued after them are outstanding:
            // the loads of the next PDP - 1 planes and the stores of the planes since
            constexpr int NL = 2 * TU_NR_, NST = TU_RB_;
            static_assert((TU_PDP_ - 1) * NL + TU_PDP_ * NST < 64, "vmcnt");
            if (pi >= TU_PDP_) {
                wait(std::integral_constant<int, (TU_PDP_ - 1) * NL + TU_PDP_ * NST>{});
            } else {
                tu_static_for<TU_PDP_>([&](auto Pc) {
                    constexpr int P_ = decltype(Pc)::value;
                    if (pi == P_) wait(std::integral_constant<int, (TU_PDP_ - 1) * NL + P_ * NST>{});
                });
            }
#pragma unroll
            for (int q = 0; q < TU_NR_; ++q) {
                *reinterpret_cast<unsigned*>(ring + q * TU_ROWB + 4 * lane) = rv[SL][q][0];
                if (lane < 8) *reinterpret_cast<unsigned*>(ring + q * TU_ROWB + 256 + 4 * lane) = rv[SL][q][1];
            }
            vld(pi + TU_PDP_, SLc);                         // the slot's registers are free again
            const unsigned char* const sb = ring;
            const unsigned so = (unsigned)pi * oplane;
#pragma unroll
            for (int k = 0; k < TU_RB_; ++k) {
                unsigned pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    unsigned bits;
                    if constexpr (NEAR) {
                        bits = *reinterpret_cast<const UIn*>(sb + off[k][kk][0]);
                    } else {
                        const float v0 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][0]));
                        const float v1 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][1]));
                        const float v2 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][2]));
                        bits = tu_bits<Tout>(wt[k][kk][0] * v0 + wt[k][kk][1] * v1 + wt[k][kk][2] * v2);   // :354
                    }
                    constexpr int SB = (int)sizeof(Tout) * 8;
                    if constexpr (SB == 32) pk[kk] = bits;
                    else pk[(kk * SB) / 32] |= bits << ((kk * SB) % 32);
                }
                tu_store<OB>(pk, yr, vo, __builtin_amdgcn_readfirstlane(so + yo[k]));
            }
        };
        if constexpr (TU_VLD) {
            tu_static_for<TU_PDP_>([&](auto Pc) { vld(decltype(Pc)::value, Pc); });   // prologue
            int pi = 0;
            for (; pi + TU_PDP_ <= np; pi += TU_PDP_)
                tu_static_for<TU_PDP_>([&](auto Sc) { body_v(pi + decltype(Sc)::value, Sc); });
            tu_static_for<TU_PDP_ - 1>([&](auto Sc) {
                if (pi + decltype(Sc)::value < np) body_v(pi + decltype(Sc)::value, Sc);
            });
            __builtin_amdgcn_s_waitcnt(0x0f70);             // vmcnt(0): no load in flight at exit
            continue;
        }
        auto body = [&](int pi, auto SLc) {
            constexpr int SL = decltype(SLc)::value;
            dma(pi + TU_PDP_, std::integral_constant<int, (SL + TU_PDP_) % TU_NP_>{});
            if (pi >= TU_PDP_) {
                wait(std::integral_constant<int, TU_PDP_ * NPC_ + TU_PDP_ * NST>{});
            } else {                                        // the first planes: fewer stores since
                tu_static_for<TU_PDP_>([&](auto Pc) {
                    constexpr int P_ = decltype(Pc)::value;
                    if (pi == P_) wait(std::integral_constant<int, TU_PDP_ * NPC_ + P_ * NST>{});
                });
            }
            asm volatile("" ::: "memory");                  // LDS reads after the wait
            const unsigned char* const sb = ring + SL * TU_SLOT_;
            const unsigned so = (unsigned)pi * oplane;
#pragma unroll
            for (int k = 0; k < TU_RB_; ++k) {
                unsigned pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    unsigned bits;
                    if constexpr (NEAR) {
                        bits = *reinterpret_cast<const UIn*>(sb + off[k][kk][0]);
                    } else {
                        const float v0 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][0]));
                        const float v1 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][1]));
                        const float v2 = tu_f32<Tin>(*reinterpret_cast<const UIn*>(sb + off[k][kk][2]));
                        bits = tu_bits<Tout>(wt[k][kk][0] * v0 + wt[k][kk][1] * v1 + wt[k][kk][2] * v2);   // :354
                    }
                    constexpr int SB = (int)sizeof(Tout) * 8;
                    if constexpr (SB == 32) pk[kk] = bits;
                    else pk[(kk * SB) / 32] |= bits << ((kk * SB) % 32);
                }
                tu_store<OB>(pk, yr, vo, __builtin_amdgcn_readfirstlane(so + yo[k]));
            }
        };
        tu_static_for<TU_PDP_>([&](auto Pc) { dma(decltype(Pc)::value, Pc); });   // prologue
        // plane pi uses ring slot pi % NP: the loop runs NP planes per trip so every slot
        // offset is an immediate of the ds_read / LDS-DMA
        int pi = 0;
        for (; pi + TU_NP_ <= np; pi += TU_NP_)
            tu_static_for<TU_NP_>([&](auto Sc) { body(pi + decltype(Sc)::value, Sc); });
        tu_static_for<TU_NP_ - 1>([&](auto Sc) {
            if (pi + decltype(Sc)::value < np) body(pi + decltype(Sc)::value, Sc);
        });
        // the trailing pieces (zeros past the last plane) land before the ring is reused
        __builtin_amdgcn_s_waitcnt(0x0f70);                   // vmcnt(0)
    }
}

template <typename Tin, typename Tout, int K, bool NEAR>
static int tu_launch(const void* src, void* dst, TriUpGeom& D, hipStream_t st) {
    // units ~ the resident waves (256 CUs x 4 SIMDs x 4): plane chunks only when the tiles
    // alone leave most of them idle (the records are recomputed per chunk)
    // Round 5: a unit is (window, band, chunk of ~TU_CPP planes) and the grid has one wave per
    // unit (no wave strides over units): the records are amortised over >= 24 planes and the
    // short-lived waves stream better than resident waves walking all planes (4K b32 linear:
    // 0.592 -> 0.546 ms; 8 planes per chunk: 0.773, records dominate; profiles/r05/triup_grid_ab.txt).
    // Calls with few planes keep the old rule: chunks until the units about fill the resident
    // waves once, waves striding over units.
    constexpr int64_t RESIDENT = 256 * 4 * 4;
    const int64_t tiles = (int64_t)D.nwin * D.nband;
    int64_t nchunk = std::max<int64_t>(1, std::min<int64_t>(D.planes, (RESIDENT + tiles / 2) / tiles));
    bool grid = false;
    // ('nearest' too since its records no longer use scratch: with the 128-B-per-lane stack
    // object the grid ran u8 0.407 -> 0.789 ms, profiles/r05/triup_grid_ab.txt; r05 tu A/Bs)
    if (!env_is("HYGRID_TU_GRID", "0") && D.planes >= 2 * TU_CPP) {
        nchunk = std::max<int64_t>(nchunk, D.planes / TU_CPP);
        grid = true;
    }
    if (const char* e = getenv("HYGRID_TU_CHUNKS"))   // A/B switch: plane chunks per tile
        nchunk = std::max<int64_t>(1, std::min<int64_t>(D.planes, atoi(e)));
    // a chunk's planes are one buffer each way: 32-bit offsets, including the planes past the
    // chunk the prefetch addresses (out of range: zeros)
    const int64_t plane_bytes = std::max<int64_t>((int64_t)D.h * D.w * (int64_t)sizeof(Tin),
                                                  (int64_t)D.h1 * D.w1 * (int64_t)sizeof(Tout));
    const int64_t max_pc = std::max<int64_t>(1, (((int64_t)1 << 31) - 1) / plane_bytes - TuCfg<NEAR>::PDP - 1);
    nchunk = std::max<int64_t>(nchunk, (D.planes + max_pc - 1) / max_pc);
    D.pc = (int)((D.planes + nchunk - 1) / nchunk);
    nchunk = (D.planes + D.pc - 1) / D.pc;
    D.units = tiles * nchunk;
    int64_t waves = std::min<int64_t>(D.units, RESIDENT);
    if (grid || env_is("HYGRID_TU_GRID", "1")) waves = std::min<int64_t>(D.units, (int64_t)1 << 30);
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    hipLaunchKernelGGL((k_tri_up<Tin, Tout, K, NEAR>), dim3(blocks), dim3(TU_THREADS), 0, st,
                       (const Tin*)src, (Tout*)dst, D);
    return launch_status();
}

// An upsampling triangle resample (op HG_OP_HEX_TO_RECT or HG_OP_HEXRESIZE; 'linear' with
// fp32 accumulation, 16/32-bit float in and out; 'nearest' on 8/16/32-bit elements) on the
// streaming kernel, or HG_EUNSUP (the caller runs the general kernels).  dry: check only.
int triup_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
              int64_t w, int64_t h1, int64_t w1, int interp, hipStream_t st, bool dry) {
    if (env_is("HYGRID_DOWN", "0") || env_is("HYGRID_UP", "0")) return HG_EUNSUP;   // A/B switches
    if (op != HG_OP_HEX_TO_RECT && op != HG_OP_HEXRESIZE) return HG_EUNSUP;
    const bool near_ = interp == HG_NEAREST;
    if (near_) {
        if (sdt != ddt || (dtype_size(sdt) != 1 && dtype_size(sdt) != 2 && dtype_size(sdt) != 4))
            return HG_EUNSUP;
    } else {
        if (interp != HG_LINEAR) return HG_EUNSUP;
        if ((sdt != HG_F16 && sdt != HG_BF16 && sdt != HG_F32) ||
            (ddt != HG_F16 && ddt != HG_BF16 && ddt != HG_F32))
            return HG_EUNSUP;
    }
    if (planes < 1 || h < 2 || w < 2 || h1 < 2 || w1 < 1) return HG_EUNSUP;
    const int E = dtype_size(sdt), EO = dtype_size(ddt);
    // LDS-DMA moves whole dwords from dword-aligned addresses: every input row starts on one
    if ((w * E) % 4 || (reinterpret_cast<uintptr_t>(src) & 3)) return HG_EUNSUP;
    if ((h * w * E) * 4 >= ((int64_t)1 << 31) || (h1 * w1 * EO) * 4 >= ((int64_t)1 << 31))
        return HG_EUNSUP;
    const Geom g = make_tri(h, w, h1, w1, op == HG_OP_HEXRESIZE ? 0.5 : 0.75);
    if (!tri_fast_ok(g)) return HG_EUNSUP;
    // upsampling only: output steps of at most one input sample in both directions
    // (tri_fast_ok above: h1, w1 > 1)
    if ((double)(h - 1) > (double)(h1 - 1) || (double)(w - 1) > (double)(w1 - 1)) return HG_EUNSUP;
    TriUpGeom D = {};
    double qmax;
    if (!tsk_rows_ok(g, &D.qmin, &qmax)) return HG_EUNSUP;
    const int RB = near_ ? TuCfg<true>::RB : TuCfg<false>::RB, NR = RB / 2 + 2;
    if (!tsk_bands_ok(g, RB, NR)) return HG_EUNSUP;
    // K output columns per lane: the natural width (one dword of input samples per lane:
    // 8 / 4 / 2 for 1 / 2 / 4-byte inputs; stores of <= 16 B), or one column when that window
    // of 64 K columns does not keep its vertices in the WC input columns or K does not divide w1
    // ('nearest' used half that width while its records spilled to scratch; without the spill
    // the full width is faster: u8 0.297 -> 0.254 ms, r05 tu A/Bs)
    const int wc = TU_PCB / E, kn = std::max(1, (E == 1 ? 8 : E == 2 ? 4 : 2) / TU_KDIV);
    int K = 0;
    for (const int k : {kn, 1})
        if (!K && w1 % k == 0 && tsk_lattice_ok(g, 64 * k, wc, 4 / E, D.qmin, qmax)) K = k;
    if (!K) return HG_EUNSUP;
    D.g = g;
    D.planes = planes;
    D.h = (int)h; D.w = (int)w; D.h1 = (int)h1; D.w1 = (int)w1;
    D.nwin = (int)((w1 + 64 * K - 1) / (64 * K));
    D.nband = (int)((h1 + RB - 1) / RB);
    if (dry) return HG_OK;
#define HG_TU_K(TI, TO, KN, NR_)                                                                \
    return K == 1 ? tu_launch<TI, TO, 1, NR_>(src, dst, D, st) : tu_launch<TI, TO, KN, NR_>(src, dst, D, st);
    if (near_) {
        if (E == 1) { HG_TU_K(uint8_t, uint8_t, 8 / TU_KDIV, true) }
        if (E == 2) { HG_TU_K(unsigned short, unsigned short, 4 / TU_KDIV, true) }
        HG_TU_K(unsigned, unsigned, (2 / TU_KDIV > 0 ? 2 / TU_KDIV : 1), true)
    }
#define HG_TU_OUT(TI, KN)                                                                       \
    if (ddt == HG_BF16) { HG_TU_K(TI, __bf16, KN, false) }                                      \
    if (ddt == HG_F16) { HG_TU_K(TI, _Float16, KN, false) }                                     \
    HG_TU_K(TI, float, KN, false)
    if (sdt == HG_BF16) { HG_TU_OUT(__bf16, 4 / TU_KDIV) }
    if (sdt == HG_F16) { HG_TU_OUT(_Float16, 4 / TU_KDIV) }
    HG_TU_OUT(float, (2 / TU_KDIV > 0 ? 2 / TU_KDIV : 1))
#undef HG_TU_OUT
#undef HG_TU_K
}

}  // namespace hg
