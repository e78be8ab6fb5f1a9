// conv_mfma.hip — HexConv2d for wide channel counts (HexConvModule in segmentation
// models, HexModules.py:97-288) as an implicit GEMM on the f32 matrix cores.
//
// For one output row r of image b (HexFrames.py:96-169 restated as in hexconv.hip):
//     Y[o][q] = bias[o] + sum_{c,t} W[o][c][t] * P[c][r + dy_t][q + dk_t(r & 1)]
// i.e. a GEMM with M = O (output channels), N = q (columns), K = 7 C (taps x input
// channels), where P is the padded input and a column past the padded width is the
// type1 raster's structural zero (heximage_to_type1, HexFrames.py:417-445).
//
// v_mfma_f32_16x16x4_f32 computes it exactly as an f32 fmaf chain (MI355X matrix cores
// take f32 operands at the vector rate, cdna_hip_programming.md §3), so the result has
// the reference's fp32 semantics (F.conv2d in fp32, :107, :157-160) up to summation
// order, for every input dtype (16-bit inputs are staged as their exact f32 values).
//
// Workgroup = 4 waves = 4 consecutive output rows (one per wave: its parity fixes its tap
// columns) x 32 or 64 output channels.  Per chunk of CM_CC = 8 input channels the
// workgroup stages P (6 rows x 72 columns x 8 channels, padding applied) and the
// weights (8 x 7 x 64) in LDS; each wave then runs 7 taps x 2 channel quads x
// (2-4 x 4 tiles of 16x16) MFMAs into up to 64 accumulator registers.  Fragment maps
// (MI355X_MICROARCH.md / cdna_hip_programming.md §3): A[i=o][k] from lane (k*16 + i),
// B[k][j=q] from lane (k*16 + j), D[4*(l/16)+v][l%16] in register v of lane l.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "common.h"
#include "hexconv_geom.h"

namespace hg {

constexpr int CM_THREADS = 256;
constexpr int CM_ROWS = 4;                  // output rows per workgroup (one per wave)
constexpr int CM_Q = 64;                    // output columns per workgroup
constexpr int CM_OMAX = 64;                 // output channels per workgroup (NOT = 4 tiles;
                                            // 2 tiles = 32 channels when O <= 32)
constexpr int CM_CC = 8;                    // input channels per LDS chunk (28.6 KB LDS: 4 WGs per CU)
constexpr int CM_PR = CM_ROWS + 2;          // staged P rows (taps reach rows r .. r+2)
constexpr int CM_PP = 72;                   // staged P pitch: 64 + tap column span (<= 4),
                                            // 6*72 = 432 = 16 mod 32 banks: conflict-free B reads
constexpr int CM_CST = CM_PR * CM_PP;       // P channel stride
constexpr int CM_WST = 7 * CM_OMAX + 16;    // weight channel stride (= 16 mod 32 banks)

typedef float cm_f4 __attribute__((ext_vector_type(4)));
#ifndef CM_TD
#define CM_TD 1                             // MFMA kernels, 16-bit outputs: D as [column][channel] (below)
#endif

struct MfmaGeom {
    int64_t B;
    int C, O, h, w, ho, wo, p, pad_mode;
    int mink;                   // smallest tap column offset over both parities
    int dy[7], dk[2][7];        // tap rows / columns (padded frame, relative to mink)
    int ntq, ntr, nto;          // tiles along columns / rows / output channels
    float pad_value;
    Epilogue epi;
};

// CM_TD epilogue (16-bit outputs): lane (li, lk) holds output channel oc + 16 ot, columns
// q + 16 qt .. + 3 in its 4 registers: one 8-B store per (ot, qt) when every row's start keeps
// q % 4 == 0 aligned (wo % 4 == 0); scalar stores otherwise
template <typename Tout, int NOT, int NQT>
__device__ __forceinline__ void cm_store_cols(const cm_f4 (&acc)[NOT][NQT], Tout* yb, const MfmaGeom& G,
                                              int oc, int q, int r) {
    const bool vec = (G.wo & 3) == 0;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
        const int o = oc + ot * 16;
        if (o >= G.O) continue;
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
            const int qq = q + qt * 16;
            if (qq >= G.wo) continue;
            float val[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                val[v] = acc[ot][qt][v];
                if (G.epi.on) val[v] = epi_apply(val[v], o, G.epi);
            }
            Tout* const dst = yb + ((int64_t)o * G.ho + r) * G.wo + qq;
            if (vec && sizeof(Tout) == 2) {
                typedef Tout t4v __attribute__((ext_vector_type(4)));
                *reinterpret_cast<t4v*>(dst) = t4v{(Tout)val[0], (Tout)val[1], (Tout)val[2], (Tout)val[3]};
            } else {
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    if (qq + v < G.wo) dst[v] = (Tout)val[v];
            }
        }
    }
}

template <typename Tin, typename Tout, int NOT>
__global__ __launch_bounds__(CM_THREADS) void k_hexconv_mfma(const Tin* __restrict__ x,
                                                                const float* __restrict__ kern,
                                                                const float* __restrict__ bias,
                                                                Tout* __restrict__ y, MfmaGeom G) {
    __shared__ float ps[CM_CC * CM_CST];                 // P chunk [c][row][col]
    __shared__ float ws[CM_CC * CM_WST];                 // weight chunk [c][t][o]
    constexpr int CM_O = 16 * NOT;                       // output channels of this workgroup
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int tq = (int)(bid % G.ntq); bid /= G.ntq;
    const int tr = (int)(bid % G.ntr); bid /= G.ntr;
    const int to = (int)(bid % G.nto);
    const int64_t b = bid / G.nto;
    const int q0 = tq * CM_Q, r0 = tr * CM_ROWS, o0 = to * (16 * NOT);
    const int r = r0 + wv;                               // this wave's output row
    const int par = r & 1;
    const int Wp = G.w + 2 * G.p, Hp = G.h + 2 * G.p;
    const int li = lane & 15, lk = lane >> 4;            // fragment row / k of this lane

    // 16-bit outputs only (fp32 outputs as two 8-B stores: 3.9 % slower than 2-B stores,
    // profiles/r06/conv_mfma_transposed_d_ab.txt)
    constexpr bool TD = CM_TD && sizeof(Tout) == 2;
    cm_f4 acc[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + (TD ? li : lk * 4 + v);   // TD: D is [column][channel]
            const float bv = (bias && o < G.O) ? bias[o] : 0.f;
#pragma unroll
            for (int qt = 0; qt < 4; ++qt) acc[ot][qt][v] = bv;
        }
    }

    const Tin* xb = x + b * (int64_t)G.C * G.h * G.w;
    for (int c0 = 0; c0 < G.C; c0 += CM_CC) {
        // ---- stage P rows r0 .. r0+5 (padded frame), columns q0 + mink + (0..71) ---------
        // 216 threads = 72 columns x 3 row phases; each thread keeps its column's source
        // index (padding rules applied once) and walks rows pr = phase, phase + 3, ... of
        // every channel of the chunk.  (Loading the next chunk into registers during the
        // MFMAs instead needs ~60 more VGPRs and spilled at 2 waves per SIMD.)
        if (tid < 3 * CM_PP) {
            const int pc = tid % CM_PP, ph = tid / CM_PP;
            const int px = q0 + G.mink + pc;
            const bool zc = px >= Wp;                        // type1 structural zero column
            const int64_t xi = zc ? -1 : pad_map(px - G.p, G.w, G.pad_mode);
#pragma unroll 4
            for (int rr = ph; rr < CM_CC * CM_PR; rr += 3) {
                const int cc = rr / CM_PR, pr = rr - cc * CM_PR;
                const int c = c0 + cc, py = r0 + pr;
                float v = 0.f;
                if (!zc && c < G.C && py < Hp) {
                    const int64_t yi = pad_map(py - G.p, G.h, G.pad_mode);
                    v = (yi < 0 || xi < 0) ? G.pad_value
                                           : (float)xb[((int64_t)c * G.h + yi) * G.w + xi];
                }
                ps[cc * CM_CST + pr * CM_PP + pc] = v;
            }
        }
        // ---- stage weights W[o0 .. o0+63][c0 .. c0+CM_CC-1][t] as [c][t][o] --------------
        // per output channel the chunk's CM_CC x 7 = 56 weights are contiguous: 14 float4 loads
        for (int e = tid; e < CM_O * (CM_CC * 7 / 4); e += CM_THREADS) {
            const int o = e / (CM_CC * 7 / 4), f = e - o * (CM_CC * 7 / 4);
            const int og = o0 + o;
            float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
            const int64_t base = ((int64_t)og * G.C + c0) * 7 + 4 * f;   // first of 4 (c, t)
            if (og < G.O) {
                if (c0 + CM_CC <= G.C && (base & 3) == 0) {
                    v4 = *reinterpret_cast<const float4*>(kern + base);
                } else {
                    float tmp[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int ct = 4 * f + j, c = c0 + ct / 7;
                        tmp[j] = c < G.C ? kern[((int64_t)og * G.C + c) * 7 + ct % 7] : 0.f;
                    }
                    v4 = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
                }
            }
            const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ct = 4 * f + j, cc = ct / 7, t = ct - cc * 7;
                ws[cc * CM_WST + t * CM_O + o] = vv[j];
            }
        }
        __syncthreads();
        // ---- 7 taps x 4 channel quads x 16 MFMAs --------------------------------------
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int dy = G.dy[t], dk = par ? G.dk[1][t] : G.dk[0][t];
            const float* pb = ps + lk * CM_CST + (wv + dy) * CM_PP + dk + li;
            const float* wb = ws + lk * CM_WST + t * CM_O + li;
#pragma unroll
            for (int cq = 0; cq < CM_CC / 4; ++cq) {
                float af[NOT], bf[4];
#pragma unroll
                for (int ot = 0; ot < NOT; ++ot) af[ot] = wb[cq * 4 * CM_WST + ot * 16];
#pragma unroll
                for (int qt = 0; qt < 4; ++qt) bf[qt] = pb[cq * 4 * CM_CST + qt * 16];
#pragma unroll
                for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
                    for (int qt = 0; qt < 4; ++qt)
                        acc[ot][qt] = TD ? __builtin_amdgcn_mfma_f32_16x16x4f32(bf[qt], af[ot], acc[ot][qt], 0, 0, 0)
                                            : __builtin_amdgcn_mfma_f32_16x16x4f32(af[ot], bf[qt], acc[ot][qt], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // ---- epilogue: bias was the accumulator's start; BN / activation; store -------------
    if (r >= G.ho) return;
    Tout* yb = y + b * (int64_t)G.O * G.ho * G.wo;
    if constexpr (TD) {
        cm_store_cols<Tout, NOT, 4>(acc, yb, G, o0 + li, q0 + lk * 4, r);
        return;
    }
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + lk * 4 + v;
            if (o >= G.O) continue;
#pragma unroll
            for (int qt = 0; qt < 4; ++qt) {
                const int q = q0 + qt * 16 + li;
                if (q >= G.wo) continue;
                float val = acc[ot][qt][v];
                if (G.epi.on) val = epi_apply(val, o, G.epi);
                yb[((int64_t)o * G.ho + r) * G.wo + q] = (Tout)val;
            }
        }
}

typedef __bf16 cm_b8 __attribute__((ext_vector_type(8)));
typedef unsigned cm_u4 __attribute__((ext_vector_type(4)));
// The bf16 kernels' weight-fragment LDS layout: channel o's four k-group fragments (16 B each)
// in a rotated order, so each of ds_read_b128's four 16-lane groups ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, and the same + 32: MI355X_MICROARCH.md section LDS) reads 16 distinct
// 16-B bank slots; the plain order o * 4 + g put lanes li and li + 12 (and li + 4, li + 8) of a
// group on one slot (2-way conflicts; r04 session O counters: 39 % of the LDS cycles).
__host__ __device__ constexpr int cd_wslot(int o, int g) { return (g + 2 * ((o & 15) >> 2)) & 3; }

constexpr int CB_PP = 72;                   // staged columns (as CM_PP)
constexpr int CB_PSZ = CM_PR * CB_PP + 1;   // P fragments per chunk (+1: the zero fragment)

template <typename Tout, int NOT>
__global__ __launch_bounds__(CM_THREADS) void k_hexconv_mfma_bf16(const __bf16* __restrict__ x,
                                                                  const float* __restrict__ kern,
                                                                  const float* __restrict__ bias,
                                                                  Tout* __restrict__ y, MfmaGeom G) {
    constexpr int CM_O = 16 * NOT;                       // output channels of this workgroup
    // P chunk: [row][col] fragments of the 8 channels (16 B each, channel innermost);
    // weights: [part][kb][o][g] fragments of the 8 channels of tap 4 kb + g
    __shared__ cm_u4 psb[CB_PSZ];
    __shared__ cm_u4 wsb[3 * 2 * CM_O * 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int tq = (int)(bid % G.ntq); bid /= G.ntq;
    const int tr = (int)(bid % G.ntr); bid /= G.ntr;
    const int to = (int)(bid % G.nto);
    const int64_t b = bid / G.nto;
    const int q0 = tq * CM_Q, r0 = tr * CM_ROWS, o0 = to * CM_O;
    const int r = r0 + wv;
    const int par = r & 1;
    const int Wp = G.w + 2 * G.p, Hp = G.h + 2 * G.p;
    const int li = lane & 15, lg = lane >> 4;            // fragment row / column, k group
    const unsigned short padv = __builtin_bit_cast(unsigned short, (__bf16)G.pad_value);

    cm_f4 acc[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + lg * 4 + v;
            const float bv = (bias && o < G.O) ? bias[o] : 0.f;
#pragma unroll
            for (int qt = 0; qt < 4; ++qt) acc[ot][qt][v] = bv;
        }
    }
    if (tid == 0) psb[CB_PSZ - 1] = cm_u4{0u, 0u, 0u, 0u};
    // this lane's P fragment (per k block and column tile): tap t = 4 kb + lg, row wv + dy_t,
    // column qt * 16 + li + dk_t; the 8th tap slot reads the zero fragment
    int pidx[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        const int t = 4 * kb + lg;
        pidx[kb] = t < 7 ? (wv + G.dy[t]) * CB_PP + li + (par ? G.dk[1][t] : G.dk[0][t]) : -1;
    }

    const unsigned short* xb = reinterpret_cast<const unsigned short*>(x) + b * (int64_t)G.C * G.h * G.w;
    for (int c0 = 0; c0 < G.C; c0 += CM_CC) {
        // ---- stage P rows r0 .. r0+5, columns q0 + mink + (0..71), 8 channels ------------
        if (tid < 3 * CB_PP) {
            const int pc = tid % CB_PP, ph = tid / CB_PP;
            const int px = q0 + G.mink + pc;
            const bool zc = px >= Wp;                        // type1 structural zero column
            const int64_t xi = zc ? -1 : pad_map(px - G.p, G.w, G.pad_mode);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int pr = ph + 3 * k, py = r0 + pr;
                const int64_t yi = (!zc && py < Hp) ? pad_map(py - G.p, G.h, G.pad_mode) : -1;
                unsigned short v[8];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const int c = c0 + cc;
                    unsigned short e = 0;
                    if (!zc && c < G.C && py < Hp)
                        e = (yi < 0 || xi < 0) ? padv : xb[((int64_t)c * G.h + yi) * G.w + xi];
                    v[cc] = e;
                }
                psb[pr * CB_PP + pc] = cm_u4{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                                             v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)};
            }
        }
        // ---- stage the weights of taps (o, t), 8 channels, as 3 bf16 parts ----------------
        // (ml: some weight of the chunk needs its second / third part; when none does, the
        // pt = 1, 2 passes are skipped: half the MFMA work for bf16-exact weights, and an
        // infinite input times a weight then stays +-Inf as in one fp32 product instead of
        // meeting a zero part as Inf * 0 = NaN)
        int ml = 0;
        for (int e = tid; e < CM_O * 8; e += CM_THREADS) {
            const int o = e >> 3, t = e & 7, og = o0 + o;
            unsigned short h[8], m[8], l[8];
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
                const int c = c0 + cc;
                const float wf = (t < 7 && og < G.O && c < G.C) ? kern[((int64_t)og * G.C + c) * 7 + t] : 0.f;
                const __bf16 bh = (__bf16)wf;
                const float r1 = wf - (float)bh;
                const __bf16 bm = (__bf16)r1;
                const __bf16 bl = (__bf16)(r1 - (float)bm);
                h[cc] = __builtin_bit_cast(unsigned short, bh);
                m[cc] = __builtin_bit_cast(unsigned short, bm);
                l[cc] = __builtin_bit_cast(unsigned short, bl);
                ml |= (m[cc] | l[cc]) & 0x7fff;              // a nonzero part (+-0 is zero)
            }
            const int kb = t >> 2, g = t & 3;
            auto pk = [](const unsigned short* u) {
                return cm_u4{u[0] | ((unsigned)u[1] << 16), u[2] | ((unsigned)u[3] << 16),
                             u[4] | ((unsigned)u[5] << 16), u[6] | ((unsigned)u[7] << 16)};
            };
            wsb[((0 * 2 + kb) * CM_O + o) * 4 + cd_wslot(o, g)] = pk(h);
            wsb[((1 * 2 + kb) * CM_O + o) * 4 + cd_wslot(o, g)] = pk(m);
            wsb[((2 * 2 + kb) * CM_O + o) * 4 + cd_wslot(o, g)] = pk(l);
        }
        const int nparts = __syncthreads_or(ml != 0) ? 3 : 1;   // uniform per workgroup
        // ---- 2 k blocks x 4 column tiles x 3 weight parts x NOT channel tiles -------------
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            cm_b8 bf[4];
#pragma unroll
            for (int qt = 0; qt < 4; ++qt)
                bf[qt] = __builtin_bit_cast(cm_b8, psb[pidx[kb] < 0 ? CB_PSZ - 1 : pidx[kb] + qt * 16]);
#pragma unroll
            for (int pt = 0; pt < 3; ++pt) {
                if (pt >= nparts) break;
#pragma unroll
                for (int ot = 0; ot < NOT; ++ot) {
                    const cm_b8 af = __builtin_bit_cast(cm_b8, wsb[((pt * 2 + kb) * CM_O + ot * 16 + li) * 4 + cd_wslot(li, lg)]);
#pragma unroll
                    for (int qt = 0; qt < 4; ++qt)
                        acc[ot][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[qt], acc[ot][qt], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    if (r >= G.ho) return;
    Tout* yb = y + b * (int64_t)G.O * G.ho * G.wo;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + lg * 4 + v;
            if (o >= G.O) continue;
#pragma unroll
            for (int qt = 0; qt < 4; ++qt) {
                const int q = q0 + qt * 16 + li;
                if (q >= G.wo) continue;
                float val = acc[ot][qt][v];
                if (G.epi.on) val = epi_apply(val, o, G.epi);
                yb[((int64_t)o * G.ho + r) * G.wo + q] = (Tout)val;
            }
        }
}

// ---- bf16 inputs, staging by LDS-DMA (round 4) -------------------------------------------
// The same GEMM and fragment maps as k_hexconv_mfma_bf16, with the staging taken off the
// critical path: (1) the three bf16 weight parts are split once per call by k_wsplit_bf16
// into a stream-ordered scratch buffer already in the LDS fragment layout, so a workgroup's
// weight chunk is a plain 1-KiB-piece LDS-DMA copy (double-buffered: chunk i + 1 lands while
// chunk i's MFMAs run); (2) P's rows arrive by LDS-DMA in their natural [channel][row][col]
// order (one dword per lane, 40 lanes = 80 columns per piece), also one chunk ahead, and a
// short LDS -> LDS pass packs them channel-innermost for the ds_read_b128 B fragments.  No
// staging value passes through VGPRs, so the prefetch costs no occupancy (the register
// prefetch of round 3 did: 2 waves per SIMD, 27 % slower).  Workgroups whose P tile needs
// padding or the type1 structural zero column keep the register staging for P.
constexpr int CD_PRW = 40;                    // raw P row: 40 dwords = 80 columns (>= 72 + 1)
constexpr int CD_PRAW = CM_CC * CM_PR * CD_PRW;   // dwords of one raw P chunk

// one block per (chunk of 8 input channels, 16 output channels); thread (o, t) splits the
// 8 channels' weights of tap t (t = 7: zeros) into h + m + l and stores the three fragments;
// flag[chunk][o / 16] = some m / l part is nonzero (else the MFMA kernel skips parts 2, 3)
__global__ __launch_bounds__(128) void k_wsplit_bf16(const float* __restrict__ kern, cm_u4* __restrict__ wf,
                                                     int* __restrict__ flag, int C, int O, int Opad) {
    const int ci = blockIdx.x, ob = blockIdx.y;
    const int o = ob * 16 + (threadIdx.x >> 3), t = threadIdx.x & 7;
    unsigned short h[8], m[8], l[8];
    int ml = 0;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
        const int c = ci * 8 + cc;
        const float wv = (t < 7 && o < O && c < C) ? kern[((int64_t)o * C + c) * 7 + t] : 0.f;
        const __bf16 bh = (__bf16)wv;
        const float r1 = wv - (float)bh;
        const __bf16 bm = (__bf16)r1;
        const __bf16 bl = (__bf16)(r1 - (float)bm);
        h[cc] = __builtin_bit_cast(unsigned short, bh);
        m[cc] = __builtin_bit_cast(unsigned short, bm);
        l[cc] = __builtin_bit_cast(unsigned short, bl);
        ml |= (m[cc] | l[cc]) & 0x7fff;
    }
    auto pk = [](const unsigned short* u) {
        return cm_u4{u[0] | ((unsigned)u[1] << 16), u[2] | ((unsigned)u[3] << 16),
                     u[4] | ((unsigned)u[5] << 16), u[6] | ((unsigned)u[7] << 16)};
    };
    const int kb = t >> 2, g = t & 3;
    auto at = [&](int pt) { return ((((int64_t)ci * 3 + pt) * 2 + kb) * Opad + o) * 4 + cd_wslot(o, g); };
    wf[at(0)] = pk(h);
    wf[at(1)] = pk(m);
    wf[at(2)] = pk(l);
    const int any = __syncthreads_or(ml != 0);
    if (threadIdx.x == 0) flag[ci * (Opad / 16) + ob] = any;
}

template <int N>
__device__ __forceinline__ void cd_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((0x0f70 & ~0xf) | (N & 0xf) | ((N >> 4) << 14));
}

// Weight chunks are single-buffered: the DMA of chunk i + 1 is issued once chunk i's MFMAs are
// done and waited for at the top of the next chunk (47 KB of LDS -> 3 workgroups per CU, whose
// MFMAs cover each other's waits; double-buffered, 71 KB and 2 workgroups per CU, was 18 %
// slower, and 3 column tiles with one raw-P buffer for a 4th wave per SIMD 4 % slower: both
// removed in round 6).  The raw P rows are double-buffered.
template <typename Tout, int NOT>
__global__ __launch_bounds__(CM_THREADS) __attribute__((amdgpu_waves_per_eu(1)))
void k_hexconv_mfma_bf16d(const __bf16* __restrict__ x,
                                                                   const cm_u4* __restrict__ wf,
                                                                   const int* __restrict__ flag,
                                                                   const float* __restrict__ bias,
                                                                   Tout* __restrict__ y, MfmaGeom G,
                                                                   int Opad) {
    constexpr int CM_O = 16 * NOT;
    constexpr int WSZ = 3 * 2 * CM_O * 4;                // weight fragments of one chunk
    constexpr int WPC = WSZ / 64;                         // their 1-KiB pieces
    constexpr int WPW = WPC / 4;                          // ... per wave
    constexpr int PPW = CM_CC * CM_PR / 4;                // raw P row pieces per wave (12)
    static_assert(WPC % 4 == 0, "pieces");
    // one LDS array (so the DMA's M0 bases come from it): [psb | wsb x 2 | praw x 2]
    constexpr int NQT = 4;                                // 16-column tiles per workgroup
    constexpr int LPSB = CB_PSZ * 16, LWSB = WSZ * 16, LPRAW = CD_PRAW * 4, NWB = 1;
    constexpr int NPB = 2;                                // raw P buffers
    constexpr int TQ = 16 * NQT;                          // output columns of this workgroup
    __shared__ __attribute__((aligned(16))) unsigned char lds[LPSB + NWB * LWSB + NPB * LPRAW];
    cm_u4* const psb = reinterpret_cast<cm_u4*>(lds);
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int tq = (int)(bid % G.ntq); bid /= G.ntq;
    const int tr = (int)(bid % G.ntr); bid /= G.ntr;
    const int to = (int)(bid % G.nto);
    const int64_t b = bid / G.nto;
    const int q0 = tq * TQ, r0 = tr * CM_ROWS, o0 = to * CM_O;
    const int r = r0 + wv;
    const int par = r & 1;
    const int Wp = G.w + 2 * G.p, Hp = G.h + 2 * G.p;
    const int li = lane & 15, lg = lane >> 4;
    const unsigned short padv = __builtin_bit_cast(unsigned short, (__bf16)G.pad_value);
    const int nch = (G.C + CM_CC - 1) / CM_CC;
    // this tile's P is all inside the image (no padding, no structural zero): DMA staging
    const int px0 = q0 + G.mink - G.p;                    // first staged source column
    const bool interior = r0 - G.p >= 0 && r0 + CM_PR - 1 - G.p < G.h && px0 >= 0 &&
                          px0 + CB_PP - 1 < G.w && q0 + G.mink + CB_PP - 1 < Wp;
    const int xs = px0 & ~1, sh = px0 - xs;               // dword-aligned raw start, shift

    // CM_TD: the MFMAs take the P fragment as A and the weights as B, so D is [column][channel]:
    // a lane's 4 registers are 4 adjacent output columns of one channel (one 8-B store for
    // 16-bit outputs instead of four 2-B stores); the same products summed in the same order
    // 16-bit outputs only (fp32 outputs as two 8-B stores: 3.9 % slower than 2-B stores,
    // profiles/r06/conv_mfma_transposed_d_ab.txt)
    constexpr bool TD = CM_TD && sizeof(Tout) == 2;
    cm_f4 acc[NOT][NQT];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + (TD ? li : lg * 4 + v);
            const float bv = (bias && o < G.O) ? bias[o] : 0.f;
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt) acc[ot][qt][v] = bv;
        }
    }
    if (tid == 0) psb[CB_PSZ - 1] = cm_u4{0u, 0u, 0u, 0u};
    int pidx[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        const int t = 4 * kb + lg;
        pidx[kb] = t < 7 ? (wv + G.dy[t]) * CB_PP + li + (par ? G.dk[1][t] : G.dk[0][t]) : -1;
    }
    const unsigned short* xb = reinterpret_cast<const unsigned short*>(x) + b * (int64_t)G.C * G.h * G.w;
    // buffer views: the image's planes (rows of channels >= C read past the range: zeros),
    // the weight fragments
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)xb, (short)0, (int)((int64_t)G.C * G.h * G.w * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)wf, (short)0, 0x7fffffff, 0x00020000);

    // the DMA address terms are recomputed at every chunk from values the compiler cannot see
    // through (no hoisting: the hoisted per-piece offsets spilled 57-73 SGPRs, round 5)
    auto opq = [](int v) {
        asm volatile("" : "+s"(v));
        return v;
    };
    auto dma_w = [&](int ci) {                            // chunk ci's weights -> the buffer
        const int wvo = opq(wv);
        // weights: pieces j = wv * WPW + i of the chunk's (pt, kb) blocks of CM_O * 4 fragments
#pragma unroll
        for (int i = 0; i < WPW; ++i) {
            const int j = wvo * WPW + i;
            const int blk = j / (CM_O / 16), part = j % (CM_O / 16);   // (pt * 2 + kb), 1-KiB part
            const unsigned so = (unsigned)((((int64_t)ci * 6 + blk) * Opad + o0) * 64 + part * 1024);
            const unsigned lda = lds0 + LPSB + (blk * CM_O * 4) * 16 + part * 1024;
            const unsigned vo = lane * 16u;
            unsigned keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                         "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo), "s"(wr), "s"(lda), "s"(so) : "memory");
        }
    };
    auto dma_p = [&](int ci) {                            // chunk ci's raw P rows -> buffer (ci & 1)
        const int buf = ci & 1;
        if (interior) {
            const int wvo = opq(wv), ho = opq(G.h), wo = opq(G.w);
            // P rows: pieces j = wv * PPW + i = (cc, pr); lanes 0-39 one dword each
#pragma unroll
            for (int i = 0; i < PPW; ++i) {
                const int j = wvo * PPW + i;
                const int cc = j / CM_PR, pr = j % CM_PR;
                const int c = ci * CM_CC + cc;
                const unsigned so = c < G.C ? (unsigned)((((int64_t)c * ho + (r0 + pr - G.p)) * wo + xs) * 2)
                                            : 0x80000000u;
                const unsigned lda = lds0 + LPSB + NWB * LWSB + buf * LPRAW + j * CD_PRW * 4;
                const unsigned vo = lane * 4u;
                unsigned keep;
                if (lane < CD_PRW)
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                                 "buffer_load_dword %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(vo), "s"(xr), "s"(lda), "s"(so) : "memory");
                else
                    asm volatile("" ::: "memory");
            }
        }
    };
    // every wave issues the same number of DMA instructions per chunk (counted waits)
    constexpr int NP_ = PPW;

    dma_w(0);
    dma_p(0);
    for (int ci = 0; ci < nch; ++ci) {
        const int buf = ci & 1;
        const int c0 = ci * CM_CC;
        // chunk ci's pieces are done once at most the ones issued after them are outstanding
        // (vmcnt counts them in issue order): only P(ci+1) (W(ci) was issued at the end of
        // chunk ci-1, before P(ci+1))
        if (ci + 1 < nch) {
            dma_p(ci + 1);
            if (interior) cd_wait_vm<NP_>(); else cd_wait_vm<0>();
        } else {
            cd_wait_vm<0>();
        }
        // ---- P chunk -> psb (channel-innermost fragments) -------------------------------
        if (interior) {
            __builtin_amdgcn_s_barrier();                 // every wave's raw rows have landed
            const unsigned short* raw = reinterpret_cast<const unsigned short*>(lds + LPSB + NWB * LWSB + buf * LPRAW);
            for (int f = tid; f < CM_PR * CB_PP; f += CM_THREADS) {
                const int pr = f / CB_PP, pc = f - pr * CB_PP;
                unsigned short v[8];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) v[cc] = raw[(cc * CM_PR + pr) * (2 * CD_PRW) + pc + sh];
                psb[f] = cm_u4{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                               v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)};
            }
        }
        if (!interior && tid < 3 * CB_PP) {               // the register staging (padding rules)
            const int pc = tid % CB_PP, ph = tid / CB_PP;
            const int px = q0 + G.mink + pc;
            const bool zc = px >= Wp;
            const int64_t xi = zc ? -1 : pad_map(px - G.p, G.w, G.pad_mode);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int pr = ph + 3 * k, py = r0 + pr;
                const int64_t yi = (!zc && py < Hp) ? pad_map(py - G.p, G.h, G.pad_mode) : -1;
                unsigned short v[8];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const int c = c0 + cc;
                    unsigned short e = 0;
                    if (!zc && c < G.C && py < Hp)
                        e = (yi < 0 || xi < 0) ? padv : xb[((int64_t)c * G.h + yi) * G.w + xi];
                    v[cc] = e;
                }
                psb[pr * CB_PP + pc] = cm_u4{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                                             v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)};
            }
        }
        int nparts = 1;
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) nparts |= flag[ci * (Opad / 16) + o0 / 16 + ot] ? 3 : 1;
        __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): this wave's LDS writes
        __builtin_amdgcn_s_barrier();                     // psb and the weights complete
        // ---- 2 k blocks x NQT column tiles x 3 weight parts x NOT channel tiles -----------
        const cm_u4* const wsb = reinterpret_cast<const cm_u4*>(lds + LPSB);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            cm_b8 bf[NQT];
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt)
                bf[qt] = __builtin_bit_cast(cm_b8, psb[pidx[kb] < 0 ? CB_PSZ - 1 : pidx[kb] + qt * 16]);
#pragma unroll
            for (int pt = 0; pt < 3; ++pt) {
                if (pt >= nparts) break;
#pragma unroll
                for (int ot = 0; ot < NOT; ++ot) {
                    const cm_b8 af = __builtin_bit_cast(cm_b8, wsb[((pt * 2 + kb) * CM_O + ot * 16 + li) * 4 + cd_wslot(li, lg)]);
#pragma unroll
                    for (int qt = 0; qt < NQT; ++qt)
                        acc[ot][qt] = TD ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[qt], af, acc[ot][qt], 0, 0, 0)
                                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[qt], acc[ot][qt], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();                     // psb / this buffer free again
        if (ci + 1 < nch) dma_w(ci + 1);                  // the single weight buffer is free
    }

    if (r >= G.ho) return;
    Tout* yb = y + b * (int64_t)G.O * G.ho * G.wo;
    if constexpr (TD) {
        cm_store_cols<Tout, NOT, NQT>(acc, yb, G, o0 + li, q0 + lg * 4, r);
        return;
    }
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + lg * 4 + v;
            if (o >= G.O) continue;
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt) {
                const int q = q0 + qt * 16 + li;
                if (q >= G.wo) continue;
                float val = acc[ot][qt][v];
                if (G.epi.on) val = epi_apply(val, o, G.epi);
                yb[((int64_t)o * G.ho + r) * G.wo + q] = (Tout)val;
            }
        }
}

// Runs the MFMA kernel when it covers the call and pays (dense radius-2, stride-1,
// dilation-1 conv with O >= 16, f32 weights); HG_EUNSUP otherwise.  Narrow inputs (C < 8: the
// 3-channel stem of a segmentation model, HexModules.py:97-288) run here too, their channel
// chunk padded with zeros (staging and weights read 0 past C): HexConv2d(3 -> 64) 1080p b4
// 2.76 -> 0.50 ms (bf16) and 2.84 -> 1.02 ms (f32) against the generic kernel, round 6,
// profiles/r06/stem_conv_ab.txt.
int conv_mfma_try(const void* x, const float* k, const float* b, void* y, int x_dtype,
                  int y_dtype, int64_t B, int64_t C, int64_t O, int64_t h, int64_t w, int radius,
                  int stride, int padding, int dilation, int groups, int off, int pad_mode,
                  double pad_value, const Epilogue& epi, hipStream_t st) {
    if (env_is("HYGRID_CONV_MFMA", "0")) return HG_EUNSUP;   // A/B switch: generic kernels
    if (radius != 2 || stride != 1 || dilation != 1 || groups != 1) return HG_EUNSUP;
    if (C < 1 || O < 16 || padding < 0 || padding > 2) return HG_EUNSUP;
    if (C > INT_MAX / 16 || O > INT_MAX / 16 || h > INT_MAX / 4 || w > INT_MAX / 4) return HG_EUNSUP;
    if (C * h * w * 4 >= ((int64_t)1 << 31)) return HG_EUNSUP;   // 32-bit buffer offsets
    MfmaGeom G = {};
    G.B = B; G.C = (int)C; G.O = (int)O; G.h = (int)h; G.w = (int)w; G.p = padding;
    G.pad_mode = pad_mode; G.pad_value = (float)pad_value; G.epi = epi;
    int64_t ho, wo;
    if (conv_out_shape(h, w, radius, stride, padding, dilation, &ho, &wo)) return HG_EUNSUP;
    G.ho = (int)ho; G.wo = (int)wo;
    const int op = (off + padding) & 1;
    int mink = INT_MAX, maxk = INT_MIN;
    int dyv[7], dk0[7], dk1[7];
    for (int t = 0; t < 7; ++t) {
        tap_geom(radius, stride, dilation, op, t, &dyv[t], &dk0[t], &dk1[t]);
        mink = std::min(mink, std::min(dk0[t], dk1[t]));
        maxk = std::max(maxk, std::max(dk0[t], dk1[t]));
    }
    if (maxk - mink + CM_Q > CM_PP) return HG_EUNSUP;
    G.mink = mink;
    for (int t = 0; t < 7; ++t) {
        G.dy[t] = dyv[t];
        G.dk[0][t] = dk0[t] - mink;
        G.dk[1][t] = dk1[t] - mink;
    }
    G.ntq = (G.wo + CM_Q - 1) / CM_Q;
    G.ntr = (G.ho + CM_ROWS - 1) / CM_ROWS;
    // output-channel tiles per workgroup (A/B switch HYGRID_CONV_NT=2: two for any O)
    const int nt = (G.O <= 32 || env_is("HYGRID_CONV_NT", "2")) ? 2 : 4;
    G.nto = (G.O + 16 * nt - 1) / (16 * nt);
    const int64_t blocks = B * (int64_t)G.ntq * G.ntr * G.nto;
    if (blocks > INT_MAX || blocks == 0) return blocks == 0 ? HG_OK : HG_EUNSUP;
    const dim3 grid((unsigned)blocks), blk(CM_THREADS);
    // bf16 inputs: the split-weight bf16 kernel, when the pad value is a bf16 (the padded
    // input keeps the input's dtype, as F.pad does; anything else keeps the f32 kernel)
    const bool bf_pad = (double)(float)(__bf16)(float)pad_value == pad_value;
    // A/B switch HYGRID_CONV_MFMA_BF16=0: the f32 kernel
    if (x_dtype == HG_BF16 && bf_pad && !env_is("HYGRID_CONV_MFMA_BF16", "0") &&
        (y_dtype == HG_BF16 || y_dtype == HG_F32)) {
        // LDS-DMA staging (A/B switch HYGRID_CONV_DMA=0: the register-staged kernel below):
        // rows must be dword-aligned (even width, 4-B aligned base)
        if (!env_is("HYGRID_CONV_DMA", "0") && (G.w % 2) == 0 && (reinterpret_cast<uintptr_t>(x) & 3) == 0) {
            const int nch = (G.C + CM_CC - 1) / CM_CC, Opad = G.nto * 16 * nt;
            const size_t wbytes = (size_t)nch * 6 * Opad * 64, fbytes = (size_t)nch * (Opad / 16) * 4;
            void* ws = nullptr;
            hipError_t e = hipMallocAsync(&ws, wbytes + fbytes, st);
            if (e != hipSuccess) return (int)e;
            cm_u4* wfr = static_cast<cm_u4*>(ws);
            int* flg = reinterpret_cast<int*>(static_cast<char*>(ws) + wbytes);
            hipLaunchKernelGGL(k_wsplit_bf16, dim3(nch, Opad / 16), dim3(128), 0, st, k, wfr, flg, G.C, G.O, Opad);
#define HG_CD_LAUNCH2(TO, NT_)                                                                \
            hipLaunchKernelGGL((k_hexconv_mfma_bf16d<TO, NT_>), grid, blk, 0, st, (const __bf16*)x, wfr, flg, b, (TO*)y, G, Opad);
#define HG_CD_LAUNCH(TO)                                                                      \
            if (nt == 2) { HG_CD_LAUNCH2(TO, 2) } else { HG_CD_LAUNCH2(TO, 4) }
            if (y_dtype == HG_BF16) { HG_CD_LAUNCH(__bf16) } else { HG_CD_LAUNCH(float) }
#undef HG_CD_LAUNCH
#undef HG_CD_LAUNCH2
            const int ls = launch_status();
            const hipError_t fe = hipFreeAsync(ws, st);
            return ls != HG_OK ? ls : (int)fe;
        }
#define HG_CB_LAUNCH(TO)                                                                      \
        if (nt == 2)                                                                          \
            hipLaunchKernelGGL((k_hexconv_mfma_bf16<TO, 2>), grid, blk, 0, st, (const __bf16*)x, k, b, (TO*)y, G); \
        else                                                                                  \
            hipLaunchKernelGGL((k_hexconv_mfma_bf16<TO, 4>), grid, blk, 0, st, (const __bf16*)x, k, b, (TO*)y, G); \
        return launch_status();
        if (y_dtype == HG_BF16) { HG_CB_LAUNCH(__bf16) }
        HG_CB_LAUNCH(float)
#undef HG_CB_LAUNCH
    }
#define HG_CM_LAUNCH(TI, TO)                                                                  \
    if (nt == 2)                                                                              \
        hipLaunchKernelGGL((k_hexconv_mfma<TI, TO, 2>), grid, blk, 0, st, (const TI*)x, k, b, (TO*)y, G); \
    else                                                                                      \
        hipLaunchKernelGGL((k_hexconv_mfma<TI, TO, 4>), grid, blk, 0, st, (const TI*)x, k, b, (TO*)y, G); \
    return launch_status();
    switch (x_dtype) {
    case HG_BF16:
        if (y_dtype == HG_BF16) { HG_CM_LAUNCH(__bf16, __bf16) }
        if (y_dtype == HG_F32) { HG_CM_LAUNCH(__bf16, float) }
        return HG_EUNSUP;
    case HG_F16:
        if (y_dtype == HG_F16) { HG_CM_LAUNCH(_Float16, _Float16) }
        if (y_dtype == HG_F32) { HG_CM_LAUNCH(_Float16, float) }
        return HG_EUNSUP;
    case HG_F32:
        if (y_dtype == HG_F32) { HG_CM_LAUNCH(float, float) }
        if (y_dtype == HG_BF16) { HG_CM_LAUNCH(float, __bf16) }
        if (y_dtype == HG_F16) { HG_CM_LAUNCH(float, _Float16) }
        return HG_EUNSUP;
    default:
        return HG_EUNSUP;
    }
#undef HG_CM_LAUNCH
}

}  // namespace hg
