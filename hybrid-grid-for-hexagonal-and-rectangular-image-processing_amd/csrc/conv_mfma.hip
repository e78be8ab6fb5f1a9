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

struct MfmaGeom {
    int64_t B;
    int C, O, h, w, ho, wo, p, pad_mode;
    int mink;                   // smallest tap column offset over both parities
    int dy[7], dk[2][7];        // tap rows / columns (padded frame, relative to mink)
    int ntq, ntr, nto;          // tiles along columns / rows / output channels
    float pad_value;
    Epilogue epi;
};

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

    cm_f4 acc[NOT][4];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = o0 + ot * 16 + lk * 4 + v;
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
                        acc[ot][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[ot], bf[qt],
                                                                           acc[ot][qt], 0, 0, 0);
            }
        }
        __syncthreads();
    }

    // ---- epilogue: bias was the accumulator's start; BN / activation; store -------------
    if (r >= G.ho) return;
    Tout* yb = y + b * (int64_t)G.O * G.ho * G.wo;
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
            wsb[((0 * 2 + kb) * CM_O + o) * 4 + g] = pk(h);
            wsb[((1 * 2 + kb) * CM_O + o) * 4 + g] = pk(m);
            wsb[((2 * 2 + kb) * CM_O + o) * 4 + g] = pk(l);
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
                    const cm_b8 af = __builtin_bit_cast(cm_b8, wsb[((pt * 2 + kb) * CM_O + ot * 16 + li) * 4 + lg]);
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

// Runs the MFMA kernel when it covers the call and pays (dense radius-2, stride-1,
// dilation-1 conv with C >= 8 and O >= 16, f32 weights); HG_EUNSUP otherwise.
int conv_mfma_try(const void* x, const float* k, const float* b, void* y, int x_dtype,
                  int y_dtype, int64_t B, int64_t C, int64_t O, int64_t h, int64_t w, int radius,
                  int stride, int padding, int dilation, int groups, int off, int pad_mode,
                  double pad_value, const Epilogue& epi, hipStream_t st) {
    if (env_is("HYGRID_CONV_MFMA", "0")) return HG_EUNSUP;   // A/B switch: generic kernels
    if (radius != 2 || stride != 1 || dilation != 1 || groups != 1) return HG_EUNSUP;
    if (C < 8 || O < 16 || padding < 0 || padding > 2) return HG_EUNSUP;
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
    const int nt = G.O <= 32 ? 2 : 4;                  // output-channel tiles per workgroup
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
