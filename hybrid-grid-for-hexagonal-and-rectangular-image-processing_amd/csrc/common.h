// common.h — dtype plumbing and launch helpers shared by the HyGrid gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hygrid.h"

namespace hg {

// Element types of the C-ABI dtype enum (include/hygrid.h).  bf16/f16 are the
// compiler's native storage types: hipcc lowers (__bf16)f to v_cvt_pk_bf16_f32
// (round-to-nearest-even, NaN kept NaN) and (float)b to a 16-bit shift.
template <int DT> struct dtype_of;
template <> struct dtype_of<HG_U8>   { using T = uint8_t; };
template <> struct dtype_of<HG_I8>   { using T = int8_t; };
template <> struct dtype_of<HG_U16>  { using T = uint16_t; };
template <> struct dtype_of<HG_I16>  { using T = int16_t; };
template <> struct dtype_of<HG_I32>  { using T = int32_t; };
template <> struct dtype_of<HG_I64>  { using T = int64_t; };
template <> struct dtype_of<HG_F16>  { using T = _Float16; };
template <> struct dtype_of<HG_BF16> { using T = __bf16; };
template <> struct dtype_of<HG_F32>  { using T = float; };
template <> struct dtype_of<HG_F64>  { using T = double; };

inline int dtype_size(int dt) {
    switch (dt) {
    case HG_U8: case HG_I8: return 1;
    case HG_U16: case HG_I16: case HG_F16: case HG_BF16: return 2;
    case HG_I32: case HG_F32: return 4;
    case HG_I64: case HG_F64: return 8;
    default: return 0;
    }
}
inline bool dtype_is_float(int dt) {
    return dt == HG_F16 || dt == HG_BF16 || dt == HG_F32 || dt == HG_F64;
}

template <typename A, typename T> __device__ __forceinline__ A to_acc(T v) { return (A)v; }
template <typename T, typename A> __device__ __forceinline__ T from_acc(A v) { return (T)v; }

// Map (in dtype, out dtype) of a floating-point kernel onto its template.
// Integer inputs are exact in f32 up to 2^24, so the accumulator is f64 only when
// the caller asks for f64 output or feeds f64/i32/i64 data.
inline bool acc_is_double(int in_dt, int out_dt) {
    return out_dt == HG_F64 || in_dt == HG_F64 || in_dt == HG_I32 || in_dt == HG_I64;
}

inline int hip_status(hipError_t e) { return e == hipSuccess ? HG_OK : (int)e; }

inline int launch_status() { return hip_status(hipGetLastError()); }

// The library's A/B / test switches (HYGRID_*, read on every call): true iff the variable is
// set to exactly `value`.
inline bool env_is(const char* name, const char* value) {
    const char* e = getenv(name);
    return e && !strcmp(e, value);
}

// XCD-aware block order.  Blocks are dealt to the 8 XCDs round-robin (bid % 8 labels
// the blocks that share an XCD and its private L2); this bijection hands each XCD a
// contiguous run of logical blocks, so neighbouring windows / tiles, whose halos
// share 128-B lines, are fetched into the same L2 instead of into two
// (cdna_hip_programming.md T1, bijective form for nwg % 8 != 0).  Speed only: any
// placement is correct.
// Every buffer store wider than 8 bytes goes through this: the row offset is added into the
// VGPR offset and soffset is 0.  With an SGPR soffset the compiler's hazard recognizer puts no
// wait state between a > 8-byte MUBUF store and a VALU write of its data registers, and the
// MI355X then stored the overwritten value (k_tri_up, round 5; tests/test_store_hazard.py scans
// the built library for the pattern).  A voff of 0x80000000 (a dropped store) stays out of
// range: every soff here is a byte offset inside a buffer of < 2^31 bytes.
typedef unsigned hg_u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void hg_store_b128(hg_u4v v, __amdgpu_buffer_rsrc_t rs, unsigned voff,
                                              unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff + soff, 0, 0);
}

__device__ __forceinline__ unsigned xcd_swizzle(unsigned bid, unsigned nwg) {
    const unsigned q = nwg >> 3, r = nwg & 7u, x = bid & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
// The same for a 2-D grid in dispatch (x-fastest) order: returns the logical (x, y).
__device__ __forceinline__ void xcd_swizzle2(unsigned* bx, unsigned* by) {
    const unsigned s = xcd_swizzle(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    *bx = s % gridDim.x;
    *by = s / gridDim.x;
}

// Fused conv epilogue (hg_hexconv2d_epilogue): v -> act(scale[o] * v + shift[o]).
struct Epilogue {
    const void* scale;   // (O,) accumulator type, or null (1)
    const void* shift;   // (O,) accumulator type, or null (0)
    int act;             // hg_act
    double slope;        // LeakyReLU negative slope
    int on;              // any of the above present
};

template <typename A>
__device__ __forceinline__ A epi_apply(A v, int o, const Epilogue& e) {
    if (e.scale) v = v * static_cast<const A*>(e.scale)[o];
    if (e.shift) v = v + static_cast<const A*>(e.shift)[o];
    switch (e.act) {
    case HG_ACT_RELU: return v > (A)0 ? v : (A)0;
    case HG_ACT_LEAKY_RELU: return v > (A)0 ? v : v * (A)e.slope;
    case HG_ACT_RELU6: return v > (A)0 ? (v < (A)6 ? v : (A)6) : (A)0;
    case HG_ACT_SIGMOID: return (A)1 / ((A)1 + exp(-v));
    case HG_ACT_TANH: return tanh(v);
    default: return v;
    }
}

}  // namespace hg

// Instantiate `FN<Tin, Tout>(args...)` for every supported (in, out) dtype pair.
// The body returns HG_EDTYPE for pairs it does not support.
#define HG_DISPATCH_IN(dt, TIN, ...)                                         \
    switch (dt) {                                                            \
    case HG_U8:   { using TIN = uint8_t;  __VA_ARGS__; } break;              \
    case HG_I8:   { using TIN = int8_t;   __VA_ARGS__; } break;              \
    case HG_U16:  { using TIN = uint16_t; __VA_ARGS__; } break;              \
    case HG_I16:  { using TIN = int16_t;  __VA_ARGS__; } break;              \
    case HG_I32:  { using TIN = int32_t;  __VA_ARGS__; } break;              \
    case HG_F16:  { using TIN = _Float16; __VA_ARGS__; } break;              \
    case HG_BF16: { using TIN = __bf16;   __VA_ARGS__; } break;              \
    case HG_F32:  { using TIN = float;    __VA_ARGS__; } break;              \
    case HG_F64:  { using TIN = double;   __VA_ARGS__; } break;              \
    default: return HG_EDTYPE;                                               \
    }

#define HG_DISPATCH_FLOAT_OUT(dt, TOUT, ...)                                 \
    switch (dt) {                                                            \
    case HG_F16:  { using TOUT = _Float16; __VA_ARGS__; } break;             \
    case HG_BF16: { using TOUT = __bf16;   __VA_ARGS__; } break;             \
    case HG_F32:  { using TOUT = float;    __VA_ARGS__; } break;             \
    case HG_F64:  { using TOUT = double;   __VA_ARGS__; } break;             \
    default: return HG_EDTYPE;                                               \
    }
