// fused.h — the two-column streaming fused kernel (fused.hip), tried first by
// hg_pipeline_r2h_conv_h2r (pipeline.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hg {

// Runs the fused pass if the call is in the kernel's domain (same-size round trip,
// padding 1 with pad value 0, radius 2, C/O/groups in {3/3/1, 3/3/3, 1/1/1}, 16/32-bit
// floats, even widths); returns HG_EUNSUP (nothing launched) otherwise.
int fused_try(const void* x, const float* kernel, const float* bias, void* y, int x_dtype,
              int y_dtype, int64_t batch, int C, int O, int G, int64_t h, int64_t w,
              int64_t h1, int64_t w1, int64_t h2, int64_t w2, int padding, int op,
              double pad_value, hipStream_t st);

// rect -> hex -> rect round trip (no conv) on the same kernel, same-size lattices, even
// widths, planes of (h, w) -> (h1, w1); HG_EUNSUP otherwise.
int fused_rt_try(const void* x, void* y, int x_dtype, int y_dtype, int64_t planes, int64_t h,
                 int64_t w, int64_t h1, int64_t w1, hipStream_t st);

// HexConv2d alone on the same kernel (fused_conv.hip): radius 2, stride 1, padding 1,
// pad value 0, no epilogue, C/O/groups as above, even widths; HG_EUNSUP otherwise.
int fused_conv_try(const void* x, const float* kernel, const float* bias, void* y, int x_dtype,
                   int y_dtype, int64_t batch, int C, int O, int G, int64_t h, int64_t w,
                   int padding, int off, double pad_value, bool epilogue, hipStream_t st);

}  // namespace hg
