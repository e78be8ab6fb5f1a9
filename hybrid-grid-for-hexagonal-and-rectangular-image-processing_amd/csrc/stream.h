// stream.h — row-streaming resample kernels for near-identity lattices
// (resample_stream.hip), tried first by hg_rect_to_hex / hg_hex_to_rect (resample.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hg {

// Runs the streaming kernel if the call is in its domain (r2h with a near-identity
// lattice, h2r at the same size; 16/32-bit float in and out; widths a multiple of 4);
// returns HG_EUNSUP (nothing launched) otherwise.  Bit-identical to the general kernels.
// dry: only the domain check (HG_OK = the kernel would run), nothing launched.
int stream_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
               int64_t w, int64_t h1, int64_t w1, hipStream_t st, bool dry = false);

// ~2x downsampling rect->hex (ConvertToHexagon's (h//2, w//2) 'nearest' on 8/16-bit data, the
// demo's bilinear on bf16/f16; resample_down.hip); HG_EUNSUP (nothing launched) otherwise.
// hexresize_down.hip: triangle-blend resamples (op HG_OP_HEXRESIZE / HG_OP_HEX_TO_RECT,
// linear, 16-bit in) whose vertices for a run of output columns fit a 128-column input
// window (~2x hexresize: the pyramid levels; hex (h/2, w/2) -> rect (h, w)); HG_EUNSUP otherwise
int tristream_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
                  int64_t w, int64_t h1, int64_t w1, hipStream_t st, bool dry);
// tri_up.hip: upsampling triangle resamples (op HG_OP_HEX_TO_RECT / HG_OP_HEXRESIZE whose output
// steps are <= one input sample: the inverse of ConvertToHexagon's lattice), 'linear' on 16/32-bit
// floats with fp32 accumulation and 'nearest' on 8/16/32-bit elements; HG_EUNSUP otherwise
int triup_try(int op, const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h,
              int64_t w, int64_t h1, int64_t w1, int interp, hipStream_t st, bool dry);
int down_try(const void* src, void* dst, int sdt, int ddt, int64_t planes, int64_t h, int64_t w,
             int64_t h1, int64_t w1, int interp, hipStream_t st, bool dry = false);

}  // namespace hg
