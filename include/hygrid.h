/*
 * hygrid.h — C ABI of libhygrid_hip.so, the MI355X (gfx950) hex<->rect lattice
 * resampling and hex-convolution hot path.
 *
 * Contract (all entry points):
 *   - Plain pointers to DEVICE memory, caller-allocated and contiguous
 *     (planar, row-major: (planes, h, w) for the resamplers, (B, C, H, W) for
 *     the convolution).  The library never allocates, frees or retains caller
 *     memory and holds no global mutable state: every call is reentrant.
 *   - Work is enqueued on `stream` (a hipStream_t; NULL = the null stream) with
 *     no host synchronisation inside, so calls may be captured in a hipGraph.
 *   - Return value: HG_OK (0) on success, a negative HG_E* for argument / shape
 *     / dtype errors (nothing is launched), or a positive hipError_t.
 *     hg_strerror() renders either kind.
 *
 * Each entry point cites the reference interface it replaces
 * (paths under Tesla-Albert/Hybrid-Grid-for-Hexagonal-and-Rectangular-Image-Processing).
 * The reference has no native code and no FFI of its own; its Python surface is
 * mirrored on top of this ABI by the HyGrid package.
 */
#ifndef HYGRID_H
#define HYGRID_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HG_ABI_VERSION 1

/* Element types (dtype codes). */
enum hg_dtype {
    HG_U8 = 0, HG_I8 = 1, HG_U16 = 2, HG_I16 = 3, HG_I32 = 4, HG_I64 = 5,
    HG_F16 = 6, HG_BF16 = 7, HG_F32 = 8, HG_F64 = 9
};

/* Interpolation codes.  HG_LINEAR is 'bilinear' for rect->hex
 * (geometry_np.py:359-363) and 'linear' (3-vertex triangle) for hex->rect and
 * hexresize (geometry_np.py:192-197, :672). */
enum hg_interp { HG_NEAREST = 0, HG_LINEAR = 1 };

/* Padding modes of HexConv2d (HexFrames.py:13-21 -> torch.nn.functional.pad). */
enum hg_pad_mode { HG_PAD_CONSTANT = 0, HG_PAD_REFLECT = 1, HG_PAD_REPLICATE = 2,
                   HG_PAD_CIRCULAR = 3 };

/* Activations of the fused HexConv2d epilogue (hg_hexconv2d_epilogue): the act layers
 * HexConvModule builds (HexModules.py:229-236, mmcv ReLU / LeakyReLU / ReLU6 / Sigmoid /
 * Tanh). */
enum hg_act { HG_ACT_NONE = 0, HG_ACT_RELU = 1, HG_ACT_LEAKY_RELU = 2, HG_ACT_RELU6 = 3,
              HG_ACT_SIGMOID = 4, HG_ACT_TANH = 5 };

/* Lattice-map operation codes for hg_lattice_maps. */
enum hg_op { HG_OP_RECT_TO_HEX = 0, HG_OP_HEX_TO_RECT = 1, HG_OP_HEXRESIZE = 2 };

/* Status codes. */
#define HG_OK 0
#define HG_EINVAL (-1)   /* bad argument (null pointer, non-positive size, bad enum) */
#define HG_EDTYPE (-2)   /* unsupported dtype or dtype combination */
#define HG_ESHAPE (-3)   /* input too small for the operator / size overflow */
#define HG_EUNSUP (-4)   /* combination not implemented */
#define HG_EOVERFLOW (-5) /* a kernel's on-chip tile overflowed (k_pyr_level; not expected:
                            * the host bounds every tile's footprint before launching) */

int hg_abi_version(void);
const char* hg_strerror(int status);

/* The kernel-source digest the library was built from (16 hex digits; the Python loader
 * refuses a library whose digest differs from its source tree's). */
const char* hg_build_digest(void);

/* Work decomposition of the streaming fused kernel for mode md (0: hg_pipeline_r2h_conv_h2r,
 * 1: its HexConv2d mode, 2: hg_pipeline_r2h_h2r; 6: mode 0's four-column variant that runs
 * bf16 C = O = 3 calls with widths a multiple of 4): output rows per band, owned columns per
 * window and the window's left halo; HG_EINVAL for any other md.  Host-only; for tests that
 * place inputs at band / window edges. */
int hg_fused_layout(int md, int* band_rows, int* win_own, int* win_halo);

/* rect -> hex lattice resample.
 * Replaces geometry_np.rect_to_hex_resample(rect_image, hex_dsize, interpolation,
 * offset) (HyGrid/geometry_np.py:358-519) for `planes` images at once.
 * src: (planes, h, w) of src_dtype; dst: (planes, h1, w1) of dst_dtype.
 * HG_NEAREST copies the chosen source element (dst_dtype must equal src_dtype);
 * HG_LINEAR needs a floating dst_dtype (F64 reproduces the reference's fp64
 * output bit for bit).  `offset` is dead in the reference (:358), so absent here. */
int hg_rect_to_hex(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t planes,
                   int64_t h, int64_t w, int64_t h1, int64_t w1, int interp, void* stream);

/* hex -> rect lattice resample.
 * Replaces geometry_np.hex_to_rect_resample (HyGrid/geometry_np.py:191-356,
 * 'linear') and geometry_torch.hex_to_square_resample
 * (HyGrid/geometry_torch.py:191-358, 'nearest' rule :335-347). */
int hg_hex_to_rect(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t planes,
                   int64_t h, int64_t w, int64_t h1, int64_t w1, int interp, void* stream);

/* hex -> hex resize.  Replaces geometry_np.hexresize (HyGrid/geometry_np.py:520-681). */
int hg_hexresize(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t planes,
                 int64_t h, int64_t w, int64_t h1, int64_t w1, int interp, void* stream);

/* Gradient of a resample: d src (planes, h, w) of acc_dtype (F32 or F64) for an
 * upstream gradient gy (planes, h1, w1) of acc_dtype.  op: HG_OP_RECT_TO_HEX /
 * HG_OP_HEX_TO_RECT / HG_OP_HEXRESIZE with the forward's interp.  Replaces torch
 * autograd through geometry_torch's gathers and blends (geometry_torch.py:290-358);
 * the transpose of the forward's lattice weights (geometry_np.py:514-517 bilinear,
 * :347-354 triangle, nearest = the chosen neighbour).  dx is overwritten; the
 * scatter uses float atomics (last-bit run-to-run differences). */
int hg_resample_backward(int op, const void* gy, void* dx, int acc_dtype, int64_t planes,
                         int64_t h, int64_t w, int64_t h1, int64_t w1, int interp, void* stream);

/* Which kernel hg_rect_to_hex / hg_hex_to_rect / hg_hexresize would run for this call
 * (nothing is launched): HG_KERNEL_GENERAL (k_resample_lds / k_resample_direct),
 * HG_KERNEL_NEAREST (k_resample_nearest), HG_KERNEL_STREAM (near-identity row streaming,
 * resample_stream.hip), HG_KERNEL_DOWN (~2x downsampling streaming kernels: rect->hex,
 * resample_down.hip; hexresize (pyramid levels), hexresize_down.hip), HG_KERNEL_UP
 * (upsampling triangle lattices, linear and nearest: hex (h/2, w/2) -> rect (h, w), tri_up.hip), or a
 * negative status.  Introspection for tests and tools; the reference has no counterpart.
 * The query has no source pointer, so it answers for a source whose base is 16-B aligned (what
 * torch allocations are); a real call with a 4-B but not 16-B aligned source (a sliced view)
 * takes the hexresize streaming kernel's 4-B-piece layout, whose narrower windows can decline
 * where the query said HG_KERNEL_DOWN: that call then runs the general kernel. */
enum hg_kernel { HG_KERNEL_GENERAL = 0, HG_KERNEL_NEAREST = 1, HG_KERNEL_STREAM = 2,
                 HG_KERNEL_DOWN = 3, HG_KERNEL_UP = 4 };
int hg_resample_kernel(int op, int src_dtype, int dst_dtype, int64_t planes, int64_t h, int64_t w,
                       int64_t h1, int64_t w1, int interp);

/* Integer lattice maps (and fp64 coefficients) of one resample, for parity tests.
 * imaps: int32 [5][h1][w1] = i_n, j_n, up_down_flag, valid bitmask (bit k-1 =
 *        valid_indices_k), nearest argmin — the locals of the reference function
 *        (geometry_np.py:444-476 / :280-315, geometry_torch.py:341).
 * fmaps: float64 [5][h1][w1] = i_f, j_f, alpha, beta, gamma (rect->hex fills the
 *        first two).  Either may be NULL. */
int hg_lattice_maps(int op, int64_t h, int64_t w, int64_t h1, int64_t w1, int32_t* imaps,
                    double* fmaps, void* stream);

/* Output size of HexConv2d (HexFrames.py:127-169): ho = floor((H'-k_h)/s)+1,
 * wo = floor((2W'-s-k_w)/(2s))+1 with H' = h+2p, W' = w+2p, k_h = (2r-2)d+1,
 * k_w = 2d(2r-2)+1.  Host-only; returns HG_ESHAPE when the reference would fail. */
int hg_hexconv2d_out_shape(int64_t h, int64_t w, int radius, int stride, int padding,
                           int dilation, int64_t* ho, int64_t* wo);

/* HexConv2d forward.  Replaces HexFrames.HexConv2d.forward (HexFrames.py:96-169)
 * including pad (:13-21) and heximage_to_type1 (:417-445), which are folded into
 * index arithmetic: no type1 image is materialised.
 * x: (B, C, h, w) of x_dtype; kernel: (O, C/groups, K) with K = 3r^2-3r+1 (the
 * reference parameter `kernel` [O, C/g, 1, K], :74) of w_dtype (F32 or F64);
 * bias: (O,) of w_dtype or NULL; y: (B, O, ho, wo) of y_dtype.
 * Accumulates in w_dtype, as the reference (`input.to(self.kernel.dtype)`, :107). */
int hg_hexconv2d(const void* x, const void* kernel, const void* bias, void* y, int x_dtype,
                 int w_dtype, int y_dtype, int64_t batch, int64_t in_channels,
                 int64_t out_channels, int64_t h, int64_t w, int radius, int stride,
                 int padding, int dilation, int groups, int even_odd_offset, int pad_mode,
                 double pad_value, void* stream);

/* hg_hexconv2d with a fused per-output-channel epilogue: replaces HexConvModule's
 * conv -> norm -> act sequence (HexModules.py:258-268) when the norm is an affine map
 * (BatchNorm in eval mode, folded by the caller into scale = gamma / sqrt(var + eps),
 * shift = beta - mean * scale) or absent:
 *     y[b, o] = act(scale[o] * (conv + bias[o]) + shift[o]),
 * scale / shift: (O,) of w_dtype, either may be NULL (1 / 0); act: hg_act;
 * act_param: the LeakyReLU negative slope.  One pass: the norm and activation never
 * re-read the conv output from HBM. */
int hg_hexconv2d_epilogue(const void* x, const void* kernel, const void* bias, void* y,
                          int x_dtype, int w_dtype, int y_dtype, int64_t batch,
                          int64_t in_channels, int64_t out_channels, int64_t h, int64_t w,
                          int radius, int stride, int padding, int dilation, int groups,
                          int even_odd_offset, int pad_mode, double pad_value,
                          const void* scale, const void* shift, int act, double act_param,
                          void* stream);

/* HexConv2d backward: gradients of hg_hexconv2d for an upstream gradient gy
 * (B, O, ho, wo) of w_dtype.  Replaces the reference's autograd path through
 * HexConv2d.forward (HexFrames.py:96-169: pad -> heximage_to_type1 -> two strided
 * F.conv2d -> interleave); computed as the exact adjoint of the forward index map.
 * dx: (B, C, h, w) of x_dtype (float), or NULL; dkernel: (O, C/groups, K) of
 * w_dtype, or NULL; dbias: (O,) of w_dtype, or NULL.  Outputs are overwritten.
 * x is read only for dkernel, kernel only for dx.  d kernel / d bias are sums
 * over B*ho*wo samples accumulated with float atomics (run-to-run last-bit
 * differences, as torch's own conv weight gradients). */
int hg_hexconv2d_backward(const void* x, const void* kernel, const void* gy, void* dx,
                          void* dkernel, void* dbias, int x_dtype, int w_dtype, int64_t batch,
                          int64_t in_channels, int64_t out_channels, int64_t h, int64_t w,
                          int radius, int stride, int padding, int dilation, int groups,
                          int even_odd_offset, int pad_mode, double pad_value, void* stream);

/* Hex raster storage formats (pure memory permutes; any element size 1/2/4/8).
 * hg_hex_to_type1: (planes, h, w) offset-row hex image -> (planes, h*row_repeat, 2w+1)
 * "type1" double-width raster T[y][2k+L] = T[y][2k+1+L] = x[y][k], L = (y%2+off)%2,
 * zeros elsewhere; row_repeat 1 replaces HexFrames.heximage_to_type1
 * (HexFrames.py:417-445) / HEXIMAGE.GenerateType1Image (HexImage.py:139-153),
 * row_repeat 2 the type2 raster (HexFrames.py:446-449, HexImage.py:154-170).
 * hg_strided_copy2d: dst[p][i][j] = src[p][row_start + i*row_step][col_start + j*col_step]
 * (contiguous decode of type1 / type2 rasters, HexImage.py:108-111, HexFrames.py:450-458). */
int hg_hex_to_type1(const void* src, void* dst, int elem_size, int64_t planes, int64_t h,
                    int64_t w, int even_odd_offset, int row_repeat, void* stream);
int hg_strided_copy2d(const void* src, void* dst, int elem_size, int64_t planes, int64_t H,
                      int64_t W, int64_t row_start, int64_t row_step, int64_t col_start,
                      int64_t col_step, int64_t h_out, int64_t w_out, void* stream);

/* Affine transform of a hex raster onto a new hex lattice: replaces the per-sample work
 * of image_geometric_transformation (geometry_np.py:6-189, geometry_torch.py:7-189).
 * xs (h1) / ys (w1): DEVICE fp64 output axes, np.arange(h1_inf, h1_sup + 1, 1) and
 * np.arange(w1_inf, w1_sup + 0.5, 1) of the transformed corners (:56-87); odd rows are
 * shifted by +0.5 in the kernel (:87).  hinv: HOST fp64 3x3 row-major inv(H) (:97-102;
 * its third row is unused, as in the reference).  interp HG_LINEAR: 3-vertex triangle
 * blend in fp64, dst F64/F32/F16/BF16 (:175-184); HG_NEAREST: first-minimum vertex,
 * dst_dtype == src_dtype (geometry_torch.py:165-173; the NumPy twin raises there).
 * hg_hex_homography_maps: int32 [5][h1][w1] maps as hg_lattice_maps, fp64 [7][h1][w1]
 * = i_f, j_f, alpha, beta, gamma, x_, y_ (parity tests). */
int hg_hex_homography(const void* src, void* dst, int src_dtype, int dst_dtype, int64_t planes,
                      int64_t h, int64_t w, int64_t h1, int64_t w1, const double* xs,
                      const double* ys, const double* hinv, int interp, void* stream);
/* Hex pooling: replaces HexPool2d / HexAdaptivePool2d / HexGlobalPool2d
 * (HexFrames.py:255-410) with the NaN-aware reductions max_pooling / min_pooling /
 * average_pooling (:461-479); method 0 max, 1 min, 2 average.  x: (planes, h, w) of
 * dtype F16/BF16/F32/F64, y: (planes, hn, wn) of the same dtype.  Window (i, j) covers
 * rows i*sh + [0, kh) and cols ((i % 2) * sw) / 2 + j*sw + [0, kw) (:314-319) of the
 * frame pad(x, pad, pad_mode, pad_value) extended by ext_h rows / ext_w cols of
 * ext_value (ceil mode, :295-300).  Windows outside the frame -> HG_ESHAPE (the
 * reference raises IndexError).  Backward: dx (planes, h, w) in grad_dtype F32/F64
 * (overwritten) from gy (planes, hn, wn) in grad_dtype, the reference's autograd. */
int hg_hex_pool2d(const void* x, void* y, int dtype, int method, int64_t planes, int64_t h,
                  int64_t w, int pad, int pad_mode, double pad_value, int64_t ext_h,
                  int64_t ext_w, double ext_value, int kh, int kw, int sh, int sw, int64_t hn,
                  int64_t wn, void* stream);
int hg_hex_pool2d_backward(const void* x, const void* gy, void* dx, int dtype, int grad_dtype,
                           int method, int64_t planes, int64_t h, int64_t w, int pad,
                           int pad_mode, double pad_value, int64_t ext_h, int64_t ext_w,
                           double ext_value, int kh, int kw, int sh, int sw, int64_t hn,
                           int64_t wn, void* stream);
int hg_hex_homography_maps(int64_t h, int64_t w, int64_t h1, int64_t w1, const double* xs,
                           const double* ys, const double* hinv, int32_t* imaps, double* fmaps,
                           void* stream);

/* Fused rect -> hex -> HexConv2d -> hex -> rect pass over a batch.
 * Replaces the chain rect_to_hex_resample(x, (h1,w1), 'bilinear')
 * (geometry_np.py:358-519) -> HexConv2d(C, O, even_odd_offset, 2, stride=1,
 * padding, dilation=1, groups, padding_mode='constant', padding_value)
 * (HexFrames.py:22-169) -> hex_to_rect_resample(., (h2,w2), 'linear')
 * (geometry_np.py:191-356), as a user script runs it (SURVEY.md §3 B+C).
 * x: (B, C, h, w); kernel: (O, C/groups, 7) float32; bias: (O,) float32 or NULL;
 * y: (B, O, h2, w2).  Intermediates stay on chip in fp32 (one read of x, one
 * write of y).  C, O in {1, 3}; x_dtype in {U8, F16, BF16, F32}, y_dtype in
 * {F16 (f16 in only), BF16, F32}.  Returns HG_EUNSUP when the geometry is not
 * near-identity (then run the three operators instead). */
int hg_pipeline_r2h_conv_h2r(const void* x, const float* kernel, const float* bias, void* y,
                             int x_dtype, int y_dtype, int64_t batch, int64_t channels,
                             int64_t out_channels, int64_t h, int64_t w, int64_t h1, int64_t w1,
                             int64_t h2, int64_t w2, int padding, int groups,
                             int even_odd_offset, double pad_value, void* stream);

/* rect -> hex -> rect round trip (BASELINE config 2) in one pass, no conv: replaces
 * hex_to_rect_resample(rect_to_hex_resample(x, (h1, w1), 'bilinear'), (h1, w1), 'linear')
 * (HyGrid/geometry_np.py:358-519, then :191-356).  x: (planes, h, w); y: (planes, h1, w1);
 * the hex image stays on chip in fp32.  x_dtype in {F16, BF16, F32}, y_dtype in {x_dtype,
 * F32}.  Returns HG_EUNSUP unless the lattice is the same-size near-identity one and the
 * widths are even (then run hg_rect_to_hex + hg_hex_to_rect). */
int hg_pipeline_r2h_h2r(const void* x, void* y, int x_dtype, int y_dtype, int64_t planes,
                        int64_t h, int64_t w, int64_t h1, int64_t w1, void* stream);

/* One level of a hex Gaussian pyramid (BASELINE config 5) in one pass:
 *   from_rect = 0:  y = hexresize(HexConv2d_dw(x), (h1, w1))
 *   from_rect = 1:  y = hexresize(HexConv2d_dw(rect_to_hex(x, (h, w), 'bilinear')), (h1, w1))
 * Replaces the chain rect_to_hex_resample (geometry_np.py:358-519) ->
 * HexConv2d(C, C, even_odd_offset, 2, stride=1, padding=1, dilation=1, groups=C,
 * padding_mode='constant', padding_value=0) (HexFrames.py:22-169) -> hexresize(.,
 * (h1, w1), 'linear') (geometry_np.py:520-681).  x: (B, C, h, w); taps: (C, 7) float32
 * (the depthwise kernel, HexConv2d.kernel (C, 1, 1, 7)); bias: (C,) float32 or NULL;
 * y: (B, C, h1, w1).  Intermediates stay on chip in fp32.  x_dtype in {F16, BF16, F32},
 * y_dtype in {x_dtype, F32} (F32 in: also F16, BF16).  Returns HG_EUNSUP when the
 * resize footprint does not fit the kernel's tile (e.g. > 2x downsampling) or the r2h
 * lattice is not near-identity (then run the operators instead). */
int hg_hex_pyramid_level(const void* x, void* y, int x_dtype, int y_dtype, int64_t batch,
                         int64_t channels, int64_t h, int64_t w, int64_t h1, int64_t w1,
                         const float* taps, const float* bias, int even_odd_offset,
                         int from_rect, void* stream);
/* Which kernel hg_hex_pyramid_level would run for this call (nothing is launched):
 * HG_PYR_FUSED (k_fused MD 3 / 4, pyramid_fused.hip), HG_PYR_FUSED_SHORT (MD 5: the same on
 * short bands, for levels too small to fill the chip), HG_PYR_STREAM (k_pyr_stream), HG_PYR_LDS
 * (k_pyr_level, the LDS-tiled fallback), or a negative status.  The environment variable
 * HYGRID_PYR_KERNEL = "fused" | "stream" | "lds" restricts both calls to that kernel (the
 * call returns HG_EUNSUP when it cannot run it); for tests and A/B measurements.
 * The LDS fallback synchronises `stream` once to report HG_EOVERFLOW; the other kernels
 * never synchronise. */
enum hg_pyr_kernel { HG_PYR_FUSED = 0, HG_PYR_FUSED_SHORT = 1, HG_PYR_STREAM = 2, HG_PYR_LDS = 3 };
int hg_hex_pyramid_level_kernel(int x_dtype, int y_dtype, int64_t batch, int64_t channels,
                                int64_t h, int64_t w, int64_t h1, int64_t w1, int even_odd_offset,
                                int from_rect);

/* Several pyramid levels in ONE launch (round 6): ys[l] = level l of the chain
 *   ys[0] = hg_hex_pyramid_level(x, from_rect = 1, (h/2, w/2)),
 *   ys[l] = hg_hex_pyramid_level(ys[l-1], from_rect = 0, (h_l/2, w_l/2))   (same taps / bias)
 * — the chain the reference's user code builds from rect_to_hex_resample (geometry_np.py:358-519),
 * HexConv2d (HexFrames.py:96-169) and hexresize (geometry_np.py:520-681) — bit-identical to those
 * per-level calls, with the levels' workgroups in one grid: a band of level l starts when the
 * bands of level l - 1 that wrote its input rows are complete (per-band counters in `workspace`),
 * so the launches' ramps and tails overlap the neighbouring level's work.  x: (B, C, h, w) rect;
 * ys[l]: (B, C, h >> (l+1), w >> (l+1)), all of `dtype` (F16 or BF16).  workspace: >=
 * hg_hex_pyramid_chain_workspace(levels, batch, h) bytes, 16-byte aligned; the call zeroes it
 * on `stream` before the launch (the ticket, fault and per-band counter words), and after the
 * launch int [1] is a fault word, 1 if a workgroup waited longer than ~1 s for its input
 * (output then invalid; not expected: the tests assert 0).  One workspace per call in flight.
 * Returns HG_EUNSUP outside the
 * chain's domain (levels 2-3, C = 3, 16-bit, level 0 on the fused kernel's MD 3 and the later
 * levels on its short bands, i.e. the hg_hex_pyramid_level_kernel answers HG_PYR_FUSED then
 * HG_PYR_FUSED_SHORT): then call hg_hex_pyramid_level per level.  Measured 2.7x slower than
 * the per-level launches on config 5 (the hand-off's release / acquire / ticket costs exceed
 * the launch edges it hides): HyGrid's hex_pyramid uses it only with
 * HYGRID_PYR_CHAIN=1. */
int64_t hg_hex_pyramid_chain_workspace(int levels, int64_t batch, int64_t h);
int hg_hex_pyramid_chain(const void* x, void* const* ys, int levels, int dtype, int64_t batch,
                         int64_t channels, int64_t h, int64_t w, const float* taps,
                         const float* bias, int even_odd_offset, void* workspace,
                         int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HYGRID_H */
