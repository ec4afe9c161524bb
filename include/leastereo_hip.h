/*
 * leastereo_hip.h — C ABI of libleastereo_hip.so, the MI355X (gfx950) kernels
 * behind LEAStereo's inference hot path.
 *
 * The reference (devmentality/LEAStereo) is pure PyTorch and has no FFI; each
 * entry point below replaces the aten op sequence at the cited reference line,
 * and is what a ctypes/cffi binding of that path binds.
 *
 * Conventions
 *   - All tensors are caller-owned device buffers, NCDHW (or NCHW) contiguous
 *     in W, H, D order; channel stride is always D*H*W.  A per-batch stride
 *     (in elements) lets an operand be a channel slice of a larger tensor, which
 *     is how torch.cat (skip_model_3d.py:74,150,155) becomes free.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  No call
 *     allocates, synchronises or touches the host after argument checks, so every
 *     call is hipGraph-capturable.
 *   - Return 0 on success; LEA_E_INVALID / LEA_E_UNSUPPORTED on bad arguments
 *     (nothing launched); otherwise a hipError_t from the launch.
 *     lea_last_error() describes the last failure on the calling thread.
 *   - dtype: LEA_F32 (the reference's arithmetic) for the entries below that take
 *     one; the bf16 path (configs 3/4) has its own *_bf16 entries at the end.
 */
#ifndef LEASTEREO_HIP_H
#define LEASTEREO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LEA_ABI_VERSION 13

#define LEA_F32 0
#define LEA_BF16 1

#define LEA_OK 0
#define LEA_E_INVALID 1001
#define LEA_E_UNSUPPORTED 1002

/* conv epilogue flags */
#define LEA_RELU 1u     /* ReLU after the BN affine (operations_3d.py:45-46)          */
#define LEA_RESIDUAL 2u /* y = act(...) + residual: the cell's `sum(new_states)`
                           (skip_model_3d.py:69); residual may alias y               */
#define LEA_PAIR_SUM 4u /* two ConvBRs summed, a cell step of two conv terms
                           (skip_model_3d.py:57-69): y = act(BN_a(conv_a(x))) +
                           act(BN_b(conv_b(x2))) -- input channels [0, cin - cin2) are
                           conv_a's, [cin - cin2, cin) conv_b's (the weights packed as one
                           conv over the concatenation), scale/shift hold 2 * cout values
                           (a's, then b's); exclusive with LEA_RESIDUAL.  Where an engine
                           supports it (lea_conv3d_bnrelu_wino: cout <= 32, W % 4 == 0;
                           lea_conv3d_bnrelu_bf16: the D-streaming 3x3x3 layers), else
                           LEA_E_UNSUPPORTED                                           */

int lea_abi_version(void);
const char* lea_last_error(void);

/* Cost volume.  Replaces retrain/LEAStereo.py:34-48 (zero-init + 2*D3 strided copies).
 *   cost[b, c,   i, h, w] = left [b, c, h, w]     for w >= i
 *   cost[b, C+c, i, h, w] = right[b, c, h, w - i] for w >= i,   0 for w < i
 * left/right: [B, C, H, W]; cost: [B, 2C, D3, H, W].  D3 = int(maxdisp / 3). */
int lea_build_cost_volume(const void* left, const void* right, void* cost,
                          int B, int C, int H, int W, int D3, int dtype, void* stream);

/* Packed-weight size (in floats) for a ConvBR of the given shape; k in {1, 3}. */
size_t lea_conv3d_packed_floats(int cout, int cin, int k);

/* Re-lay an OIDHW fp32 weight ([cout, cin, k, k, k], device) into the kernel's
 * packed layout (device).  Done once per load_state_dict. */
int lea_conv3d_pack_weights(const float* w, float* packed, int cout, int cin, int k,
                            void* stream);

/* ConvBR3d.  Replaces models/operations_3d.py:41-47 (Conv3d no bias, stride 1,
 * pad k/2 -> BatchNorm3d eval -> ReLU) with BN folded on the host into
 *   scale = gamma / sqrt(var + eps),  shift = beta - mean * scale
 * (both NULL = bn=False).  Input channels [0, cin-cin2) come from x and
 * [cin-cin2, cin) from x2 (cin2 = 0: single source), i.e. the conv reads
 * torch.cat((x, x2), 1) without it existing (skip_model_3d.py:150,155).
 * x: [B, cin-cin2, D, H, W], x2: [B, cin2, D, H, W], y/residual: [B, cout, D, H, W],
 * each at its own batch stride. */
int lea_conv3d_bnrelu(const void* x, int64_t x_bstride,
                      const void* x2, int64_t x2_bstride, int cin2,
                      const float* w_packed, const float* scale, const float* shift,
                      const void* residual, int64_t r_bstride,
                      void* y, int64_t y_bstride,
                      int B, int cin, int cout, int D, int H, int W, int k,
                      unsigned flags, int dtype, void* stream);

/* ConvBR3d of a trilinearly resampled input: conv(interp(x, [D, H, W],
 * align_corners=True)) with the interpolation done while staging, so the
 * resampled volume never reaches HBM.  Replaces the F.interpolate + ConvBR pairs
 * of Cell.forward (skip_model_3d.py:44-53) and the head's Upsample + last_3
 * (:162-173).  x: [B, cin, Di, Hi, Wi]; y/residual: [B, cout, D, H, W]. */
int lea_conv3d_bnrelu_resampled(const void* x, int64_t x_bstride, int Di, int Hi, int Wi,
                                const float* w_packed, const float* scale, const float* shift,
                                const void* residual, int64_t r_bstride,
                                void* y, int64_t y_bstride,
                                int B, int cin, int cout, int D, int H, int W, int k,
                                unsigned flags, int dtype, void* stream);

/* Matching-net stem0 on the cost volume without materialising it: the ConvBR3d
 * (3x3x3) of cost = [B, 2C, D3, H, W] as built by lea_build_cost_volume
 * (retrain/LEAStereo.py:34-48 then skip_model_3d.py:141), reading the feature maps
 * left/right [B, C, H, W] (batch stride f_bstride) directly.  Bit-identical to
 * lea_build_cost_volume + lea_conv3d_bnrelu; saves the 2*4*B*C*D3*H*W-byte volume's
 * write and read.  C must be a multiple of 4.  y: [B, cout, D3, H, W]. */
int lea_conv3d_bnrelu_costvolume(const void* left, const void* right, int64_t f_bstride,
                                 const float* w_packed, const float* scale, const float* shift,
                                 void* y, int64_t y_bstride, int B, int C, int cout, int D3,
                                 int H, int W, unsigned flags, int dtype, void* stream);
const char* lea_conv3d_costvolume_kernel_name(int B, int cout, int D3, int H, int W);

/* Name of the kernel instantiation a conv of this output shape launches
 * (matches the demangled name rocprofv3 reports); NULL if unsupported. */
const char* lea_conv3d_kernel_name(int B, int cout, int D, int H, int W, int k, int resampled);

/* ---- 2D feature net (retrain/new_model_2d.py; models/operations_2d.py:31-47) ----
 * 1x1 Conv2d and bilinear (align_corners) resizes of the feature net use the 3D
 * entry points with D = Di = 1 (a bilinear resize is the trilinear one on a
 * single plane, bit for bit).  The 3x3 convs have their own packing and entry. */

/* Packed-weight size (floats) / packing of a Conv2d 3x3 weight [cout, cin, 3, 3]. */
size_t lea_conv2d_packed_floats(int cout, int cin);
int lea_conv2d_pack_weights(const float* w, float* packed, int cout, int cin, void* stream);

/* ConvBR2d 3x3, stride 1, pad 1 (folded BN as in lea_conv3d_bnrelu, LEA_RELU,
 * LEA_RESIDUAL -- the 2D cell's sum, including its skip_connect terms).
 * x: [B, cin, H, W], y/residual: [B, cout, H, W], each at its own batch stride. */
int lea_conv2d_bnrelu(const void* x, int64_t x_bstride, const float* w_packed,
                      const float* scale, const float* shift, const void* residual,
                      int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin, int cout,
                      int H, int W, unsigned flags, int dtype, void* stream);

/* Kernel instantiation lea_conv2d_bnrelu launches for this shape. */
const char* lea_conv2d_kernel_name(int B, int cout, int H, int W);

/* Two ConvBR2d 3x3 s1 p1 of the same input in one launch (a feature-net cell's two ops
 * on s0, retrain/new_model_2d.py:41-75 -- the reference runs them as two convs): weights
 * and folded BN of both stacked along cout (w_packed: lea_conv2d_pack_weights of the
 * [cout, cin, 3, 3] stack), couts [0, c1) written to y with the residual (flags as for
 * lea_conv2d_bnrelu), couts [c1, cout) to y2 without it.  cin <= 16, cout <= 32 and
 * c1 % 8 == 0 (the few-channel tile; LEA_E_UNSUPPORTED beyond it); fp32. */
int lea_conv2d_bnrelu_pair(const void* x, int64_t x_bstride, const float* w_packed,
                           const float* scale, const float* shift, const void* residual,
                           int64_t r_bstride, void* y, int64_t y_bstride, void* y2,
                           int64_t y2_bstride, int B, int cin, int cout, int c1, int H, int W,
                           unsigned flags, void* stream);

/* Feature-net stem1: Conv2d 3x3, stride 3, pad 1 -> BN -> ReLU (new_model_2d.py:94).
 * w: the raw [cout, cin, 3, 3] weight (no packing).  x: [B, cin, Hi, Wi];
 * y: [B, cout, (Hi-1)/3+1, (Wi-1)/3+1]. */
int lea_conv2d_s3_bnrelu(const void* x, int64_t x_bstride, const float* w, const float* scale,
                         const float* shift, void* y, int64_t y_bstride, int B, int cin, int cout,
                         int Hi, int Wi, unsigned flags, int dtype, void* stream);

/* Feature-net stems 0 + 1 fused (retrain/new_model_2d.py:93-94): ConvBR2d 3x3 s1 p1
 * (cin -> c0) then ConvBR2d 3x3 s3 p1 (c0 -> c1), both with folded BN and ReLU, without
 * writing stem0's full-resolution output (stride 3 tiles it: each stem0 pixel feeds one
 * stem1 pixel).  w0: [c0, cin, 3, 3], w1: [c1, c0, 3, 3] raw f32.  x: [B, cin, Hi, Wi] f32;
 * y: [B, c1, Ho, Wo] f32 (dtype LEA_F32) or c8 [B, c1/8, 1, Ho, Wo, 8] bf16 (LEA_BF16),
 * Ho = (Hi - 1) / 3 + 1.  Instantiated for 3 -> 16 -> 32 (the searched feature net).
 * Image b is read at x + b * x_bstride (elements, any sign): two separately allocated
 * images (the left / right pair) run as one B = 2 launch with x_bstride = right - left. */
int lea_feature_stem_bnrelu(const float* x, int64_t x_bstride, const float* w0, const float* scale0,
                            const float* shift0, const float* w1, const float* scale1,
                            const float* shift1, void* y, int64_t y_bstride, int B, int cin, int c0,
                            int c1, int Hi, int Wi, int dtype, void* stream);


/* Trilinear resample.  Replaces F.interpolate(mode='trilinear') at
 * skip_model_3d.py:48,50 and nn.Upsample at :162-164 (align_corners=1), with
 * PyTorch's source-index rule, then an optional epilogue
 *   y = act(scale[c] * interp(x) + shift[c])      (scale/shift NULL: identity)
 * with act = ReLU under LEA_RELU.  With the epilogue it completes an up-sampling
 * ConvBR1x1 whose conv ran at the input resolution (the conv and the
 * interpolation commute). */
int lea_resample3d_trilinear(const void* x, int64_t x_bstride, void* y, int64_t y_bstride,
                             int B, int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                             int align_corners, const float* scale, const float* shift,
                             unsigned flags, int dtype, void* stream);

/* Head conv of an upsampled tensor, from per-tap partial sums.  Replaces
 * last_3(Upsample(y)) (skip_model_3d.py:161-173, 3x3x3 conv after a trilinear
 * align_corners=True resize): with q[b][co*27 + tap] = sum_ci W[co][ci][tap]*y[ci]
 * computed at the low resolution (lea_conv3d_bnrelu, k=1, 27*cout outputs),
 *   y_out[b][co](v) = act(scale[co] * sum_tap interp(q[b][co*27+tap])(v + off(tap)) + shift[co])
 * over the [Do, Ho, Wo] output, taps outside it contributing 0 (zero padding).
 * q: [B, 27*cout, Di, Hi, Wi]; y_out: [B, cout, Do, Ho, Wo].  workspace: device
 * scratch of lea_tapsum_workspace_bytes(B, cout, Hi, Wi, Do) bytes, 16-B aligned
 * (the d-interpolated partial sums; the caller owns it, as every buffer here). */
size_t lea_tapsum_workspace_bytes(int B, int cout, int Hi, int Wi, int Do);
int lea_tapsum_upsample(const void* q, int64_t q_bstride, void* y, int64_t y_bstride,
                        int B, int cout, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                        const float* scale, const float* shift, unsigned flags,
                        void* workspace, int dtype, void* stream);

/* Disparity regression.  Replaces models/build_model_2d.py:52-57 + :33-42:
 *   U = trilinear(cost, [maxdisp, 3*H3, 3*W3], align_corners=False)
 *   disp[b, h, w] = sum_d d * softmax(-U, dim=d)
 * fused, U never materialised.  cost: [B, 1, D3, H3, W3]; disp: [B, 3H3, 3W3] fp32.
 * dtype LEA_BF16 (the bf16 path; cost still f32) uses the hardware exp. */
int lea_disparity_regression(const void* cost, float* disp, int B, int D3, int H3, int W3,
                             int maxdisp, int dtype, void* stream);

/* ---- bf16 path (BASELINE configs 3 and 4) ----
 * Activations are bf16 in the "c8" layout: NCDHW with channels blocked by 8
 * innermost, x[b][c/8][d][h][w][c%8] (one voxel's 8 channels = one 16-byte word;
 * channel counts multiples of 8; a channel slice on a multiple of 8 is a block
 * slice, so the free-cat trick carries over).  Convs run on the bf16 matrix cores
 * (v_mfma_f32_16x16x32_bf16) with f32 accumulation and the f32 BN epilogue;
 * outputs are rounded to bf16.  Batch strides are in elements. */

/* Packed bf16 weights for a ConvBR of this shape (elements; 0 = unsupported), and
 * the packing of an f32 OIDHW weight into them (k in {1, 3}, cin % 8 == 0). */
size_t lea_conv3d_packed_elems_bf16(int cout, int cin, int k);
int lea_conv3d_pack_weights_bf16(const float* w, void* packed, int cout, int cin, int k,
                                 void* stream);

/* lea_conv3d_bnrelu on c8 tensors (cout, cin, cin2 multiples of 8). */
int lea_conv3d_bnrelu_bf16(const void* x, int64_t x_bstride, const void* x2, int64_t x2_bstride,
                           int cin2, const void* w_packed, const float* scale, const float* shift,
                           const void* residual, int64_t r_bstride, void* y, int64_t y_bstride,
                           int B, int cin, int cout, int D, int H, int W, int k, unsigned flags,
                           void* stream);

/* lea_conv3d_bnrelu_costvolume on c8 feature maps [B, C/8, H, W, 8] (C % 16 == 0). */
int lea_conv3d_bnrelu_costvolume_bf16(const void* left, const void* right, int64_t f_bstride,
                                      const void* w_packed, const float* scale, const float* shift,
                                      void* y, int64_t y_bstride, int B, int C, int cout, int D3,
                                      int H, int W, unsigned flags, void* stream);


/* Kernel instantiation the bf16 conv of this shape launches. */
const char* lea_conv3d_kernel_name_bf16(int B, int cout, int cin, int D, int H, int W, int k,
                                        int costvolume);

/* 1 if lea_conv3d_bnrelu_bf16 takes LEA_PAIR_SUM for two sources of `cin` channels each
 * into `cout` (3x3x3) at this shape -- the planner's D-streaming form under the current
 * tuning (ABI 13) -- else 0; a caller falls back to two launches when 0. */
int lea_conv3d_bf16_pair_supported(int B, int cin, int cout, int D, int H, int W);

/* ConvBR 1x1 of a trilinearly resampled c8 input (align_corners=True): the cell
 * preprocess after a level change, skip_model_3d.py:44-53, without the resampled
 * tensor -- bit-identical to lea_resample3d_trilinear_bf16 (no epilogue) followed by
 * lea_conv3d_bnrelu_bf16 (k = 1).  x: [B, cin/8, Di, Hi, Wi, 8]; y: [B, cout/8, D, H, W, 8];
 * w_packed: the k = 1 packing of lea_conv3d_pack_weights_bf16; cin % 32 == 0 (<= 128),
 * cout in {16, 32, 64}; flags: LEA_RELU. */
int lea_conv1x1_resampled_bf16(const void* x, int64_t x_bstride, int Di, int Hi, int Wi,
                               const void* w_packed, const float* scale, const float* shift,
                               void* y, int64_t y_bstride, int B, int cin, int cout, int D, int H,
                               int W, unsigned flags, void* stream);

/* lea_resample3d_trilinear on c8 tensors (same source-index rule and epilogue). */
int lea_resample3d_trilinear_bf16(const void* x, int64_t x_bstride, void* y, int64_t y_bstride,
                                  int B, int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                  int align_corners, const float* scale, const float* shift,
                                  unsigned flags, void* stream);


/* Layout converters: f32 NC[D]HW (vol = D*H*W voxels per channel) <-> bf16 c8. */
int lea_to_c8_bf16(const float* x, int64_t x_bstride, void* y, int64_t y_bstride, int B, int C,
                   int64_t vol, void* stream);
int lea_from_c8_bf16(const void* x, int64_t x_bstride, float* y, int64_t y_bstride, int B, int C,
                     int64_t vol, void* stream);

/* lea_tapsum_upsample also takes dtype LEA_BF16: q in the c8 layout, output f32. */

/* Feature-net ConvBR2d 3x3/s1/p1 (operations_2d.py:31-47) on c8 maps [B, C/8, 1, H, W, 8]
 * (the bf16 counterpart of lea_conv2d_bnrelu); weights [cout, cin, 3, 3] f32. */
size_t lea_conv2d_packed_elems_bf16(int cout, int cin);
int lea_conv2d_pack_weights_bf16(const float* w, void* packed, int cout, int cin, void* stream);
int lea_conv2d_bnrelu_bf16(const void* x, int64_t x_bstride, const void* w_packed,
                           const float* scale, const float* shift, const void* residual,
                           int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin, int cout,
                           int H, int W, unsigned flags, void* stream);

/* ---- Winograd F(2,3) / F(4,3)-along-W ConvBR3d, k = 3, fp32 (csrc/conv3d_wino.hip) ----
 * Same operation and arguments as lea_conv3d_bnrelu / lea_conv3d_bnrelu_costvolume
 * (models/operations_3d.py:31-47, retrain/LEAStereo.py:34-48), computed as
 * y[w..w+F-1] = A^T[(G g) . (B^T x)] per (kd, kh): 2/3 (F = 2) or 1/2 (F = 4, on
 * widths that fill 64-wide tile rows) of the direct form's MFMA products, all in
 * fp32.  couts <= 8 run depth-paired (the couts of two output planes share one
 * 16-row MFMA tile, MT = 0 in the kernel name).  Weights are packed by
 * lea_conv3d_wino_pack_weights (a layout of their own, ending in a 256-float zero
 * tail: size the buffer with lea_conv3d_wino_packed_floats); cin (and the first
 * source's channels, and C for the cost volume) must be multiples of 4.        */
size_t lea_conv3d_wino_packed_floats(int cout, int cin);
int lea_conv3d_wino_pack_weights(const float* w, float* packed, int cout, int cin, void* stream);
int lea_conv3d_bnrelu_wino(const void* x, int64_t x_bstride, const void* x2, int64_t x2_bstride,
                           int cin2, const float* w_packed, const float* scale, const float* shift,
                           const void* residual, int64_t r_bstride, void* y, int64_t y_bstride,
                           int B, int cin, int cout, int D, int H, int W, unsigned flags, int dtype,
                           void* stream);
int lea_conv3d_bnrelu_costvolume_wino(const void* left, const void* right, int64_t f_bstride,
                                      const float* w_packed, const float* scale,
                                      const float* shift, void* y, int64_t y_bstride, int B, int C,
                                      int cout, int D3, int H, int W, unsigned flags, int dtype,
                                      void* stream);
/* Kernel instantiation the Winograd entries launch for this shape
 * ("conv3d_wino_kernel<F, Q, MT, NP, TD, CV>", or on the W x D engine
 * "conv3d_wino2_kernel<Q, WC, MTE, NW, OCC, PV, CV>" / "conv3d_wino2p_kernel"; cin = 0:
 * unknown, planned as a deep layer).  The engines' tuning hooks are in
 * leastereo_hip_tuning.h. */
const char* lea_conv3d_wino_kernel_name(int B, int cin, int cout, int D, int H, int W, int costvolume);

/* ---- Matching-net stem0 over the cost volume, factored (csrc/cv_stem.hip) ----
 * Replaces retrain/LEAStereo.py:34-48 + skip_model_3d.py:141 like
 * lea_conv3d_bnrelu_costvolume, without a 3D convolution: every cost-volume plane is
 * a shifted copy of the feature maps, so with u = w - d
 *   conv(cost)[o, d, h, w] = sum_{kd: 0 <= d+kd-1 < D3} ( LK[kd][max(kd-u, 0)][o, h, w]
 *                                                       + Bk[kd][o, h, u-kd+1] )
 * (LK[kd][t] = 0 for kd - u >= 3; Bk[kd] at column -1 = K2[kd] at column 0; the last
 * column w = W-1 subtracts K2[kd][o, h, u-kd+2]), where LK, Bk, K2 are 2D 3x3 convs of
 * the left / right feature maps:
 *   lea_cv_stem_split_weights: stem0's [cout, 2C, 3, 3, 3] f32 weight ->
 *     wl [9 cout, C, 3, 3]: wl[(3 kd + t) cout + o][c][kh][kw] = W[o][c][kd][kh][kw] (kw >= t)
 *     wr [6 cout, C, 3, 3]: wr[kd cout + o] = W[o][C + c][kd]  (Bk)
 *                           wr[(3 + kd) cout + o][c][kh][1] = W[o][C + c][kd][kh][2]  (K2)
 *   maps: lea_conv2d_bnrelu (f32) / lea_conv2d_bnrelu_bf16 (c8) of left with wl and of
 *     right with wr, no BN/ReLU: lmaps [B, 9 cout, H, W], rmaps [B, 6 cout, H, W];
 *   lea_cv_stem_combine: the sum above, the folded BN and ReLU, written as
 *     y [B, cout, D3, H, W] (dtype LEA_F32: NCDHW, W % 4 == 0; LEA_BF16: c8 maps in,
 *     c8 out, cout % 8 == 0).  D3 >= 2.  Equal to the direct conv up to summation
 *     order (and, at bf16, the maps' rounding). */
int lea_cv_stem_split_weights(const float* w, float* wl, float* wr, int cout, int C, void* stream);
int lea_cv_stem_combine(const void* lmaps, int64_t l_bstride, const void* rmaps, int64_t r_bstride,
                        const float* scale, const float* shift, void* y, int64_t y_bstride, int B,
                        int cout, int D3, int H, int W, unsigned flags, int dtype, void* stream);

/* ---- host steps either side of forward ---- */

/* load_data + test_transform of predict.py, fused: replaces predict.py:162-184
 * (per image channel (x - mean) / std over the WHOLE image, np.mean / np.std in
 * float64, population std, stored float32) and predict.py:144-159 (zero-pad
 * top-left when H <= crop_h and W <= crop_w, else centre-crop at
 * start = int((H - crop) / 2); an image that neither fits nor covers the crop is
 * rejected, as the reference's copy into the crop fails).
 *   left/right: B uint8 HWC images [B, H, W, pix_stride] (RGB = 3, RGBA = 4; the
 *               first 3 channels are used, predict.py:170-182)
 *   out_left/out_right: [B, 3, crop_h, crop_w] float32
 *   workspace: lea_standardize_workspace_bytes(B) bytes of device memory (cleared
 *              by the call; holds the exact integer sums).                       */
size_t lea_standardize_workspace_bytes(int B);
int lea_standardize_crop_u8(const void* left, const void* right, int B, int H, int W,
                            int pix_stride, float* out_left, float* out_right, int crop_h,
                            int crop_w, void* workspace, void* stream);

/* Disparity metrics of one batch, per pair b (device out[b][8], float64):
 *   [0] n    of evaluation.py:287 mask (gt >= 0.001 & gt <= maxdisp)
 *   [1] sum |pred - gt| over that mask          (EPE = [1] / [0], evaluation.py:288)
 *   [2] n    of utils/metrics.py:6-8 validity (gt > 0.001 & gt < maxdisp)
 *   [3] n correct, utils/metrics.py:16-19        (3-px error = 1 - [3] / [2])
 *   [4..6] n with abs_diff <= thr1..thr3, :41-43 (bad-thr = 1 - [4+i] / [2])
 * abs_diff follows the reference's int64 array: |gt - pred| truncated toward zero
 * on valid pixels, 10000 elsewhere.  round_pred applies evaluation.py:169
 * (pred.round() + z_shift, half-to-even) first.  correct (optional, [B, H*W]
 * uint8) receives the 3-px correct mask of calculate_3px_error_and_correct_mask.
 * pred/gt: [B, H, W] float32 with batch strides in elements.
 * workspace: lea_disparity_metrics_workspace_bytes(B, H, W) bytes.               */
size_t lea_disparity_metrics_workspace_bytes(int B, int H, int W);
int lea_disparity_metrics(const float* pred, int64_t pred_bstride, const float* gt,
                          int64_t gt_bstride, int B, int H, int W, float maxdisp, int round_pred,
                          int z_shift, int thr1, int thr2, int thr3, unsigned char* correct,
                          double* out, void* workspace, void* stream);

/* ---- training backward of ConvBR3d (operations_3d.py:31-47
 * as train.py:130-178 runs it: BatchNorm3d in train mode) ----
 * All tensors NCDHW contiguous fp32, V = D*H*W.  Composition (csrc/conv3d_grad.hip):
 *   forward  z = lea_conv3d_bnrelu(x, w; no scale/shift, flags 0)
 *            y = lea_bn_forward_f32(z)
 *   backward dz = lea_bn_backward_f32(dy, y, z)
 *            dx = lea_conv3d_bnrelu(dz, pack(lea_conv3d_flip_weights(w)); flags 0)
 *            dw = lea_conv3d_wgrad(x, dz)                                        */

/* dw[co][ci][kd][kh][kw] = sum_{b,d,h,w} dz[b][co][d][h][w] * x[b][ci][d+kd-k/2][h+kh-k/2][w+kw-k/2]
 * (zero padding; the weight gradient of a stride-1, pad k/2 Conv3d without bias,
 * which torch computes in aten's convolution_backward).  dw is overwritten;
 * workspace: lea_conv3d_wgrad_workspace_bytes(...) bytes (per-wave partials, summed
 * in a fixed order: the result is deterministic).  k in {1, 3}.                  */
size_t lea_conv3d_wgrad_workspace_bytes(int B, int cin, int cout, int D, int H, int W, int k);
int lea_conv3d_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes,
                     int B, int cin, int cout, int D, int H, int W, int k, void* stream);

/* The feature net's Conv2d 3x3 / stride 1 / pad 1 (operations_2d.py:31-47, the cells and
 * stem0/stem2 of new_model_2d.py:93-95): dw[co][ci][kh][kw] = sum_{b,h,w} dz[b][co][h][w] *
 * x[b][ci][h+kh-1][w+kw-1], the same deterministic MFMA reduction as lea_conv3d_wgrad.
 * x: [B, cin, H, W], dz: [B, cout, H, W], dw: [cout, cin, 3, 3].  The input gradient is
 * lea_conv2d_bnrelu of dz with w flipped along (kh, kw) and transposed to [cin, cout, 3, 3]. */
size_t lea_conv2d_wgrad_workspace_bytes(int B, int cin, int cout, int H, int W);
int lea_conv2d_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes,
                     int B, int cin, int cout, int H, int W, void* stream);

/* Backward of lea_conv2d_s3_bnrelu's convolution (stem1, new_model_2d.py:94; stride 3,
 * pad 1, 3x3: every input pixel is read by at most one output tap), w: [cout, cin, 3, 3]:
 *   dx[b][ci][y][x] = sum_co w[co][ci][(y+1)%3][(x+1)%3] * dz[b][co][(y+1)/3][(x+1)/3]
 *   (0 where (y+1)/3 = Ho or (x+1)/3 = Wo: the last row / column when Hi / Wi % 3 == 0)
 *   dw[co][ci][kh][kw] = sum_{b,oy,ox} dz[b][co][oy][ox] * x[b][ci][3oy+kh-1][3ox+kw-1]
 * x/dx: [B, cin, Hi, Wi]; dz: [B, cout, (Hi-1)/3+1, (Wi-1)/3+1]; contiguous fp32.
 * workspace: lea_conv2d_s3_wgrad_workspace_bytes(...) bytes (per-slice partials, summed
 * in a fixed order). */
int lea_conv2d_s3_backward_data(const float* dz, const float* w, float* dx, int B, int cin, int cout,
                                int Hi, int Wi, void* stream);
size_t lea_conv2d_s3_wgrad_workspace_bytes(int B, int cin, int cout, int Hi, int Wi);
int lea_conv2d_s3_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes,
                        int B, int cin, int cout, int Hi, int Wi, void* stream);

/* wt[ci][co][kd][kh][kw] = w[co][ci][k-1-kd][k-1-kh][k-1-kw]: the input gradient of a
 * stride-1, pad k/2 conv is the forward conv of dz with this weight.             */
int lea_conv3d_flip_weights(const float* w, float* wt, int cout, int cin, int k, void* stream);

/* BatchNorm3d + optional ReLU (flags LEA_RELU), operations_3d.py:44-46 in
 * torch.nn.BatchNorm3d's semantics: training = 1 normalises by the batch mean and
 * biased variance over (B, D, H, W) and updates running_mean / running_var with
 * momentum (unbiased variance; both may be NULL to skip the update); training = 0
 * uses the running stats.  gamma/beta NULL = 1/0.  y = relu((z - mean) * invstd *
 * gamma + beta); mean/invstd ([C], device) are written for the backward.
 * workspace: lea_bn_workspace_bytes(C) bytes (train mode).                      */
size_t lea_bn_workspace_bytes(int C);
int lea_bn_forward_f32(const float* z, float* y, int B, int C, int64_t V, const float* gamma,
                       const float* beta, float* running_mean, float* running_var, float momentum,
                       float eps, int training, unsigned flags, float* mean, float* invstd,
                       void* workspace, void* stream);

/* Backward of lea_bn_forward_f32: g = dy * [y > 0] (LEA_RELU) or dy;
 * dbeta = sum g, dgamma = sum g * xhat (xhat = (z - mean) * invstd, either may be NULL);
 * dz = gamma * invstd * (g - dbeta/N - xhat * dgamma/N) in train mode,
 * gamma * invstd * g in eval mode (N = B * V).  workspace: lea_bn_workspace_bytes(C). */
int lea_bn_backward_f32(const float* dy, const float* y, const float* z, float* dz, int B, int C,
                        int64_t V, const float* gamma, const float* mean, const float* invstd,
                        int training, unsigned flags, float* dgamma, float* dbeta, void* workspace,
                        void* stream);

/* Backward of lea_resample3d_trilinear without epilogue (F.interpolate trilinear,
 * skip_model_3d.py:48,50,162, align_corners 1; build_model_2d.py:53, 0):
 * dx[b][c] = interp^T(dy[b][c]), as three deterministic 1-D transposed passes with
 * the forward's source-index rule.  dy: [B, C, Do, Ho, Wo], dx: [B, C, Di, Hi, Wi],
 * contiguous; workspace: lea_resample3d_backward_workspace_bytes(...) bytes.     */
size_t lea_resample3d_backward_workspace_bytes(int B, int C, int Di, int Hi, int Wi, int Do, int Ho,
                                               int Wo);
int lea_resample3d_trilinear_backward(const float* dy, float* dx, void* workspace, size_t ws_bytes,
                                      int B, int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                      int align_corners, void* stream);

/* Backward of lea_disparity_regression (build_model_2d.py:33-42,52-57): with
 * U = trilinear(cost, [maxdisp, 3H3, 3W3], align_corners=False), p = softmax(-U, d),
 * disp = sum_d d p_d (disp: the forward's output),
 *   dU[b, d, h, w] = -dout[b, h, w] * p_d * (d - disp[b, h, w]),
 * and writes dV = its transpose along D only (the depth lerp's two taps per d summed
 * onto the D3 cost planes): [B, D3, 3H3, 3W3].  dcost = the H/W part,
 * lea_resample3d_trilinear_backward(dV, [D3, H3, W3] <- [D3, 3H3, 3W3], align_corners = 0). */
int lea_disparity_regression_backward(const float* cost, const float* disp, const float* dout,
                                      float* dV, int B, int D3, int H3, int W3, int maxdisp,
                                      void* stream);

/* Backward of lea_build_cost_volume (retrain/LEAStereo.py:34-48):
 *   dleft[b,c,h,w]  = sum_{i <= w} dcost[b, c, i, h, w]
 *   dright[b,c,h,w] = sum_{i < W - w} dcost[b, C + c, i, h, w + i]
 * dcost: [B, 2C, D3, H, W]; dleft/dright: [B, C, H, W]; fp32.                    */
int lea_build_cost_volume_backward(const float* dcost, float* dleft, float* dright, int B, int C,
                                   int H, int W, int D3, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LEASTEREO_HIP_H */
