// Feature-net stem1: Conv2d 3x3, stride 3, pad 1 (no bias) -> folded BN -> ReLU.
// Replaces models/operations_2d.py:31-47 as used by retrain/new_model_2d.py:94
// (ConvBR(initial_fm // 2, initial_fm, 3, stride=3, padding=1)).
//
// Stride 3 with a 3x3 kernel tiles the input without overlap: output pixel
// (ho, wo) reads input rows 3ho-1..3ho+1, columns 3wo-1..3wo+1, and every input
// pixel is read by exactly one output.  So there is no reuse to stage: one thread
// per output pixel loads its cin x 3 x 3 patch once and runs the 9*cin-long dot
// product for a block of 16 output channels, the weights (uniform across the
// wave) coming through scalar loads.  1.1 GFLOP per stereo pair at 576x960.
#include "common.h"

namespace lea {

constexpr int kS3CoBlock = 16;

__global__ __launch_bounds__(256) void conv2d_s3_kernel(const float* __restrict__ x, long long xbs,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        float* __restrict__ y, long long ybs, int cin,
                                                        int cout, int Hi, int Wi, int Ho, int Wo,
                                                        unsigned flags) {
  const int b = blockIdx.z;
  const int co0 = blockIdx.y * kS3CoBlock;
  const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (long long)Ho * Wo) return;
  const int ho = (int)(pix / Wo), wo = (int)(pix - (long long)ho * Wo);
  const float* xb = x + (long long)b * xbs;
  const long long HWi = (long long)Hi * Wi;
  float acc[kS3CoBlock];
#pragma unroll
  for (int j = 0; j < kS3CoBlock; ++j) acc[j] = 0.f;
  for (int ci = 0; ci < cin; ++ci) {
    float v[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = 3 * ho + kh - 1, ww = 3 * wo + kw - 1;
        v[kh * 3 + kw] = ((unsigned)h < (unsigned)Hi && (unsigned)ww < (unsigned)Wi)
                             ? xb[ci * HWi + (long long)h * Wi + ww]
                             : 0.f;
      }
#pragma unroll
    for (int j = 0; j < kS3CoBlock; ++j) {
      const int co = co0 + j;
      if (co < cout) {
        const float* wc = w + ((long long)co * cin + ci) * 9;
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[j] = fmaf(wc[t], v[t], acc[j]);
      }
    }
  }
  const bool relu = flags & LEA_RELU;
#pragma unroll
  for (int j = 0; j < kS3CoBlock; ++j) {
    const int co = co0 + j;
    if (co >= cout) continue;
    float r = acc[j];
    if (scale) r = r * scale[co] + shift[co];
    if (relu) r = fmaxf(r, 0.f);
    y[(long long)b * ybs + (long long)co * Ho * Wo + pix] = r;
  }
}

}  // namespace lea

extern "C" int lea_conv2d_s3_bnrelu(const void* x, int64_t x_bstride, const float* w,
                                    const float* scale, const float* shift, void* y,
                                    int64_t y_bstride, int B, int cin, int cout, int Hi, int Wi,
                                    unsigned flags, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(x && w && y && x != y, "lea_conv2d_s3_bnrelu: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_conv2d_s3_bnrelu: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && Hi > 0 && Wi > 0,
                "lea_conv2d_s3_bnrelu: bad shape B=%d cin=%d cout=%d Hi=%d Wi=%d", B, cin, cout, Hi,
                Wi);
  LEA_CHECK_ARG(B <= 65535 && cout <= 65535 * kS3CoBlock && (long long)cin * Hi * Wi < (1LL << 31),
                "lea_conv2d_s3_bnrelu: too large");
  if (dtype != LEA_F32) {
    set_error("lea_conv2d_s3_bnrelu: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const int Ho = (Hi - 1) / 3 + 1, Wo = (Wi - 1) / 3 + 1;  // (H + 2*1 - 3) / 3 + 1
  const long long pix = (long long)Ho * Wo;
  dim3 grid((unsigned)((pix + 255) / 256), (cout + kS3CoBlock - 1) / kS3CoBlock, B);
  conv2d_s3_kernel<<<grid, 256, 0, as_stream(stream)>>>((const float*)x, x_bstride, w, scale, shift,
                                                        (float*)y, y_bstride, cin, cout, Hi, Wi, Ho,
                                                        Wo, flags);
  return launch_status("lea_conv2d_s3_bnrelu");
}
