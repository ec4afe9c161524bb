// Trilinear resample of an NCDHW volume with PyTorch's source-index rule, with an
// optional per-channel affine + ReLU epilogue.
// Replaces F.interpolate(..., mode='trilinear', align_corners=True) at
// retrain/skip_model_3d.py:48,50 and nn.Upsample at :162-164 (the level changes
// between the 1x, 1/2x and 1/4x matching-net resolutions).
//
// The epilogue serves the up-sampling cell preprocess: ConvBR1x1(interp(x)) =
// relu(scale * interp(W x) + shift) because the 1x1 conv W and the trilinear
// interpolation are both linear maps on different axes and commute.  The 1x1
// conv then runs at the *input* resolution (8x fewer voxels for x2 up-sampling)
// and only its narrow output is resampled -- straight into the cell's cat slot.
//
// One thread per output voxel along W (coalesced stores); the d and h source
// rows are uniform per workgroup, the 8 taps come from two row pairs that
// neighbouring threads share through L1/L2.  Streaming: bound by the output write.
#include "common.h"

namespace lea {

__global__ __launch_bounds__(256) void resample3d_f32(const float* __restrict__ x, long long xbs,
                                                      float* __restrict__ y, long long ybs, int C,
                                                      int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                                      float rd, float rh, float rw, int ac,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      unsigned flags) {
#pragma clang fp contract(off)
  const int ow = blockIdx.x * blockDim.x + threadIdx.x;
  if (ow >= Wo) return;
  const int oh = blockIdx.y % Ho;
  const int od = blockIdx.y / Ho;
  const int bc = blockIdx.z;  // b * C + c
  const int b = bc / C, c = bc - b * C;
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const Axis ah = axis_index(rh, oh, Hi, Ho, ac);
  const Axis aw = axis_index(rw, ow, Wi, Wo, ac);
  const long long HWi = (long long)Hi * Wi;
  const float* xc = x + (long long)b * xbs + (long long)c * Di * HWi;
  const float* p00 = xc + ad.i0 * HWi + (long long)ah.i0 * Wi;
  const float* p01 = xc + ad.i0 * HWi + (long long)ah.i1 * Wi;
  const float* p10 = xc + ad.i1 * HWi + (long long)ah.i0 * Wi;
  const float* p11 = xc + ad.i1 * HWi + (long long)ah.i1 * Wi;
  float v = trilerp(ad, ah, aw, p00, p01, p10, p11);
  if (scale) v = v * scale[c] + shift[c];
  if (flags & LEA_RELU) v = fmaxf(v, 0.f);
  y[(long long)b * ybs + (long long)c * Do * Ho * Wo + ((long long)od * Ho + oh) * Wo + ow] = v;
}

}  // namespace lea

extern "C" int lea_resample3d_trilinear(const void* x, int64_t x_bstride, void* y, int64_t y_bstride,
                                        int B, int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                        int align_corners, const float* scale, const float* shift,
                                        unsigned flags, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(x && y && x != y, "lea_resample3d_trilinear: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_resample3d_trilinear: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && C > 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 && Wo > 0,
                "lea_resample3d_trilinear: bad shape");
  LEA_CHECK_ARG((long long)Do * Ho <= 65535 && (long long)B * C <= 65535,
                "lea_resample3d_trilinear: grid too large (Do*Ho=%d, B*C=%d)", Do * Ho, B * C);
  if (dtype != LEA_F32) {
    set_error("lea_resample3d_trilinear: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const int ac = align_corners ? 1 : 0;
  dim3 block(Wo >= 256 ? 256 : ((Wo + 63) / 64) * 64);
  dim3 grid((Wo + block.x - 1) / block.x, Do * Ho, B * C);
  resample3d_f32<<<grid, block, 0, as_stream(stream)>>>(
      (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo,
      axis_ratio(Di, Do, ac), axis_ratio(Hi, Ho, ac), axis_ratio(Wi, Wo, ac), ac, scale, shift,
      flags);
  return launch_status("lea_resample3d_trilinear");
}
