// Matching-net head: last_3(Upsample(y)) without the upsampled volume.
// Replaces skip_model_3d.py:161-173 for the usual case (last cell at half
// resolution): mat = last_3(upsample_6(last_6(out11))), where upsample_6 is a
// trilinear align_corners=True resize to the cost-volume size and last_3 a
// 3x3x3 conv (32 -> 1, no BN/ReLU, :132).
//
// Both maps are linear, so with Q[co*27 + tap] = sum_ci W[co][ci][tap] * y[ci]
// (a 1x1 conv at the LOW resolution, run by the MFMA 1x1 engine) the output is
//     out[co](v) = sum_tap  interp(Q[co*27 + tap])(v + off(tap))
// where a tap whose position v + off(tap) falls outside the output volume
// contributes 0 (the conv's zero padding of the upsampled tensor).  Same math
// as the reference up to fp32 reassociation; the 32-channel full-resolution
// tensor (503 MB at 576x960 D192) is never written or read.
//
// Mapping: one thread per output voxel; workgroup = a row segment of one
// (b, co, d, h), so the d/h source rows of each tap are uniform and only the
// w-axis weights are per lane.  27 trilinear samples per voxel from the
// cache-resident Q (53 MB at 576x960 D192).
#include "common.h"

namespace lea {

__global__ __launch_bounds__(512) void tapsum_upsample_f32(
    const float* __restrict__ q, long long qbs, float* __restrict__ y, long long ybs, int cout,
    int Di, int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh, float rw,
    const float* __restrict__ scale, const float* __restrict__ shift, unsigned flags) {
#pragma clang fp contract(off)
  const int row = blockIdx.x;  // ((b * cout + co) * Do + d) * Ho + h
  const int h = row % Ho;
  int r = row / Ho;
  const int d = r % Do;
  r /= Do;
  const int co = r % cout;
  const int b = r / cout;
  const long long HWi = (long long)Hi * Wi;
  const long long vol = HWi * Di;
  const float* qb = q + (long long)b * qbs + (long long)co * 27 * vol;
  Axis aws[3];
  bool wok[3];
  for (int w = threadIdx.x; w < Wo; w += blockDim.x) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int p = w + kw - 1;
      wok[kw] = (unsigned)p < (unsigned)Wo;
      aws[kw] = axis_index(rw, wok[kw] ? p : 0, Wi, Wo, 1);
    }
    float acc = 0.f;
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      const int pd = d + kd - 1;
      if ((unsigned)pd >= (unsigned)Do) continue;
      const Axis ad = axis_index(rd, pd, Di, Do, 1);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int ph = h + kh - 1;
        if ((unsigned)ph >= (unsigned)Ho) continue;
        const Axis ah = axis_index(rh, ph, Hi, Ho, 1);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float* qt = qb + (long long)((kd * 3 + kh) * 3 + kw) * vol;
          const float* p00 = qt + ad.i0 * HWi + (long long)ah.i0 * Wi;
          const float* p01 = qt + ad.i0 * HWi + (long long)ah.i1 * Wi;
          const float* p10 = qt + ad.i1 * HWi + (long long)ah.i0 * Wi;
          const float* p11 = qt + ad.i1 * HWi + (long long)ah.i1 * Wi;
          const float v = trilerp(ad, ah, aws[kw], p00, p01, p10, p11);
          acc += wok[kw] ? v : 0.f;
        }
      }
    }
    if (scale) acc = acc * scale[co] + shift[co];
    if (flags & LEA_RELU) acc = fmaxf(acc, 0.f);
    y[(long long)b * ybs + (((long long)co * Do + d) * Ho + h) * Wo + w] = acc;
  }
}

}  // namespace lea

extern "C" int lea_tapsum_upsample(const void* q, int64_t q_bstride, void* y, int64_t y_bstride,
                                   int B, int cout, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                   const float* scale, const float* shift, unsigned flags,
                                   int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(q && y && q != y, "lea_tapsum_upsample: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_tapsum_upsample: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && cout > 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 && Wo > 0,
                "lea_tapsum_upsample: bad shape");
  LEA_CHECK_ARG((long long)B * cout * Do * Ho < (1LL << 31), "lea_tapsum_upsample: grid too large");
  if (dtype != LEA_F32) {
    set_error("lea_tapsum_upsample: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const int threads = Wo >= 512 ? 512 : ((Wo + 63) / 64) * 64;  // one row per workgroup
  dim3 grid((unsigned)((long long)B * cout * Do * Ho));
  tapsum_upsample_f32<<<grid, threads, 0, as_stream(stream)>>>(
      (const float*)q, q_bstride, (float*)y, y_bstride, cout, Di, Hi, Wi, Do, Ho, Wo,
      axis_ratio(Di, Do, 1), axis_ratio(Hi, Ho, 1), axis_ratio(Wi, Wo, 1), scale, shift, flags);
  return launch_status("lea_tapsum_upsample");
}
