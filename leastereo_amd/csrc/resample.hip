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
// Mapping: grid.y = output plane (b, c, od) -- its depth weights are uniform;
// threads walk the plane's (oh, 4-wide ow quad) cells with a grid stride, so a
// workgroup writes several KB (the first version launched one 256-thread group
// per half row and was dispatch-bound at ~0.55 TB/s).  Output is stored as one
// 16-byte vector per quad when Wo % 4 == 0.  Bound by the output write.
#include "common.h"

namespace lea {

template <bool VEC>
__global__ __launch_bounds__(256) void resample3d_f32(const float* __restrict__ x, long long xbs,
                                                      float* __restrict__ y, long long ybs, int C,
                                                      int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                                      float rd, float rh, float rw, int ac,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      unsigned flags) {
#pragma clang fp contract(off)
  const int plane = blockIdx.y;  // (b * C + c) * Do + od
  const int od = plane % Do;
  const int bc = plane / Do;
  const int b = bc / C, c = bc - b * C;
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const long long HWi = (long long)Hi * Wi;
  const float* xc = x + (long long)b * xbs + (long long)c * Di * HWi;
  const float* q0 = xc + ad.i0 * HWi;
  const float* q1 = xc + ad.i1 * HWi;
  float* yp = y + (long long)b * ybs + ((long long)c * Do + od) * Ho * Wo;
  const float sc = scale ? scale[c] : 1.f;
  const float sh = scale ? shift[c] : 0.f;
  const bool relu = flags & LEA_RELU;
  const int wq = VEC ? Wo / 4 : Wo;
  const int cells = Ho * wq;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < cells; t += gridDim.x * blockDim.x) {
    const int oh = t / wq;
    const int q = t - oh * wq;
    const Axis ah = axis_index(rh, oh, Hi, Ho, ac);
    const float* p00 = q0 + (long long)ah.i0 * Wi;
    const float* p01 = q0 + (long long)ah.i1 * Wi;
    const float* p10 = q1 + (long long)ah.i0 * Wi;
    const float* p11 = q1 + (long long)ah.i1 * Wi;
    float v[VEC ? 4 : 1];
#pragma unroll
    for (int e = 0; e < (VEC ? 4 : 1); ++e) {
      const Axis aw = axis_index(rw, (VEC ? 4 * q : q) + e, Wi, Wo, ac);
      float r = trilerp(ad, ah, aw, p00, p01, p10, p11);
      if (scale) r = r * sc + sh;
      if (relu) r = fmaxf(r, 0.f);
      v[e] = r;
    }
    if constexpr (VEC)
      *reinterpret_cast<float4*>(yp + (long long)oh * Wo + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
    else
      yp[(long long)oh * Wo + q] = v[0];
  }
}

// Row-staged variant (the up-sampling level changes, 8-16 channels at x2):
// a workgroup owns R output rows of one output plane; the <= R*rh + 2 source
// rows of its two source planes are first copied into LDS with coalesced loads,
// then every output quad interpolates from LDS.  The gather version above issued
// 32 dependent global loads per quad and ran at ~1.2 TB/s; here each source
// element is read from HBM/L2 once per workgroup.  Same Axis/trilerp arithmetic,
// so both kernels produce identical bits.
template <bool VEC>
__global__ __launch_bounds__(256) void resample3d_rows_f32(
    const float* __restrict__ x, long long xbs, float* __restrict__ y, long long ybs, int C, int Di,
    int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh, float rw, int ac, int R, int nrmax,
    const float* __restrict__ scale, const float* __restrict__ shift, unsigned flags) {
#pragma clang fp contract(off)
  extern __shared__ float rows[];  // [2][nrmax][Wi]
  const int plane = blockIdx.y;
  const int od = plane % Do;
  const int bc = plane / Do;
  const int b = bc / C, c = bc - b * C;
  const int oh0 = blockIdx.x * R;
  const int oh1 = min(oh0 + R, Ho);
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const int r_lo = axis_index(rh, oh0, Hi, Ho, ac).i0;
  const int r_hi = axis_index(rh, oh1 - 1, Hi, Ho, ac).i1;
  // nrmax = the host's exact bound (staged_rows); past it: NaN outputs, never unstaged rows
  const bool over = r_hi - r_lo + 1 > nrmax;
  const int nr = over ? 0 : r_hi - r_lo + 1;
  const long long HWi = (long long)Hi * Wi;
  const float* xc = x + (long long)b * xbs + (long long)c * Di * HWi + (long long)r_lo * Wi;
  const float* src[2] = {xc + ad.i0 * HWi, xc + ad.i1 * HWi};
  const int n1 = nr * Wi;
  for (int e = threadIdx.x; e < 2 * n1; e += blockDim.x) {
    const int p = e >= n1;
    const int r = e - p * n1;
    rows[p * nrmax * Wi + r] = src[p][r];
  }
  __syncthreads();
  float* yp = y + (long long)b * ybs + ((long long)c * Do + od) * Ho * Wo;
  const float sc = scale ? scale[c] : 1.f;
  const float sh = scale ? shift[c] : 0.f;
  const bool relu = flags & LEA_RELU;
  const int wq = VEC ? Wo / 4 : Wo;
  const int cells = (oh1 - oh0) * wq;
  const float* l0 = rows;
  const float* l1 = rows + nrmax * Wi;
  for (int t = threadIdx.x; t < cells; t += blockDim.x) {
    const int oh = oh0 + t / wq;
    const int q = t % wq;
    const Axis ah = axis_index(rh, oh, Hi, Ho, ac);
    const int r0 = over ? 0 : (ah.i0 - r_lo) * Wi, r1 = over ? 0 : (ah.i1 - r_lo) * Wi;
    float v[VEC ? 4 : 1];
#pragma unroll
    for (int e = 0; e < (VEC ? 4 : 1); ++e) {
      const Axis aw = axis_index(rw, (VEC ? 4 * q : q) + e, Wi, Wo, ac);
      float r = trilerp(ad, ah, aw, l0 + r0, l0 + r1, l1 + r0, l1 + r1);
      if (scale) r = r * sc + sh;
      if (relu) r = fmaxf(r, 0.f);
      v[e] = over ? __builtin_nanf("") : r;
    }
    if constexpr (VEC)
      *reinterpret_cast<float4*>(yp + (long long)oh * Wo + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
    else
      yp[(long long)oh * Wo + q] = v[0];
  }
}

// Separable variant (r04; the default when Wo % 4 == 0): trilerp's innermost terms are the
// W-lerps of the four source rows, aw.l0 * row[aw.i0] + aw.l1 * row[aw.i1], so a workgroup
// first forms the W-lerped rows of its <= nrmax source rows of both source planes at every
// output column (each thread owns columns: one W axis per column, loads straight from
// global), then every output quad combines four float4s of them with the H and D weights
// in trilerp's own expression tree -- bit-identical to the row-staged and gather kernels.
// Per output value: ~1.25 W-lerps (the rows two output rows share are lerped once) and one
// 16-byte LDS read per source-row pair, instead of 4 W-lerps and 8 LDS reads.
__global__ __launch_bounds__(256) void resample3d_sep_f32(
    const float* __restrict__ x, long long xbs, float* __restrict__ y, long long ybs, int C, int Di,
    int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh, float rw, int ac, int R, int nrmax,
    const float* __restrict__ scale, const float* __restrict__ shift, unsigned flags) {
#pragma clang fp contract(off)
  extern __shared__ float wrows[];  // [2][nrmax][Wo]: W-lerped source rows
  const int plane = blockIdx.y;
  const int od = plane % Do;
  const int bc = plane / Do;
  const int b = bc / C, c = bc - b * C;
  const int oh0 = blockIdx.x * R;
  const int oh1 = min(oh0 + R, Ho);
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const int r_lo = axis_index(rh, oh0, Hi, Ho, ac).i0;
  const int r_hi = axis_index(rh, oh1 - 1, Hi, Ho, ac).i1;
  // nrmax = the host's exact bound (staged_rows); past it: NaN outputs, never unstaged rows
  const bool over = r_hi - r_lo + 1 > nrmax;
  const int nr = over ? 0 : r_hi - r_lo + 1;
  const long long HWi = (long long)Hi * Wi;
  const float* xc = x + (long long)b * xbs + (long long)c * Di * HWi + (long long)r_lo * Wi;
  const float* src0 = xc + ad.i0 * HWi;
  const float* src1 = xc + ad.i1 * HWi;
  for (int xo = threadIdx.x; xo < Wo; xo += blockDim.x) {
    const Axis aw = axis_index(rw, xo, Wi, Wo, ac);
    for (int r = 0; r < nr; ++r) {
      const float* q0 = src0 + (long long)r * Wi;
      const float* q1 = src1 + (long long)r * Wi;
      wrows[r * Wo + xo] = aw.l0 * q0[aw.i0] + aw.l1 * q0[aw.i1];
      wrows[(nrmax + r) * Wo + xo] = aw.l0 * q1[aw.i0] + aw.l1 * q1[aw.i1];
    }
  }
  __syncthreads();
  float* yp = y + (long long)b * ybs + ((long long)c * Do + od) * Ho * Wo;
  const float sc = scale ? scale[c] : 1.f;
  const float sh = scale ? shift[c] : 0.f;
  const bool relu = flags & LEA_RELU;
  const int wq = Wo / 4;
  const int cells = (oh1 - oh0) * wq;
  const float4* w4 = reinterpret_cast<const float4*>(wrows);
  for (int t = threadIdx.x; t < cells; t += blockDim.x) {
    const int oh = oh0 + t / wq;
    const int q = t % wq;
    const Axis ah = axis_index(rh, oh, Hi, Ho, ac);
    const int r0 = over ? 0 : ah.i0 - r_lo, r1 = over ? 0 : ah.i1 - r_lo;
    const float4 a00 = w4[r0 * wq + q], a01 = w4[r1 * wq + q];
    const float4 a10 = w4[(nrmax + r0) * wq + q], a11 = w4[(nrmax + r1) * wq + q];
    const float p00[4] = {a00.x, a00.y, a00.z, a00.w}, p01[4] = {a01.x, a01.y, a01.z, a01.w};
    const float p10[4] = {a10.x, a10.y, a10.z, a10.w}, p11[4] = {a11.x, a11.y, a11.z, a11.w};
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float r = ad.l0 * (ah.l0 * p00[e] + ah.l1 * p01[e]) + ad.l1 * (ah.l0 * p10[e] + ah.l1 * p11[e]);
      if (scale) r = r * sc + sh;
      if (relu) r = fmaxf(r, 0.f);
      v[e] = over ? __builtin_nanf("") : r;
    }
    *reinterpret_cast<float4*>(yp + (long long)oh * Wo + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

int g_resample_mode = 0;  // lea_resample_set_mode: 0 auto, 1 row-staged, 2 gather

}  // namespace lea

extern "C" int lea_resample_set_mode(int mode) {
  lea::clear_error();
  if (mode < 0 || mode > 2) {
    lea::set_error("lea_resample_set_mode: mode=%d", mode);
    return LEA_E_INVALID;
  }
  lea::g_resample_mode = mode;
  return 0;
}

extern "C" int lea_staged_rows(int Hi, int Ho, int ac, int R, int halo) {
  lea::clear_error();
  // a row count can be any positive int (~1008 rows at config 5), so an error is -1, never
  // LEA_E_INVALID
  if (!(Hi > 0 && Ho > 0 && R > 0 && halo >= 0 && (ac == 0 || ac == 1))) {
    lea::set_error("lea_staged_rows: Hi=%d Ho=%d ac=%d R=%d halo=%d", Hi, Ho, ac, R, halo);
    return -1;
  }
  return lea::staged_rows(Hi, Ho, ac, R, halo);
}

extern "C" int lea_resample3d_trilinear(const void* x, int64_t x_bstride, void* y, int64_t y_bstride,
                                        int B, int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                        int align_corners, const float* scale, const float* shift,
                                        unsigned flags, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_resample3d_trilinear");
  LEA_CHECK_ARG(x && y && x != y, "lea_resample3d_trilinear: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_resample3d_trilinear: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && C > 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 && Wo > 0,
                "lea_resample3d_trilinear: bad shape");
  LEA_CHECK_ARG((long long)B * C * Do <= 65535 && (long long)Ho * Wo < (1LL << 31),
                "lea_resample3d_trilinear: grid too large (B*C*Do=%lld)", (long long)B * C * Do);
  if (dtype != LEA_F32) {
    set_error("lea_resample3d_trilinear: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  // 16-byte stores need Wo % 4 == 0 and a 16-byte aligned output (y and its batch stride)
  const bool vec = (Wo % 4) == 0 && ((uintptr_t)y % 16) == 0 && (y_bstride % 4) == 0;
  const int ac = align_corners ? 1 : 0;
  const long long cells = (long long)Ho * (vec ? Wo / 4 : Wo);
  const int threads = 256;
  // ~8 cells per thread: a workgroup covers 2048 cells (8 KB written with quads)
  const int gx = (int)((cells + threads * 8 - 1) / (threads * 8));
  dim3 grid(gx, B * C * Do);
  const float rd = axis_ratio(Di, Do, ac), rh = axis_ratio(Hi, Ho, ac), rw = axis_ratio(Wi, Wo, ac);
  // Separable kernel (16-byte outputs) when R output rows' W-lerped source rows fit 64 KB
  if (vec && g_resample_mode == 0) {
    for (int R = 16; R >= 2; R /= 2) {
      const int nrmax = staged_rows(Hi, Ho, ac, R, 0);  // exact (common.h)
      const size_t lds = (size_t)2 * nrmax * Wo * sizeof(float);
      if (lds > 65536) continue;
      dim3 g((Ho + R - 1) / R, B * C * Do);
      resample3d_sep_f32<<<g, threads, lds, as_stream(stream)>>>(
          (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo, rd, rh, rw, ac, R, nrmax,
          scale, shift, flags);
      return launch_status("lea_resample3d_trilinear");
    }
  }
  // Row-staged kernel when R output rows' sources fit 64 KB of LDS: R = 16 rows
  // (20 KB of output per workgroup at Wo = 320), fewer for wide rows.
  for (int R = 16; R >= 2 && g_resample_mode != 2; R /= 2) {
    const int nrmax = staged_rows(Hi, Ho, ac, R, 0);  // exact (common.h)
    const size_t lds = (size_t)2 * nrmax * Wi * sizeof(float);
    if (lds > 65536) continue;
    dim3 g((Ho + R - 1) / R, B * C * Do);
    if (vec)
      resample3d_rows_f32<true><<<g, threads, lds, as_stream(stream)>>>(
          (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo, rd, rh, rw, ac,
          R, nrmax, scale, shift, flags);
    else
      resample3d_rows_f32<false><<<g, threads, lds, as_stream(stream)>>>(
          (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo, rd, rh, rw, ac,
          R, nrmax, scale, shift, flags);
    return launch_status("lea_resample3d_trilinear");
  }
  if (vec)
    resample3d_f32<true><<<grid, threads, 0, as_stream(stream)>>>(
        (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo, rd, rh, rw, ac,
        scale, shift, flags);
  else
    resample3d_f32<false><<<grid, threads, 0, as_stream(stream)>>>(
        (const float*)x, x_bstride, (float*)y, y_bstride, C, Di, Hi, Wi, Do, Ho, Wo, rd, rh, rw, ac,
        scale, shift, flags);
  return launch_status("lea_resample3d_trilinear");
}
