// Feature-net stems 0 and 1 fused: ConvBR2d 3x3 s1 (3 -> C0) then ConvBR2d 3x3 s3
// (C0 -> C1).  Replaces retrain/new_model_2d.py:93-94 (stem0, stem1 of newFeature;
// models/operations_2d.py:31-47) without writing stem0's full-resolution output.
//
// Stride 3 with a 3x3 kernel tiles stem0's output without overlap: stem1 pixel (ho, wo)
// reads stem0 at rows 3ho-1..3ho+1, columns 3wo-1..3wo+1, and every stem0 pixel feeds
// exactly one stem1 pixel.  So a thread computes its nine stem0 pixels (each a 27-tap
// dot product over a 5x5x3 image patch, folded BN, ReLU; zero where the pixel lies in
// stem1's padding) channel by channel and accumulates them straight into its C1 stem1
// outputs: no stem0 pixel is computed twice and its 16 x 4 B per pixel never reach HBM
// (70 MB per stereo pair at 576x960).  A workgroup stages its image patch and the weights
// (c0-major) in LDS with coalesced loads, all in flight at once; the weights are read as
// wave-uniform LDS broadcasts.
#include "common.h"

namespace lea {
namespace fstem {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int TW = 64, TH = 4;                       // stem1 outputs per workgroup
constexpr int PW = 3 * TW + 2, PH = 3 * TH + 2;      // image patch (input rows/cols 3ho-2 ..)

template <int CIN, int C0, int C1, bool C8>
__global__ __launch_bounds__(TW * TH) void feature_stem_kernel(
    const float* __restrict__ x, long long xbs, const float* __restrict__ w0, const float* __restrict__ sc0,
    const float* __restrict__ sh0, const float* __restrict__ w1, const float* __restrict__ sc1,
    const float* __restrict__ sh1, void* __restrict__ y, long long ybs, int Hi, int Wi, int Ho, int Wo) {
  static_assert(C1 % 2 == 0, "stem1's packed FMAs read w1s as float2 pairs of couts");
  __shared__ float patch[CIN][PH][PW];
  // the weights, c0-major, staged once (r04; read as wave-uniform scalar loads, each c0
  // iteration waited on ~70 of them): w0s[c0][c][3][3] as given, w1s[c0][tap][cout]
  // (r05: cout innermost, so stem1's packed f32x2 FMAs read two couts per LDS word)
  __shared__ __attribute__((aligned(16))) float w0s[C0 * CIN * 9 + 1];
  __shared__ __attribute__((aligned(16))) float w1s[C0 * C1 * 9];
  __shared__ float bn0[2][C0];  // stem0's folded BN (scale, shift)
  const int b = blockIdx.z;
  const int ho0 = blockIdx.y * TH, wo0 = blockIdx.x * TW;
  const int hi0 = 3 * ho0 - 2, wi0 = 3 * wo0 - 2;
  const float* xb = x + (long long)b * xbs;
  const long long HWi = (long long)Hi * Wi;
  {
    // every load of the patch in flight before the first LDS write (r04: the rolled loop
    // waited for each of its 32 loads in turn); branch-free, clamped in-range addresses
    constexpr int N = CIN * PH * PW, NST = (N + TW * TH - 1) / (TW * TH);
    float v[NST];
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const int e = min((int)threadIdx.x + k * TW * TH, N - 1);
      const int c = e / (PH * PW), r = (e / PW) % PH, q = e % PW;
      const int h = hi0 + r, w = wi0 + q;
      const bool ok = (unsigned)h < (unsigned)Hi && (unsigned)w < (unsigned)Wi;
      const float t = xb[(long long)c * HWi + (long long)min(max(h, 0), Hi - 1) * Wi + min(max(w, 0), Wi - 1)];
      v[k] = ok ? t : 0.f;
    }
    constexpr int N0 = C0 * CIN * 9, N1 = C0 * C1 * 9;
    constexpr int NW = (N0 + N1 + TW * TH - 1) / (TW * TH);
    float wv[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int e = min((int)threadIdx.x + k * TW * TH, N0 + N1 - 1);
      if (e < N0) {
        wv[k] = w0[e];
      } else {  // w1s index (c0, t, o) <- w1[(o * C0 + c0) * 9 + t]
        const int f = e - N0, c0 = f / (C1 * 9), t = (f / C1) % 9, o = f % C1;
        wv[k] = w1[(o * C0 + c0) * 9 + t];
      }
    }
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const int e = (int)threadIdx.x + k * TW * TH;
      if (e < N) (&patch[0][0][0])[e] = v[k];
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int e = (int)threadIdx.x + k * TW * TH;
      if (e < N0) w0s[e] = wv[k];
      else if (e < N0 + N1) w1s[e - N0] = wv[k];
    }
    if (threadIdx.x < 2 * C0) {
      const int c0 = threadIdx.x % C0;
      bn0[threadIdx.x / C0][c0] = sc0 ? (threadIdx.x < C0 ? sc0[c0] : sh0[c0]) : (threadIdx.x < C0 ? 1.f : 0.f);
    }
  }
  __syncthreads();
  const int tx = threadIdx.x % TW, ty = threadIdx.x / TW;
  const int ho = ho0 + ty, wo = wo0 + tx;
  // the 5x5xCIN patch of this output (rows 3ty .. 3ty+4, cols 3tx .. 3tx+4 of the tile's)
  float in[CIN][5][5];
#pragma unroll
  for (int c = 0; c < CIN; ++c)
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int q = 0; q < 5; ++q) in[c][r][q] = patch[c][3 * ty + r][3 * tx + q];
  // stem0 pixel (kh, kw) of this output: image row 3ho - 1 + kh, column 3wo - 1 + kw
  bool valid[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      valid[kh][kw] = (unsigned)(3 * ho - 1 + kh) < (unsigned)Hi && (unsigned)(3 * wo - 1 + kw) < (unsigned)Wi;
  // stem1 on packed f32 FMAs (r05): two couts per v_pk_fma_f32 (same stem0 value; w1s is
  // [c0][tap][cout], so a cout pair is one 8-byte LDS word) -- each element sees the scalar
  // form's fmaf sequence: identical bits (stem0 stays scalar: pairing its pixels or channels
  // needs the input values broadcast into register pairs -- 256 VGPRs)
  f32x2 acc[C1 / 2];
#pragma unroll
  for (int o = 0; o < C1 / 2; ++o) acc[o] = f32x2{0.f, 0.f};
  for (int c0 = 0; c0 < C0; ++c0) {
    const float s0 = bn0[0][c0], t0 = bn0[1][c0];
    float s[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < CIN; ++c)
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) v = fmaf(w0s[((c0 * CIN + c) * 3 + i) * 3 + j], in[c][kh + i][kw + j], v);
        v = fmaxf(v * s0 + t0, 0.f);  // stem0's BN + ReLU (new_model_2d.py:93)
        s[kh * 3 + kw] = valid[kh][kw] ? v : 0.f;
      }
    const f32x2* w1p = reinterpret_cast<const f32x2*>(w1s + c0 * 9 * C1);
#pragma unroll
    for (int o = 0; o < C1 / 2; ++o)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[o] = __builtin_elementwise_fma(w1p[t * (C1 / 2) + o], f32x2{s[t], s[t]}, acc[o]);
  }
  if (ho >= Ho || wo >= Wo) return;
  const long long HWo = (long long)Ho * Wo, pix = (long long)ho * Wo + wo;
  float r[C1];
#pragma unroll
  for (int o = 0; o < C1; ++o) r[o] = fmaxf(acc[o / 2][o % 2] * (sc1 ? sc1[o] : 1.f) + (sc1 ? sh1[o] : 0.f), 0.f);
  if constexpr (C8) {  // bf16 c8: [B][C1/8][1][Ho][Wo][8]
    bf16x8* yp = reinterpret_cast<bf16x8*>(static_cast<__bf16*>(y) + (long long)b * ybs);
#pragma unroll
    for (int cb = 0; cb < C1 / 8; ++cb) {
      bf16x8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = (__bf16)r[cb * 8 + j];
      yp[cb * HWo + pix] = o8;
    }
  } else {
    float* yp = static_cast<float*>(y) + (long long)b * ybs;
#pragma unroll
    for (int o = 0; o < C1; ++o) yp[o * HWo + pix] = r[o];
  }
}

}  // namespace fstem
}  // namespace lea

using namespace lea;

extern "C" int lea_feature_stem_bnrelu(const float* x, int64_t x_bstride, const float* w0, const float* scale0,
                                       const float* shift0, const float* w1, const float* scale1,
                                       const float* shift1, void* y, int64_t y_bstride, int B, int cin, int c0,
                                       int c1, int Hi, int Wi, int dtype, void* stream) {
  clear_error();
  LEA_CHECK_ARG(x && w0 && w1 && y && (const void*)x != y, "lea_feature_stem_bnrelu: null or aliased pointer");
  LEA_CHECK_ARG((scale0 == nullptr) == (shift0 == nullptr) && (scale1 == nullptr) == (shift1 == nullptr),
                "lea_feature_stem_bnrelu: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && B <= 65535 && Hi > 0 && Wi > 0, "lea_feature_stem_bnrelu: bad shape");
  LEA_CHECK_ARG(dtype == LEA_F32 || dtype == LEA_BF16, "lea_feature_stem_bnrelu: dtype %d", dtype);
  if (!(cin == 3 && c0 == 16 && c1 == 32)) {
    set_error("lea_feature_stem_bnrelu: channels %d -> %d -> %d not instantiated (3 -> 16 -> 32)", cin, c0, c1);
    return LEA_E_UNSUPPORTED;
  }
  const int Ho = (Hi - 1) / 3 + 1, Wo = (Wi - 1) / 3 + 1;
  LEA_CHECK_ARG((Ho + fstem::TH - 1) / fstem::TH <= 65535, "lea_feature_stem_bnrelu: image too tall");
  const dim3 grid((Wo + fstem::TW - 1) / fstem::TW, (Ho + fstem::TH - 1) / fstem::TH, B);
  if (dtype == LEA_F32)
    fstem::feature_stem_kernel<3, 16, 32, false><<<grid, fstem::TW * fstem::TH, 0, as_stream(stream)>>>(
        x, x_bstride, w0, scale0, shift0, w1, scale1, shift1, y, y_bstride, Hi, Wi, Ho, Wo);
  else
    fstem::feature_stem_kernel<3, 16, 32, true><<<grid, fstem::TW * fstem::TH, 0, as_stream(stream)>>>(
        x, x_bstride, w0, scale0, shift0, w1, scale1, shift1, y, y_bstride, Hi, Wi, Ho, Wo);
  return launch_status("lea_feature_stem_bnrelu");
}
