// ConvBR3d (Conv3d k in {1,3}, stride 1, pad k/2, no bias -> folded BN -> ReLU
// [-> + residual]) as an implicit GEMM on the gfx950 fp32 matrix cores.
// Replaces models/operations_3d.py:31-47 for every ConvBR of the matching net
// (retrain/skip_model_3d.py) and, via LEA_RESIDUAL, the cell's pairwise sums
// (skip_model_3d.py:69).
//
// GEMM view (per batch b, output plane d):
//     Y[co][v] = sum_{ci, tap} Wt[co][ci][tap] * X[ci][v + off(tap)]
// M = cout (blocks of <= 64 per workgroup, 16-row MFMA tiles), N = voxels (16-wide runs along W,
// coalesced NCDHW), K = cin * k^3.  MFMA = v_mfma_f32_16x16x4_f32 (exact f32
// products, f32 accumulate):
//     A (lane l) = Wt[co = 16*mt + (l & 15)][k = l >> 4]
//     B (lane l) = X [k = l >> 4][v = 16*nt + (l & 15)]
//     D (lane l, reg r) = Y[co = 16*mt + 4*(l >> 4) + r][v = l & 15]
// so the epilogue stores 16 consecutive w per cout row (64-B segments).
//
// Workgroup = 4 waves = one output plane tile of TH x TW voxels and all couts.
// K is streamed in chunks of CIN_B input channels: per chunk the workgroup stages
//   * X: CIN_B x KS x (TH+KS-1) x (TW+KS-1) input halo block (zero padded at the
//     volume border = the conv's zero padding), and
//   * W: KS^3 x CIN_B x COPS weights (a linear copy of the pre-packed layout),
// into LDS, then every wave runs KS^3 * CIN_B/4 k-steps of MT x NT MFMAs whose
// operands are single ds_read_b32 at per-lane base + compile-time offset.
// LDS strides are chosen so each 32-lane read group hits 32 distinct banks
// (the two k-rows of a half-wave sit 16 banks apart).
#include "common.h"

namespace lea {

constexpr int kConvWaves = 4;
constexpr int kConvThreads = kConvWaves * kWave;

using f32x4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;

// Row stride of the staged weight block / packed weights, congruent 16 mod 32
// so lanes 0-15 and 16-31 of one ds_read_b32 fall on disjoint banks.
__host__ __device__ constexpr int cout_stride(int cop) { return (cop % 32 == 0) ? cop + 16 : cop; }
__host__ __device__ constexpr int round_16mod32(int n) {
  return (n % 32 <= 16) ? n + (16 - n % 32) : n + (48 - n % 32);
}

template <int KS, int MT>
struct PackCfg {
  static constexpr int KT = KS * KS * KS;
  static constexpr int CIN_B = (KS == 3) ? 4 : 32;
  static constexpr int COP = MT * 16;
  static constexpr int COPS = cout_stride(COP);
  static constexpr int CHUNK = KT * CIN_B * COPS;  // floats per K chunk
};

template <int KS, int MT, int NT, int TW>
struct ConvCfg : PackCfg<KS, MT> {
  using P = PackCfg<KS, MT>;
  static constexpr int PAD = KS / 2;
  static constexpr int NTILES = kConvWaves * NT;
  static constexpr int TPR = TW / 16;  // 16-voxel N tiles per row
  static constexpr int TH = NTILES / TPR;
  static_assert(NTILES % TPR == 0, "tile rows");
  static constexpr int RH = TH + KS - 1;
  static constexpr int RW = TW + KS - 1;
  static constexpr int PLANE = RH * RW;
  static constexpr int CIS = round_16mod32(KS * PLANE);  // LDS stride between input channels
  static constexpr int XS = P::CIN_B * CIS;
  static constexpr int WS = P::CHUNK;
  static constexpr int XELEMS = P::CIN_B * KS * PLANE;
};

template <int KS, int MT, int NT, int TW>
__global__ __launch_bounds__(kConvThreads, 2) void conv3d_f32_kernel(
    const float* __restrict__ x, long long xbs, const float* __restrict__ wp,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* res,
    long long rbs, float* y, long long ybs, int cin, int cout, int D, int H, int W, int tiles_w,
    int ncob, unsigned flags) {
  using C = ConvCfg<KS, MT, NT, TW>;
  constexpr int CIN_B = C::CIN_B;
  __shared__ __attribute__((aligned(16))) float smem[C::XS + C::WS];
  float* xs = smem;
  float* ws = smem + C::XS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tile = blockIdx.x;
  const int h0 = (tile / tiles_w) * C::TH;
  const int w0 = (tile % tiles_w) * TW;
  const int d0 = blockIdx.y;
  const int b = blockIdx.z / ncob;    // batch
  const int cob = blockIdx.z - b * ncob;  // block of COP output channels
  const int co0 = cob * C::COP;
  const int nchunks = (cin + CIN_B - 1) / CIN_B;
  wp += (long long)cob * nchunks * C::WS;
  const long long HW = (long long)H * W;
  const long long DHW = HW * D;
  const float* xb = x + (long long)b * xbs;

  const int kq = lane >> 4;  // k row of this lane inside an MFMA (0..3)
  const int n = lane & 15;   // voxel column / cout row inside a 16 tile

  int xoff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int g = wave * NT + j;
    xoff[j] = kq * C::CIS + (g / C::TPR) * C::RW + (g % C::TPR) * 16 + n;
  }
  const int woff = kq * C::COPS + n;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = ch * CIN_B;
    __syncthreads();  // previous chunk's reads are done
    {  // weights: linear 16-byte copy of the packed chunk
      const float4* src = reinterpret_cast<const float4*>(wp + (long long)ch * C::WS);
      float4* dst = reinterpret_cast<float4*>(ws);
#pragma unroll 4
      for (int i = tid; i < C::WS / 4; i += kConvThreads) dst[i] = src[i];
    }
    // input halo block, zero outside the volume (= conv zero padding)
#pragma unroll 4
    for (int i = tid; i < C::XELEMS; i += kConvThreads) {
      const int ci = i / (KS * C::PLANE);
      int rem = i - ci * (KS * C::PLANE);
      const int kd = rem / C::PLANE;
      rem -= kd * C::PLANE;
      const int rr = rem / C::RW;
      const int cc = rem - rr * C::RW;
      const int d = d0 + kd - C::PAD;
      const int h = h0 + rr - C::PAD;
      const int w = w0 + cc - C::PAD;
      float v = 0.f;
      if ((unsigned)d < (unsigned)D && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W &&
          c0 + ci < cin)
        v = xb[(long long)(c0 + ci) * DHW + (long long)d * HW + (long long)h * W + w];
      xs[ci * C::CIS + kd * C::PLANE + rr * C::RW + cc] = v;
    }
    __syncthreads();

#pragma unroll
    for (int s = 0; s < CIN_B / 4; ++s) {
#pragma unroll
      for (int kd = 0; kd < KS; ++kd) {
#pragma unroll
        for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            const int tap = (kd * KS + kh) * KS + kw;
            float a[MT], bv[NT];
#pragma unroll
            for (int m = 0; m < MT; ++m) a[m] = ws[woff + (tap * CIN_B + 4 * s) * C::COPS + m * 16];
#pragma unroll
            for (int j = 0; j < NT; ++j)
              bv[j] = xs[xoff[j] + 4 * s * C::CIS + kd * C::PLANE + kh * C::RW + kw];
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
              for (int j = 0; j < NT; ++j)
                acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bv[j], acc[m][j], 0, 0, 0);
          }
        }
      }
    }
  }

  // epilogue: folded BN affine, ReLU, residual, masked store
  const bool relu = flags & LEA_RELU;
  const bool resid = flags & LEA_RESIDUAL;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + m * 16 + kq * 4 + r;
      if (co >= cout) continue;
      const float sc = scale ? scale[co] : 1.f;
      const float sh = shift ? shift[co] : 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int g = wave * NT + j;
        const int h = h0 + g / C::TPR;
        const int w = w0 + (g % C::TPR) * 16 + n;
        if (h >= H || w >= W) continue;
        const long long o = (long long)co * DHW + (long long)d0 * HW + (long long)h * W + w;
        float v = acc[m][j][r] * sc + sh;
        if (relu) v = fmaxf(v, 0.f);
        if (resid) v += res[(long long)b * rbs + o];
        y[(long long)b * ybs + o] = v;
      }
    }
  }
}

// Packed layout: [ceil(cout/COP)][ceil(cin/CIN_B)][KS^3][CIN_B][COPS], zero outside (cin, cout).
template <int KS, int MT>
__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ packed,
                                    int cout, int cin, int nchunks, long long total) {
  using P = PackCfg<KS, MT>;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(i % P::COPS);
    long long r = i / P::COPS;
    const int cb = (int)(r % P::CIN_B);
    r /= P::CIN_B;
    const int tap = (int)(r % P::KT);
    r /= P::KT;
    const int ch = (int)(r % nchunks);
    const int co = (int)(r / nchunks) * P::COP + col;
    const int ci = ch * P::CIN_B + cb;
    float v = 0.f;
    if (col < P::COP && co < cout && ci < cin) v = w[((long long)co * cin + ci) * P::KT + tap];
    packed[i] = v;
  }
}

inline int mt_for(int cout) { return cout <= 16 ? 1 : (cout <= 32 ? 2 : 4); }

template <int KS, int MT>
size_t packed_floats_t(int cout, int cin) {
  using P = PackCfg<KS, MT>;
  return (size_t)((cout + P::COP - 1) / P::COP) * ((cin + P::CIN_B - 1) / P::CIN_B) * P::CHUNK;
}

size_t packed_floats(int cout, int cin, int k) {
  const int mt = mt_for(cout);
  if (k == 3)
    return mt == 1 ? packed_floats_t<3, 1>(cout, cin)
                   : mt == 2 ? packed_floats_t<3, 2>(cout, cin) : packed_floats_t<3, 4>(cout, cin);
  return mt == 1 ? packed_floats_t<1, 1>(cout, cin)
                 : mt == 2 ? packed_floats_t<1, 2>(cout, cin) : packed_floats_t<1, 4>(cout, cin);
}

template <int KS, int MT, int NT, int TW>
int launch_conv(const float* x, long long xbs, const float* wp, const float* scale,
                const float* shift, const float* res, long long rbs, float* y, long long ybs,
                int B, int cin, int cout, int D, int H, int W, unsigned flags, hipStream_t st) {
  using C = ConvCfg<KS, MT, NT, TW>;
  const int tiles_w = (W + TW - 1) / TW;
  const int tiles_h = (H + C::TH - 1) / C::TH;
  const long long nt = (long long)tiles_w * tiles_h;
  const int ncob = (cout + C::COP - 1) / C::COP;
  LEA_CHECK_ARG(nt < (1LL << 31) && D <= 65535 && (long long)B * ncob <= 65535,
                "lea_conv3d_bnrelu: grid too large");
  dim3 grid((unsigned)nt, D, B * ncob);
  conv3d_f32_kernel<KS, MT, NT, TW><<<grid, kConvThreads, 0, st>>>(
      x, xbs, wp, scale, shift, res, rbs, y, ybs, cin, cout, D, H, W, tiles_w, ncob, flags);
  return launch_status("lea_conv3d_bnrelu");
}

// Pick the tile width with the least padding waste along W (ties -> wider).
inline bool prefer_tw64(int W) {
  const int w64 = (W + 63) / 64 * 64, w32 = (W + 31) / 32 * 32;
  return (w64 - W) <= (w32 - W) || W >= 1024;
}

template <int MT, int NT>
int dispatch_k3(const float* x, long long xbs, const float* wp, const float* scale,
                const float* shift, const float* res, long long rbs, float* y, long long ybs,
                int B, int cin, int cout, int D, int H, int W, unsigned flags, hipStream_t st) {
  if (prefer_tw64(W))
    return launch_conv<3, MT, NT, 64>(x, xbs, wp, scale, shift, res, rbs, y, ybs, B, cin, cout, D,
                                      H, W, flags, st);
  return launch_conv<3, MT, NT, 32>(x, xbs, wp, scale, shift, res, rbs, y, ybs, B, cin, cout, D, H,
                                    W, flags, st);
}

}  // namespace lea

extern "C" const char* lea_conv3d_kernel_name(int cout, int cin, int D, int H, int W, int k) {
  (void)cin;
  (void)D;
  (void)H;
  if (cout <= 0 || (k != 1 && k != 3) || W <= 0) return nullptr;
  const int mt = lea::mt_for(cout);
  if (k == 1)
    return mt == 1 ? "conv3d_f32_kernel<1, 1, 8, 512>" : mt == 2 ? "conv3d_f32_kernel<1, 2, 4, 256>"
                                                               : "conv3d_f32_kernel<1, 4, 4, 256>";
  const bool w64 = lea::prefer_tw64(W);
  if (mt == 1) return w64 ? "conv3d_f32_kernel<3, 1, 8, 64>" : "conv3d_f32_kernel<3, 1, 8, 32>";
  if (mt == 2) return w64 ? "conv3d_f32_kernel<3, 2, 4, 64>" : "conv3d_f32_kernel<3, 2, 4, 32>";
  return w64 ? "conv3d_f32_kernel<3, 4, 4, 64>" : "conv3d_f32_kernel<3, 4, 4, 32>";
}

extern "C" size_t lea_conv3d_packed_floats(int cout, int cin, int k) {
  if (cout <= 0 || cin <= 0 || (k != 1 && k != 3)) return 0;
  return lea::packed_floats(cout, cin, k);
}

extern "C" int lea_conv3d_pack_weights(const float* w, float* packed, int cout, int cin, int k,
                                       void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(w && packed, "lea_conv3d_pack_weights: null pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0 && (k == 1 || k == 3),
                "lea_conv3d_pack_weights: unsupported shape cout=%d cin=%d k=%d", cout, cin, k);
  const long long total = (long long)packed_floats(cout, cin, k);
  const int threads = 256;
  const int grid = (int)((total + threads - 1) / threads < 4096 ? (total + threads - 1) / threads : 4096);
  const int mt = mt_for(cout);
  hipStream_t st = as_stream(stream);
  const int nchunks = (cin + (k == 3 ? PackCfg<3, 1>::CIN_B : PackCfg<1, 1>::CIN_B) - 1) /
                      (k == 3 ? PackCfg<3, 1>::CIN_B : PackCfg<1, 1>::CIN_B);
#define LEA_PACK(KS, MT) \
  pack_weights_kernel<KS, MT><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total)
  if (k == 3) {
    if (mt == 1) LEA_PACK(3, 1); else if (mt == 2) LEA_PACK(3, 2); else LEA_PACK(3, 4);
  } else {
    if (mt == 1) LEA_PACK(1, 1); else if (mt == 2) LEA_PACK(1, 2); else LEA_PACK(1, 4);
  }
#undef LEA_PACK
  return launch_status("lea_conv3d_pack_weights");
}

extern "C" int lea_conv3d_bnrelu(const void* x, int64_t x_bstride, const float* w_packed,
                                 const float* scale, const float* shift, const void* residual,
                                 int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                 int cout, int D, int H, int W, int k, unsigned flags, int dtype,
                                 void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(x && w_packed && y, "lea_conv3d_bnrelu: null pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr), "lea_conv3d_bnrelu: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(!(flags & LEA_RESIDUAL) || residual, "lea_conv3d_bnrelu: LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && D > 0 && H > 0 && W > 0,
                "lea_conv3d_bnrelu: bad shape B=%d cin=%d cout=%d D=%d H=%d W=%d", B, cin, cout, D,
                H, W);
  LEA_CHECK_ARG(k == 1 || k == 3, "lea_conv3d_bnrelu: k=%d unsupported", k);
  if (dtype != LEA_F32) {
    set_error("lea_conv3d_bnrelu: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  // x must not alias y (the halo of other tiles would be overwritten mid-flight)
  LEA_CHECK_ARG(x != y, "lea_conv3d_bnrelu: x aliases y");
  const float* xf = (const float*)x;
  const float* rf = (const float*)residual;
  float* yf = (float*)y;
  hipStream_t st = as_stream(stream);
  const int mt = mt_for(cout);
  if (k == 3) {
    if (mt == 1) return dispatch_k3<1, 8>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, D, H, W, flags, st);
    if (mt == 2) return dispatch_k3<2, 4>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, D, H, W, flags, st);
    return dispatch_k3<4, 4>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, D, H, W, flags, st);
  }
  // 1x1x1: the volume is a flat run of D*H*W voxels (no halo)
  const long long dhw = (long long)D * H * W;
  LEA_CHECK_ARG(dhw < (1LL << 31), "lea_conv3d_bnrelu: volume too large");
  if (mt == 1) return launch_conv<1, 1, 8, 512>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, 1, 1, (int)dhw, flags, st);
  if (mt == 2) return launch_conv<1, 2, 4, 256>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, 1, 1, (int)dhw, flags, st);
  return launch_conv<1, 4, 4, 256>(xf, x_bstride, w_packed, scale, shift, rf, r_bstride, yf, y_bstride, B, cin, cout, 1, 1, (int)dhw, flags, st);
}
