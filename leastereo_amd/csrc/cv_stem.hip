// Matching-net stem0 over the cost volume, factored through 2D maps.
// Replaces retrain/LEAStereo.py:34-48 (the cost volume) + skip_model_3d.py:141
// (stem0 = ConvBR3d 3x3x3, 2C -> cout) without materialising the volume or running
// a 3D convolution over it.
//
// The cost volume is a stack of shifted copies of two 2D maps:
//   X[c,   i, h, x] = L[c, h, x]         for x >= i   (0 for x < i)
//   X[C+c, i, h, x] = R[c, h, x - i]     for x >= i
// so with u = w - d the conv's two halves collapse onto 2D convolutions:
//   left : sum_{kd valid} LK[kd][t](h, w),  t = max(kd - u, 0)  (0 if kd - u >= 3)
//          LK[kd][t] = 2D 3x3 conv of L with W_L[:, :, kd, :, kw >= t]  (the taps
//          whose cost-volume column x = w + kw - 1 passes the x >= i mask);
//   right: sum_{kd valid} B[kd](h, u - kd + 1)
//          B[kd] = 2D 3x3 conv of R with W_R[:, :, kd]  (the R index of every tap,
//          (w + kw - 1) - (d + kd - 1), depends on u only; the mask is R's own zero
//          padding at negative indices); at z = -1, B[kd] = K2[kd](h, 0), where
//          K2[kd] is the kw = 2 column alone; the last column w = W - 1 drops the
//          taps past the volume's right edge: - K2[kd](h, u - kd + 2);
// "kd valid" is the D padding: 0 <= d + kd - 1 < D.  The maps (9 + 6 per cout, built
// by lea_conv2d_bnrelu[_bf16] with the weights of lea_cv_stem_split_weights) cost
// 15 x 9 x 2 C taps per pixel instead of 27 x 2 C per voxel (D = 64: ~12x fewer
// FLOPs); this kernel is the rest -- per voxel two reads, BN, ReLU and the write of
// stem0's output, which bounds it (HBM).  Equal to the direct conv up to the fp32
// summation order.
#include "common.h"

namespace lea {
namespace cvs {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
constexpr int kThreads = 256;
constexpr int WS = 64;  // output columns per workgroup

struct Args {
  const void* lk;  // [B][9 cout][H][W]: channel (3 kd + t) cout + o
  long long lbs;
  const void* rk;  // [B][6 cout][H][W]: B[kd] at kd cout + o, K2[kd] at (3 + kd) cout + o
  long long rbs;
  const float* scale;
  const float* shift;
  void* y;         // [B][cout][D][H][W]
  long long ybs;
  int cout, D, H, W, nseg, ncob;
  unsigned flags;
};

// LDS right-half sums for the workgroup's u range [w0 - D + 1, w0 + WS - 1]:
// variant 0 = all kd (interior planes), 1 = kd in {1, 2} (d = 0), 2 = kd in {0, 1}
// (d = D - 1)
template <typename Load>
__device__ __forceinline__ void right_sums(Load bz, int u, float out[3]) {
  const float b0 = bz(0, u + 1), b1 = bz(1, u), b2 = bz(2, u - 1);
  out[0] = b0 + b1 + b2;
  out[1] = b1 + b2;
  out[2] = b0 + b1;
}

// left half at (d, u) from the lane's nine LK values
__device__ __forceinline__ float left_sum(const float lk[3][3], int d, int u, int D) {
  float s = 0.f;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int p = d + kd - 1;
    const int t = kd - u;
    const float v = t <= 0 ? lk[kd][0] : (t == 1 ? lk[kd][1] : (t == 2 ? lk[kd][2] : 0.f));
    if (p >= 0 && p < D) s += v;
  }
  return s;
}

// ---- f32 NCDHW: a workgroup = (batch, 16 couts, row h, 64 columns) walking all D
// planes; thread = (cout, 4 columns): one float4 store per plane
constexpr int OB = 16;

__global__ __launch_bounds__(kThreads) void cv_stem_f32_kernel(const Args a) {
  extern __shared__ float rs[];  // [3][OB][NU]
  const int D = a.D, H = a.H, W = a.W, NU = D + WS - 1;
  int blk = blockIdx.x;
  const int seg = blk % a.nseg;
  blk /= a.nseg;
  const int h = blk % H;
  blk /= H;
  const int cob = blk % a.ncob, b = blk / a.ncob;
  const int w0 = seg * WS, u0 = w0 - (D - 1);
  const long long HW = (long long)H * W;
  const float* lk = static_cast<const float*>(a.lk) + b * a.lbs;
  const float* rk = static_cast<const float*>(a.rk) + b * a.rbs;

  for (int e = threadIdx.x; e < OB * NU; e += kThreads) {
    const int ol = e / NU, iu = e % NU, o = cob * OB + ol;
    float r[3] = {0.f, 0.f, 0.f};
    if (o < a.cout) {
      auto bz = [&](int kd, int z) -> float {
        if (z >= 0 && z < W) return rk[(long long)(kd * a.cout + o) * HW + (long long)h * W + z];
        if (z == -1) return rk[(long long)((3 + kd) * a.cout + o) * HW + (long long)h * W];
        return 0.f;
      };
      right_sums(bz, u0 + iu, r);
    }
#pragma unroll
    for (int v = 0; v < 3; ++v) rs[(v * OB + ol) * NU + iu] = r[v];
  }
  __syncthreads();

  const int ol = threadIdx.x >> 4, o = cob * OB + ol;
  const int w = w0 + 4 * (threadIdx.x & 15);
  if (o >= a.cout || w >= W) return;  // W % 4 == 0 (host)
  float lkv[3][3][4];
#pragma unroll
  for (int kd = 0; kd < 3; ++kd)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const float4 v = *reinterpret_cast<const float4*>(lk + (long long)((3 * kd + t) * a.cout + o) * HW +
                                                        (long long)h * W + w);
      lkv[kd][t][0] = v.x;
      lkv[kd][t][1] = v.y;
      lkv[kd][t][2] = v.z;
      lkv[kd][t][3] = v.w;
    }
  float gl[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) gl[j] = lkv[0][0][j] + lkv[1][0][j] + lkv[2][0][j];
  const float sc = a.scale ? a.scale[o] : 1.f, sh = a.scale ? a.shift[o] : 0.f;
  const bool relu = a.flags & LEA_RELU;
  const float* r0 = rs + (0 * OB + ol) * NU;
  float* yp = static_cast<float*>(a.y) + b * a.ybs + (long long)o * D * HW + (long long)h * W + w;
  // this lane's columns avoid the band u < 2 for d <= w - 2, and the edge column W - 1
  const int dfast = min(w - 2, D - 2);
  const bool edge = w + 3 == W - 1;
  for (int d = 0; d < D; ++d) {
    const int iu = w - d - u0;
    float pre[4];
    if (d >= 1 && d <= dfast && !edge) {
#pragma unroll
      for (int j = 0; j < 4; ++j) pre[j] = gl[j] + r0[iu + j];
    } else {
      const float* rv = rs + ((d == 0 ? 1 : (d == D - 1 ? 2 : 0)) * OB + ol) * NU;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float l3[3][3];
#pragma unroll
        for (int kd = 0; kd < 3; ++kd)
#pragma unroll
          for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
        float rr = rv[iu + j];
        if (w + j == W - 1) {  // taps past the volume's right edge (kw = 2)
#pragma unroll
          for (int kd = 0; kd < 3; ++kd) {
            const int p = d + kd - 1, x = w + j - d - kd + 2;
            if (p >= 0 && p < D && x >= 0 && x < W)
              rr -= rk[(long long)((3 + kd) * a.cout + o) * HW + (long long)h * W + x];
          }
        }
        pre[j] = left_sum(l3, d, w + j - d, D) + rr;
      }
    }
    float4 out;
    float* po = reinterpret_cast<float*>(&out);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = pre[j] * sc + sh;
      po[j] = relu ? fmaxf(v, 0.f) : v;
    }
    *reinterpret_cast<float4*>(yp + (long long)d * HW) = out;
  }
}

// ---- bf16 c8: maps and output in the c8 layout ([B][C/8][D][H][W][8]); workgroup =
// (batch, 32 couts, row h, 64 columns), thread = (8-cout block, column): one 16-byte
// word per plane.  LDS sums [3][4 blocks][2 halves][NU][4] f32: a wave reads one
// block's half at consecutive u, 16 B per lane (conflict-free ds_read_b128).
constexpr int OB8 = 32;

__global__ __launch_bounds__(kThreads) void cv_stem_c8_kernel(const Args a) {
  extern __shared__ __attribute__((aligned(16))) float rs8[];  // [3][OB8 / 8][2][NU][4]
  const int D = a.D, H = a.H, W = a.W, NU = D + WS - 1;
  int blk = blockIdx.x;
  const int seg = blk % a.nseg;
  blk /= a.nseg;
  const int h = blk % H;
  blk /= H;
  const int cob = blk % a.ncob, b = blk / a.ncob;
  const int w0 = seg * WS, u0 = w0 - (D - 1);
  const long long HW = (long long)H * W;
  const __bf16* lk = static_cast<const __bf16*>(a.lk) + b * a.lbs;
  const __bf16* rk = static_cast<const __bf16*>(a.rk) + b * a.rbs;
  // word of channel block cb at (h, x)
  auto word = [&](const __bf16* m, int cb, int x) {
    return *reinterpret_cast<const bf16x8*>(m + ((long long)cb * HW + (long long)h * W + x) * 8);
  };
  const int cbo = a.cout / 8;  // channel blocks per map

  // staging: element = (iu, block of 8 couts); 8 channels per element
  for (int e = threadIdx.x; e < NU * (OB8 / 8); e += kThreads) {
    const int iu = e / (OB8 / 8), lb = e % (OB8 / 8);
    const int cb = cob * (OB8 / 8) + lb;
    float r[3][8];
#pragma unroll
    for (int v = 0; v < 3; ++v)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[v][j] = 0.f;
    if (cb < cbo) {
      float bzv[3][8];
      const int u = u0 + iu;
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const int z = u - kd + 1;
        bf16x8 q;
        bool has = true;
        if (z >= 0 && z < W) q = word(rk, kd * cbo + cb, z);
        else if (z == -1) q = word(rk, (3 + kd) * cbo + cb, 0);
        else has = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) bzv[kd][j] = has ? (float)q[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float b0 = bzv[0][j], b1 = bzv[1][j], b2 = bzv[2][j];
        r[0][j] = b0 + b1 + b2;
        r[1][j] = b1 + b2;
        r[2][j] = b0 + b1;
      }
    }
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      float4* dst = reinterpret_cast<float4*>(rs8) + ((v * (OB8 / 8) + lb) * 2) * NU + iu;
      dst[0] = make_float4(r[v][0], r[v][1], r[v][2], r[v][3]);
      dst[NU] = make_float4(r[v][4], r[v][5], r[v][6], r[v][7]);
    }
  }
  __syncthreads();

  const int lb = threadIdx.x >> 6, cb = cob * (OB8 / 8) + lb;
  const int w = w0 + (threadIdx.x & 63);
  if (cb >= cbo || w >= W) return;
  float lkv[3][3][8];
#pragma unroll
  for (int kd = 0; kd < 3; ++kd)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const bf16x8 q = word(lk, (3 * kd + t) * cbo + cb, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) lkv[kd][t][j] = (float)q[j];
    }
  float gl[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gl[j] = lkv[0][0][j] + lkv[1][0][j] + lkv[2][0][j];
    sc[j] = a.scale ? a.scale[cb * 8 + j] : 1.f;
    sh[j] = a.scale ? a.shift[cb * 8 + j] : 0.f;
  }
  const bool relu = a.flags & LEA_RELU;
  bf16x8* yp = reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.y) + b * a.ybs) +
               (long long)cb * D * HW + (long long)h * W + w;
  const bool edge = w == W - 1;
  for (int d = 0; d < D; ++d) {
    const int iu = w - d - u0, u = w - d;
    const int v = d == 0 ? 1 : (d == D - 1 ? 2 : 0);
    const float4* rp = reinterpret_cast<const float4*>(rs8) + ((v * (OB8 / 8) + lb) * 2) * NU + iu;
    const float4 ra = rp[0], rb = rp[NU];
    float pre[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    if (v == 0 && u >= 2 && !edge) {
#pragma unroll
      for (int j = 0; j < 8; ++j) pre[j] += gl[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float l3[3][3];
#pragma unroll
        for (int kd = 0; kd < 3; ++kd)
#pragma unroll
          for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
        pre[j] += left_sum(l3, d, u, D);
      }
      if (edge) {
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          const int p = d + kd - 1, x = u - kd + 2;
          if (p >= 0 && p < D && x >= 0 && x < W) {
            const bf16x8 q = word(rk, (3 + kd) * cbo + cb, x);
#pragma unroll
            for (int j = 0; j < 8; ++j) pre[j] -= (float)q[j];
          }
        }
      }
    }
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = pre[j] * sc[j] + sh[j];
      out[j] = (__bf16)(relu ? fmaxf(t, 0.f) : t);
    }
    yp[(long long)d * HW] = out;
  }
}

// stem0 weight [cout][2C][3][3][3] -> the 2D map weights
//   wl[(3 kd + t) cout + o][c][kh][kw] = W[o][c][kd][kh][kw] for kw >= t, else 0
//   wr[kd cout + o][c][kh][kw]        = W[o][C + c][kd][kh][kw]
//   wr[(3 + kd) cout + o][c][kh][kw]  = W[o][C + c][kd][kh][2] at kw = 1, else 0
__global__ void split_weights_kernel(const float* __restrict__ w, float* __restrict__ wl,
                                     float* __restrict__ wr, int cout, int C) {
  const long long nl = 9LL * cout * C * 9, nr = 6LL * cout * C * 9;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nl + nr;
       i += (long long)gridDim.x * blockDim.x) {
    const bool left = i < nl;
    long long r = left ? i : i - nl;
    const int kw = (int)(r % 3);
    r /= 3;
    const int kh = (int)(r % 3);
    r /= 3;
    const int c = (int)(r % C);
    r /= C;
    const int o = (int)(r % cout);
    const int m = (int)(r / cout);
    auto W = [&](int ci, int kd, int khh, int kww) {
      return w[((((long long)o * 2 * C + ci) * 3 + kd) * 3 + khh) * 3 + kww];
    };
    if (left) {
      const int kd = m / 3, t = m % 3;
      wl[i] = kw >= t ? W(c, kd, kh, kw) : 0.f;
    } else if (m < 3) {
      wr[i - nl] = W(C + c, m, kh, kw);
    } else {
      wr[i - nl] = kw == 1 ? W(C + c, m - 3, kh, 2) : 0.f;
    }
  }
}

}  // namespace cvs
}  // namespace lea

using namespace lea;

extern "C" int lea_cv_stem_split_weights(const float* w, float* wl, float* wr, int cout, int C,
                                         void* stream) {
  clear_error();
  LEA_CHECK_ARG(w && wl && wr, "lea_cv_stem_split_weights: null pointer");
  LEA_CHECK_ARG(cout > 0 && C > 0, "lea_cv_stem_split_weights: bad shape cout=%d C=%d", cout, C);
  const long long total = 15LL * cout * C * 9;
  const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
  cvs::split_weights_kernel<<<grid, 256, 0, as_stream(stream)>>>(w, wl, wr, cout, C);
  return launch_status("lea_cv_stem_split_weights");
}

extern "C" int lea_cv_stem_combine(const void* lmaps, int64_t l_bstride, const void* rmaps,
                                   int64_t r_bstride, const float* scale, const float* shift,
                                   void* y, int64_t y_bstride, int B, int cout, int D3, int H, int W,
                                   unsigned flags, int dtype, void* stream) {
  clear_error();
  LEA_CHECK_ARG(lmaps && rmaps && y, "lea_cv_stem_combine: null pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_cv_stem_combine: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && cout > 0 && D3 >= 2 && H > 0 && W > 0,
                "lea_cv_stem_combine: bad shape B=%d cout=%d D3=%d H=%d W=%d", B, cout, D3, H, W);
  LEA_CHECK_ARG(dtype == LEA_F32 || dtype == LEA_BF16, "lea_cv_stem_combine: dtype %d", dtype);
  LEA_CHECK_ARG(dtype != LEA_F32 || W % 4 == 0, "lea_cv_stem_combine: f32 needs W %% 4 == 0 (W=%d)", W);
  LEA_CHECK_ARG(dtype != LEA_BF16 || cout % 8 == 0, "lea_cv_stem_combine: bf16 needs cout %% 8 == 0");
  LEA_CHECK_ARG((long long)cout * D3 * H * W < (1LL << 40), "lea_cv_stem_combine: volume too large");
  cvs::Args a{};
  a.lk = lmaps;
  a.lbs = l_bstride;
  a.rk = rmaps;
  a.rbs = r_bstride;
  a.scale = scale;
  a.shift = shift;
  a.y = y;
  a.ybs = y_bstride;
  a.cout = cout;
  a.D = D3;
  a.H = H;
  a.W = W;
  a.flags = flags & LEA_RELU;
  a.nseg = (W + cvs::WS - 1) / cvs::WS;
  const int ob = dtype == LEA_F32 ? cvs::OB : cvs::OB8;
  a.ncob = (cout + ob - 1) / ob;
  const long long nblk = (long long)B * a.ncob * H * a.nseg;
  LEA_CHECK_ARG(nblk < (1LL << 31), "lea_cv_stem_combine: grid too large");
  const size_t lds = (size_t)3 * ob * (D3 + cvs::WS - 1) * sizeof(float);
  LEA_CHECK_ARG(lds <= 160 * 1024, "lea_cv_stem_combine: D3=%d too deep for LDS", D3);
  if (dtype == LEA_F32)
    cvs::cv_stem_f32_kernel<<<dim3((unsigned)nblk), cvs::kThreads, lds, as_stream(stream)>>>(a);
  else
    cvs::cv_stem_c8_kernel<<<dim3((unsigned)nblk), cvs::kThreads, lds, as_stream(stream)>>>(a);
  return launch_status("lea_cv_stem_combine");
}
