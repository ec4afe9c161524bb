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
  int nds, dchunk;  // D split into nds runs of dchunk planes (one workgroup each)
  unsigned flags;
};

// one workgroup walks every plane unless the LDS sums do not fit: splitting D re-stages
// the right-half sums per run (r02: 16-plane runs read 2.3x more and ran 1.15-1.18x slower)
constexpr int kLdsBytes = 80 * 1024;

// Right-half sums staged in LDS per cout, NT = NU + 2 WS positions:
//   [0, NU)          interior planes (all kd), u = u0 + p
//   [NU, NU + WS)    d = 0 (kd in {1, 2}),     u = w0 + p - NU
//   [NU + WS, NT)    d = D - 1 (kd in {0, 1}), u = w0 + p - NU - WS - (D - 1)
// plus, for the segment holding the last column, per (cout, plane) the correction
// sum_{kd valid} K2[kd](h, W + 1 - d - kd).  Every staging load is unconditional at a
// clamped address with the selects after it, four elements per thread per batch, so
// a thread's loads are in flight together (r02: the branchy form waited for each).
__device__ __forceinline__ int stage_u(int p, int NU, int u0, int w0, int D) {
  return p < NU ? u0 + p : (p < NU + WS ? w0 + p - NU : w0 + p - NU - WS - (D - 1));
}
__device__ __forceinline__ float stage_sum(int p, int NU, const float bz[3]) {
  return p < NU ? bz[0] + bz[1] + bz[2] : (p < NU + WS ? bz[1] + bz[2] : bz[0] + bz[1]);
}
// z = u - kd + 1 of the B[kd] column (z = -1: K2[kd] at column 0; else out of range)
__device__ __forceinline__ long long bz_offset(int kd, int z, int o, int cout, long long HW, int W) {
  return (z >= 0 && z < W) ? (long long)(kd * cout + o) * HW + z : (long long)((3 + kd) * cout + o) * HW;
}
__device__ __forceinline__ bool bz_valid(int z, int W) { return z >= -1 && z < W; }
__device__ __forceinline__ bool plane_valid(int d, int kd, int D) {
  return d + kd - 1 >= 0 && d + kd - 1 < D;
}

// left half at (d, u) from the lane's nine LK values
__device__ __forceinline__ float left_sum(const float lk[3][3], int d, int u, int D) {
  float s = 0.f;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int t = kd - u;
    const float v = t <= 0 ? lk[kd][0] : (t == 1 ? lk[kd][1] : (t == 2 ? lk[kd][2] : 0.f));
    if (plane_valid(d, kd, D)) s += v;
  }
  return s;
}

struct Tile {
  int D, H, W, NU, NT, h, cob, b, d0, d1, w0, u0;
  long long HW;
};

__device__ __forceinline__ Tile tile_of(const Args& a) {
  Tile t;
  t.D = a.D;
  t.H = a.H;
  t.W = a.W;
  t.NU = a.dchunk + WS - 1;
  t.NT = t.NU + 2 * WS;
  int blk = blockIdx.x;
  const int seg = blk % a.nseg;
  blk /= a.nseg;
  const int ds = blk % a.nds;
  blk /= a.nds;
  t.h = blk % a.H;
  blk /= a.H;
  t.cob = blk % a.ncob;
  t.b = blk / a.ncob;
  // planes [d0, d1): u = w - d spans [w0 - d0 - dchunk + 1, w0 + WS - 1 - d0]
  t.d0 = ds * a.dchunk;
  t.d1 = min(a.D, t.d0 + a.dchunk);
  t.w0 = seg * WS;
  t.u0 = t.w0 - (t.d0 + a.dchunk - 1);
  t.HW = (long long)a.H * a.W;
  return t;
}

// ---- f32 NCDHW: a workgroup = (batch, 16 couts, row h, 64 columns) walking its planes;
// thread = (cout, 4 columns): one float4 store per plane
constexpr int OB = 16;

__global__ __launch_bounds__(kThreads) void cv_stem_f32_kernel(const Args a) {
  extern __shared__ float rs[];  // [OB][NT] sums, then [OB][dchunk] edge corrections
  const Tile T = tile_of(a);
  const int D = T.D, W = T.W, NU = T.NU, NT = T.NT, d0 = T.d0, d1 = T.d1, w0 = T.w0;
  const long long HW = T.HW;
  if (a.flags & 0x100u) {  // probe: stores only
    const int ol = threadIdx.x >> 4, o = T.cob * OB + ol, w = w0 + 4 * (threadIdx.x & 15);
    if (o >= a.cout || w >= W) return;
    float* yp = static_cast<float*>(a.y) + T.b * a.ybs + (long long)o * D * HW + (long long)T.h * W + w;
    for (int d = d0; d < d1; ++d) *reinterpret_cast<float4*>(yp + (long long)d * HW) = make_float4(d, 0.f, 0.f, 1.f);
    return;
  }
  const float* lk = static_cast<const float*>(a.lk) + T.b * a.lbs;
  const float* rkh = static_cast<const float*>(a.rk) + T.b * a.rbs + (long long)T.h * W;
  float* corr = rs + OB * NT;
  const int tid = threadIdx.x;

  const int NE = OB * NT;
  for (int e0 = 0; e0 < NE; e0 += 4 * kThreads) {
    float q[4][3];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = min(e0 + k * kThreads + tid, NE - 1);
      const int ol = e / NT, p = e % NT;
      const int o = min(T.cob * OB + ol, a.cout - 1), u = stage_u(p, NU, T.u0, w0, D);
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) q[k][kd] = rkh[bz_offset(kd, u - kd + 1, o, a.cout, HW, W)];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = e0 + k * kThreads + tid;
      if (e >= NE) break;
      const int ol = e / NT, p = e % NT;
      const bool ok = T.cob * OB + ol < a.cout;
      const int u = stage_u(p, NU, T.u0, w0, D);
      float bz[3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) bz[kd] = (ok && bz_valid(u - kd + 1, W)) ? q[k][kd] : 0.f;
      rs[e] = stage_sum(p, NU, bz);
    }
  }
  if (w0 + WS >= W) {  // the last column is in this segment
    const int dl = d1 - d0;
    for (int e = tid; e < OB * dl; e += kThreads) {
      const int ol = e / dl, d = d0 + e % dl;
      const int o = min(T.cob * OB + ol, a.cout - 1);
      float v[3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const int x = min(max(W + 1 - d - kd, 0), W - 1);
        v[kd] = rkh[(long long)((3 + kd) * a.cout + o) * HW + x];
      }
      float s = 0.f;
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const int x = W + 1 - d - kd;
        if (plane_valid(d, kd, D) && x >= 0 && x < W) s += v[kd];
      }
      corr[ol * a.dchunk + (d - d0)] = s;
    }
  }
  __syncthreads();

  const int ol = tid >> 4, o = T.cob * OB + ol;
  const int w = w0 + 4 * (tid & 15);
  if (o >= a.cout || w >= W) return;  // W % 4 == 0 (host)
  // the masked maps (t = 1, 2) only matter where some plane has u = w - d <= 1
  const bool band = w - (d1 - 1) <= 1;
  float lkv[3][3][4];
#pragma unroll
  for (int kd = 0; kd < 3; ++kd)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t == 0 || band)
        v = *reinterpret_cast<const float4*>(lk + (long long)((3 * kd + t) * a.cout + o) * HW +
                                             (long long)T.h * W + w);
      lkv[kd][t][0] = v.x;
      lkv[kd][t][1] = v.y;
      lkv[kd][t][2] = v.z;
      lkv[kd][t][3] = v.w;
    }
  const float sc = a.scale ? a.scale[o] : 1.f, sh = a.scale ? a.shift[o] : 0.f;
  const float lo = (a.flags & LEA_RELU) ? 0.f : -INFINITY;  // ReLU as a floor
  const float* r0 = rs + ol * NT;
  const float* cr = corr + ol * a.dchunk - d0;
  float* yp = static_cast<float*>(a.y) + T.b * a.ybs + (long long)o * D * HW + (long long)T.h * W + w;
  const int jedge = W - 1 - w;  // the lane's column that is the last one (0..3), if any
  auto store = [&](int d, const float pre[4]) {
    float4 out;
    float* po = reinterpret_cast<float*>(&out);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      po[j] = fmaxf(pre[j] * sc + sh, lo);
    }
    *reinterpret_cast<float4*>(yp + (long long)d * HW) = out;
  };
  // the first and last planes (kd = 0 resp. 2 out of range), whole workgroup at once
  auto boundary = [&](int d, int pbase) {
    float pre[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float l3[3][3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd)
#pragma unroll
        for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
      pre[j] = left_sum(l3, d, w + j - d, D) + r0[pbase + (w - w0) + j] - (j == jedge ? cr[d] : 0.f);
    }
    store(d, pre);
  };
  if (d0 == 0) boundary(0, NU);
  if (d1 == D) boundary(D - 1, NU + WS);
  // interior planes, branch-free: the left half is gl (u >= 2), one of the band values
  // bl[u + 2] (-2 <= u <= 1) or 0 (u <= -3)
  float gl[4], bl[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float l3[3][3];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
    gl[j] = lkv[0][0][j] + lkv[1][0][j] + lkv[2][0][j];
#pragma unroll
    for (int m = 0; m < 4; ++m) bl[m][j] = left_sum(l3, 1, m - 2, D);  // (d = 1: all kd valid)
  }
  const int da = max(d0, 1), db = min(d1, D - 1);
  if (w0 - (db - 1) >= 2) {  // every lane has u >= 2 on every interior plane here
    for (int d = da; d < db; ++d) {
      const int iu = w - d - T.u0;
      const float c = cr[d];
      float pre[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pre[j] = gl[j] + r0[iu + j] - (j == jedge ? c : 0.f);
      store(d, pre);
    }
    return;
  }
  for (int d = da; d < db; ++d) {
    const int iu = w - d - T.u0;
    const float c = cr[d];
    float pre[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int u = w + j - d;
      float l = u >= 2 ? gl[j] : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) l = u == m - 2 ? bl[m][j] : l;
      pre[j] = l + r0[iu + j] - (j == jedge ? c : 0.f);
    }
    store(d, pre);
  }
}

// ---- bf16 c8: maps and output in the c8 layout ([B][C/8][D][H][W][8]); workgroup =
// (batch, 32 couts, row h, 64 columns), thread = (8-cout block, column): one 16-byte
// word per plane.  LDS sums [4 blocks][2 halves][NT][4] f32 (a wave reads one block's
// half at consecutive u, 16 B per lane: conflict-free ds_read_b128), then the edge
// corrections [4][2][dchunk][4].
constexpr int OB8 = 32;

__global__ __launch_bounds__(kThreads) void cv_stem_c8_kernel(const Args a) {
  extern __shared__ __attribute__((aligned(16))) float rs8[];
  const Tile T = tile_of(a);
  const int D = T.D, W = T.W, NU = T.NU, NT = T.NT, d0 = T.d0, d1 = T.d1, w0 = T.w0;
  const long long HW = T.HW;
  if (a.flags & 0x100u) {  // probe: stores only
    const int lb = threadIdx.x >> 6, cb = T.cob * (OB8 / 8) + lb, w = w0 + (threadIdx.x & 63);
    if (cb >= a.cout / 8 || w >= W) return;
    bf16x8* yp = reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.y) + T.b * a.ybs) +
                 (long long)cb * D * HW + (long long)T.h * W + w;
    bf16x8 z = {};
    for (int d = d0; d < d1; ++d) yp[(long long)d * HW] = z;
    return;
  }
  const __bf16* lk = static_cast<const __bf16*>(a.lk) + T.b * a.lbs;
  const __bf16* rk = static_cast<const __bf16*>(a.rk) + T.b * a.rbs;
  const int cbo = a.cout / 8;  // channel blocks per map
  // word of channel block cb at (h, x)
  auto word = [&](const __bf16* m, int cb, int x) {
    return *reinterpret_cast<const bf16x8*>(m + ((long long)cb * HW + (long long)T.h * W + x) * 8);
  };
  float4* rs4 = reinterpret_cast<float4*>(rs8);
  float4* corr4 = rs4 + (OB8 / 8) * 2 * NT;
  const int tid = threadIdx.x;

  // staging: element = (block of 8 couts, position p); 8 channels per element
  const int NE = (OB8 / 8) * NT;
  for (int e0 = 0; e0 < NE; e0 += 2 * kThreads) {
    bf16x8 q[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = min(e0 + k * kThreads + tid, NE - 1);
      const int lb = e / NT, p = e % NT;
      const int cb = min(T.cob * (OB8 / 8) + lb, cbo - 1), u = stage_u(p, NU, T.u0, w0, D);
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const int z = u - kd + 1;
        q[k][kd] = (z >= 0 && z < W) ? word(rk, kd * cbo + cb, z) : word(rk, (3 + kd) * cbo + cb, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = e0 + k * kThreads + tid;
      if (e >= NE) break;
      const int lb = e / NT, p = e % NT;
      const bool ok = T.cob * (OB8 / 8) + lb < cbo;
      const int u = stage_u(p, NU, T.u0, w0, D);
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float bz[3];
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) bz[kd] = (ok && bz_valid(u - kd + 1, W)) ? (float)q[k][kd][j] : 0.f;
        r[j] = stage_sum(p, NU, bz);
      }
      rs4[(lb * 2) * NT + p] = make_float4(r[0], r[1], r[2], r[3]);
      rs4[(lb * 2 + 1) * NT + p] = make_float4(r[4], r[5], r[6], r[7]);
    }
  }
  if (w0 + WS >= W) {  // the last column is in this segment
    const int dl = d1 - d0;
    for (int e = tid; e < (OB8 / 8) * dl; e += kThreads) {
      const int lb = e / dl, d = d0 + e % dl;
      const int cb = min(T.cob * (OB8 / 8) + lb, cbo - 1);
      bf16x8 v[3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) v[kd] = word(rk, (3 + kd) * cbo + cb, min(max(W + 1 - d - kd, 0), W - 1));
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const int x = W + 1 - d - kd;
        if (plane_valid(d, kd, D) && x >= 0 && x < W)
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += (float)v[kd][j];
      }
      corr4[(lb * 2) * a.dchunk + (d - d0)] = make_float4(s[0], s[1], s[2], s[3]);
      corr4[(lb * 2 + 1) * a.dchunk + (d - d0)] = make_float4(s[4], s[5], s[6], s[7]);
    }
  }
  __syncthreads();

  const int lb = tid >> 6, cb = T.cob * (OB8 / 8) + lb;
  const int w = w0 + (tid & 63);
  if (cb >= cbo || w >= W) return;
  const bool band = w - (d1 - 1) <= 1;  // (as the f32 kernel)
  float lkv[3][3][8];
#pragma unroll
  for (int kd = 0; kd < 3; ++kd)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      bf16x8 q = {};
      if (t == 0 || band) q = word(lk, (3 * kd + t) * cbo + cb, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) lkv[kd][t][j] = (float)q[j];
    }
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = a.scale ? a.scale[cb * 8 + j] : 1.f;
    sh[j] = a.scale ? a.shift[cb * 8 + j] : 0.f;
  }
  const float lo = (a.flags & LEA_RELU) ? 0.f : -INFINITY;  // ReLU as a floor
  bf16x8* yp = reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.y) + T.b * a.ybs) +
               (long long)cb * D * HW + (long long)T.h * W + w;
  const bool edge = w == W - 1;  // the last column subtracts its corrections
  const float4* rl = rs4 + (lb * 2) * NT;
  const float4* cl = corr4 + (lb * 2) * a.dchunk - d0;
  auto store = [&](int d, const float pre[8]) {
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      out[j] = (__bf16)fmaxf(pre[j] * sc[j] + sh[j], lo);
    }
    yp[(long long)d * HW] = out;
  };
  // staged sum minus the edge correction (a select: the corrections are only staged
  // for the segment holding the last column)
  auto right = [&](int p, int d, float pre[8]) {
    const float4 ra = rl[p], rb = rl[NT + p];
    pre[0] = ra.x, pre[1] = ra.y, pre[2] = ra.z, pre[3] = ra.w;
    pre[4] = rb.x, pre[5] = rb.y, pre[6] = rb.z, pre[7] = rb.w;
    if (edge) {
      const float4 ca = cl[d], cc = cl[a.dchunk + d];
      pre[0] -= ca.x, pre[1] -= ca.y, pre[2] -= ca.z, pre[3] -= ca.w;
      pre[4] -= cc.x, pre[5] -= cc.y, pre[6] -= cc.z, pre[7] -= cc.w;
    }
  };
  // the first and last planes, whole workgroup at once
  auto boundary = [&](int d, int p) {
    float pre[8];
    right(p, d, pre);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float l3[3][3];
#pragma unroll
      for (int kd = 0; kd < 3; ++kd)
#pragma unroll
        for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
      pre[j] += left_sum(l3, d, w - d, D);
    }
    store(d, pre);
  };
  if (d0 == 0) boundary(0, NU + (w - w0));
  if (d1 == D) boundary(D - 1, NU + WS + (w - w0));
  // interior planes, branch-free (as the f32 kernel)
  float gl[8], bl[4][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float l3[3][3];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int t = 0; t < 3; ++t) l3[kd][t] = lkv[kd][t][j];
    gl[j] = lkv[0][0][j] + lkv[1][0][j] + lkv[2][0][j];
#pragma unroll
    for (int m = 0; m < 4; ++m) bl[m][j] = left_sum(l3, 1, m - 2, D);
  }
  const int da = max(d0, 1), db = min(d1, D - 1);
  if (w0 - (db - 1) >= 2) {  // (as the f32 kernel)
    for (int d = da; d < db; ++d) {
      float pre[8];
      right(w - d - T.u0, d, pre);
#pragma unroll
      for (int j = 0; j < 8; ++j) pre[j] += gl[j];
      store(d, pre);
    }
    return;
  }
  for (int d = da; d < db; ++d) {
    const int u = w - d;
    float pre[8];
    right(u - T.u0, d, pre);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float l = u >= 2 ? gl[j] : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) l = u == m - 2 ? bl[m][j] : l;
      pre[j] += l;
    }
    store(d, pre);
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
  LEA_CHECK_FLAGS(flags, LEA_RELU | 0x300u, "lea_cv_stem_combine");
  a.flags = flags & (LEA_RELU | 0x300u);  // 0x100 / 0x200: probe-only variants (tools)
  a.nseg = (W + cvs::WS - 1) / cvs::WS;
  const int ob = dtype == LEA_F32 ? cvs::OB : cvs::OB8;
  // LDS floats: ob (dchunk + 3 WS - 1) sums + ob dchunk corrections
  a.dchunk = std::min(D3, (cvs::kLdsBytes / (int)sizeof(float) / ob - (3 * cvs::WS - 1)) / 2);
  a.nds = (D3 + a.dchunk - 1) / a.dchunk;
  a.ncob = (cout + ob - 1) / ob;
  const long long nblk = (long long)B * a.ncob * H * a.nds * a.nseg;
  LEA_CHECK_ARG(nblk < (1LL << 31), "lea_cv_stem_combine: grid too large");
  const size_t lds = (size_t)ob * (2 * a.dchunk + 3 * cvs::WS - 1) * sizeof(float);
  if (dtype == LEA_F32)
    cvs::cv_stem_f32_kernel<<<dim3((unsigned)nblk), cvs::kThreads, lds, as_stream(stream)>>>(a);
  else
    cvs::cv_stem_c8_kernel<<<dim3((unsigned)nblk), cvs::kThreads, lds, as_stream(stream)>>>(a);
  return launch_status("lea_cv_stem_combine");
}
