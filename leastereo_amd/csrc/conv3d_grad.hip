// Training backward of the matching net's hot op: ConvBR3d
// (models/operations_3d.py:31-47) with BatchNorm3d in train mode (batch statistics,
// running-stat update, as train.py:130-178 runs it) or eval mode, and its gradients.
//
//   forward   z = conv3d(x, w)                     (lea_conv3d_bnrelu, no BN, no ReLU)
//             y = relu(gamma * (z - mean) * invstd + beta)          lea_bn_forward_f32
//   backward  g  = dy * [y > 0]                     (ReLU mask, when the op has one)
//             dgamma = sum g * xhat, dbeta = sum g, xhat = (z - mean) * invstd
//             dz = gamma * invstd * (g - dbeta / N - xhat * dgamma / N)   (train mode)
//             dz = gamma * invstd * g                                     (eval mode)
//                                                                   lea_bn_backward_f32
//             dx = conv3d(dz, flip(w)^T)            (lea_conv3d_flip_weights + the
//                                                    forward engine: stride 1, pad k/2)
//             dw = sum_{b, v} dz[co][v] x[ci][v + tap]                lea_conv3d_wgrad
//
// Weight gradient: a GEMM with M = cout, N = cin * k^3 and K = B * D * H * W (millions
// of voxels), on v_mfma_f32_16x16x4f32.  A workgroup owns one (input-channel chunk,
// 16 * MT couts) block and walks a strided set of 64-voxel row segments (K split over
// nsplit workgroups): per segment it stages dz[co][64] and the chunk's halo rows
// x[ci][kd][kh][64 + k - 1] in LDS, and its four waves take a quarter of the segment's
// 16 K-steps each.  A (lane l) = dz[co = 16 m + (l & 15)][voxel 4 s + (l >> 4)],
// B (lane l) = x[(tap, ci) = column l & 15][same voxel]; N tile = 4 taps x 4 channels
// (k = 3: 7 tiles, the 28th tap slot zero) or 16 channels (k = 1).  Each wave stores
// its partial block once; two more kernels sum the 4 * nsplit partials in a fixed
// order (32 groups in parallel, then the groups), so dw is deterministic.  The reductions of the BN statistics are two-level
// in double (per-slice partials, then a fixed-order sum), also deterministic.
#include <algorithm>

#include "common.h"

namespace lea {
namespace grad {

using f32x4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;

constexpr int SEG = 64;   // voxels (along W) per K segment
constexpr int NWAVE = 4;  // waves per workgroup

// KD = KS: the 3D conv's taps; KD = 1, KS = 3: a Conv2d 3x3 (the feature net, D = 1)
template <int KS, int KD = KS>
struct WCfg {
  static constexpr int TAPS = KD * KS * KS;
  static constexpr int CI = KS == 3 ? 4 : 16;    // input channels per chunk
  static constexpr int TPT = 16 / CI;            // taps per 16-column N tile
  static constexpr int NT = (TAPS + TPT - 1) / TPT;
  static constexpr int XC = SEG + KS - 1;        // staged columns per halo row
  static constexpr int XR = KD * KS;             // staged (kd, kh) rows per channel
  static constexpr int XS = CI * XR * XC;        // staged halo values per segment
  // LDS strides (floats) for the A / B reads, each a ds_read_b32: two groups of 32 lanes on
  // 32 banks (MI355X_MICROARCH.md, LDS).  A row of 70 and a channel of 632 (k = 3), 216 (2D
  // 3x3), a channel of 66 (k = 1), and dz rows 66 apart put every read's 32-lane groups on 32
  // distinct banks (tools/wgrad_banks.py, exhaustive over the N tiles, waves and K steps).
  // r06: the strides had been chosen for 64 banks (630 / 210 / 68, dz rows 68 apart): two-way
  // on every read, 43 % of conv1's LDS cycles were conflict cycles
  static constexpr int XRS = KS == 3 ? 70 : SEG;
  static constexpr int CIS = KS == 3 ? (KD == 3 ? 632 : 216) : 66;
  static constexpr int XLDS = CI * CIS;
  static constexpr int GRS = 66;
  static constexpr int PX = (XS + 255) / 256;    // prefetched halo values per thread
};

struct WArgs {
  const float* x;
  const float* dz;
  float* part;
  int B, cin, cout, D, H, W;
  int nwseg, nseg, nsplit;
};

// Per segment: 4 K-steps x NT x MT MFMAs per wave from LDS; the next segment's halo
// and dz values are loaded into registers before this segment's MFMAs (they land
// under them) and written to LDS after the next barrier.
template <int KS, int KD, int MT>
__global__ __launch_bounds__(256) void wgrad_kernel(const WArgs a) {
  using C = WCfg<KS, KD>;
  constexpr int NT = C::NT, PX = C::PX, PG = MT * 4;  // 16 MT rows x 64 / 256 threads
  __shared__ float xs[C::XLDS];
  __shared__ float gs[16 * MT * C::GRS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ci0 = blockIdx.y * C::CI, co0 = blockIdx.z * 16 * MT;
  const long long HW = (long long)a.H * a.W, V = HW * a.D;
  const int j = lane & 15, kr = lane >> 4;

  // this lane's B column per N tile: (tap, channel) -> LDS offset without the voxel
  int boff[NT];
  bool bval[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int tap = nt * C::TPT + j / C::CI, ci = j % C::CI;
    const int kd = tap / (KS * KS), kh = (tap / KS) % KS, kw = tap % KS;  // kd = 0 when KD = 1
    bval[nt] = tap < C::TAPS;
    boff[nt] = bval[nt] ? ci * C::CIS + (kd * KS + kh) * C::XRS + kw : 0;
  }
  // the staging slots of this thread: halo value t = e / (ci, row, col), dz value t = (co, col)
  float px[PX], pg[PG];
  auto load_seg = [&](int seg) {
    const int wsg = seg % a.nwseg;
    int r = seg / a.nwseg;
    const int h = r % a.H;
    r /= a.H;
    const int d = r % a.D, b = r / a.D;
    const int w0 = wsg * SEG;
#pragma unroll
    for (int t = 0; t < PX; ++t) {
      const int e = tid + 256 * t;
      const int col = e % C::XC, r2 = e / C::XC;
      const int row = r2 % C::XR, c = ci0 + r2 / C::XR;
      const int dd = d + row / KS - KD / 2, hh = h + row % KS - KS / 2, ww = w0 + col - KS / 2;
      const bool ok = e < C::XS && c < a.cin && (unsigned)dd < (unsigned)a.D && (unsigned)hh < (unsigned)a.H &&
                      (unsigned)ww < (unsigned)a.W;
      px[t] = ok ? a.x[((long long)b * a.cin + c) * V + dd * HW + (long long)hh * a.W + ww] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < PG; ++t) {
      const int e = tid + 256 * t, col = e % SEG, c = co0 + e / SEG, ww = w0 + col;
      pg[t] = (c < a.cout && ww < a.W) ? a.dz[((long long)b * a.cout + c) * V + d * HW + (long long)h * a.W + ww]
                                       : 0.f;
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  if ((int)blockIdx.x < a.nseg) load_seg(blockIdx.x);
  for (int seg = blockIdx.x; seg < a.nseg; seg += a.nsplit) {
    __syncthreads();  // the previous segment's LDS reads are done
#pragma unroll
    for (int t = 0; t < PX; ++t) {
      const int e = tid + 256 * t;
      const int col = e % C::XC, r2 = e / C::XC;
      if (e < C::XS) xs[(r2 / C::XR) * C::CIS + (r2 % C::XR) * C::XRS + col] = px[t];
    }
#pragma unroll
    for (int t = 0; t < PG; ++t) {
      const int e = tid + 256 * t;
      gs[(e / SEG) * C::GRS + e % SEG] = pg[t];
    }
    __syncthreads();
    if (seg + a.nsplit < a.nseg) load_seg(seg + a.nsplit);
#pragma unroll
    for (int q = 0; q < SEG / (4 * NWAVE); ++q) {
      const int v = 4 * (wave + NWAVE * q) + kr;
      float av[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = gs[(16 * m + j) * C::GRS + v];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float bv = bval[nt] ? xs[boff[nt] + v] : 0.f;
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv, acc[m][nt], 0, 0, 0);
      }
    }
  }
  // partial (blockIdx.x, wave): [cout][cin][taps]; this block writes its (chunk, couts) part
  const long long nw = (long long)a.cout * a.cin * C::TAPS;
  float* const part = a.part + (long long)(blockIdx.x * NWAVE + wave) * nw;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tap = nt * C::TPT + j / C::CI, ci = ci0 + j % C::CI;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int co = co0 + 16 * m + 4 * kr + r4;
        if (tap < C::TAPS && ci < a.cin && co < a.cout)
          part[((long long)co * a.cin + ci) * C::TAPS + tap] = acc[m][nt][r4];
      }
    }
}

// fixed-order two-level sum of the np partials: stage 1, workgroup (element block x,
// group y) sums partials y, y + G, ... of 64 elements (wave w takes every 4th of them,
// coalesced over the lanes), then its 4 waves in order; stage 2 sums the G groups
constexpr int kSumGroups = 32;

__global__ __launch_bounds__(256) void sum_partials_stage1(const float* __restrict__ part, float* __restrict__ part2,
                                                           long long n, int np) {
  __shared__ float red[NWAVE][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long e = blockIdx.x * 64LL + lane;
  const int G = gridDim.y, y = blockIdx.y;
  float s = 0.f;
  if (e < n)
    for (int p = y + G * wave; p < np; p += G * NWAVE) s += part[(long long)p * n + e];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < n) part2[(long long)y * n + e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ void sum_partials_stage2(const float* __restrict__ part2, float* __restrict__ out, long long n, int G) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int y = 0; y < G; ++y) s += part2[(long long)y * n + i];
    out[i] = s;
  }
}

__global__ void flip_weights_kernel(const float* __restrict__ w, float* __restrict__ wt, int cout, int cin, int ks) {
  const int taps = ks * ks * ks;
  const long long n = (long long)cout * cin * taps;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int tap = (int)(i % taps);
    const long long q = i / taps;
    const int co = (int)(q % cout), ci = (int)(q / cout);  // wt[ci][co][tap]
    wt[i] = w[((long long)co * cin + ci) * taps + (taps - 1 - tap)];
  }
}

// ---- BatchNorm3d statistics: per channel, two double sums over (b, v) ----
constexpr int kSlices = 64;  // per-channel slices of the first reduction level

enum { kMomentsZ = 0, kMomentsGrad = 1 };

struct BnArgs {
  const float* z;
  const float* dy;
  const float* y;
  const float* mean;
  const float* invstd;
  int B, C;
  long long V;
  int relu;
};

__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// MODE kMomentsZ: (sum z, sum z^2); kMomentsGrad: (sum g, sum g * xhat), g = dy [* (y > 0)]
template <int MODE>
__global__ __launch_bounds__(256) void bn_moments_kernel(const BnArgs a, double* __restrict__ part) {
  __shared__ double red[8];
  const int c = blockIdx.y, s = blockIdx.x;
  const long long n = (long long)a.B * a.V;
  const long long e0 = n * s / kSlices, e1 = n * (s + 1) / kSlices;
  const float mu = MODE == kMomentsGrad ? a.mean[c] : 0.f, is = MODE == kMomentsGrad ? a.invstd[c] : 0.f;
  double s0 = 0.0, s1 = 0.0;
  long long e = e0 + threadIdx.x, b = e / a.V, v = e - b * a.V;  // (b, v) stepped, not divided
  for (; e < e1; e += blockDim.x) {
    const long long i = (b * a.C + c) * a.V + v;
    const float zv = a.z[i];
    if (MODE == kMomentsZ) {
      s0 += zv;
      s1 += (double)zv * zv;
    } else {
      float g = a.dy[i];
      if (a.relu && !(a.y[i] > 0.f)) g = 0.f;
      s0 += g;
      s1 += (double)g * ((zv - mu) * is);
    }
    v += blockDim.x;
    while (v >= a.V) {
      v -= a.V;
      ++b;
    }
  }
  const double t0 = block_sum(s0, red);
  const double t1 = block_sum(s1, red);
  if (threadIdx.x == 0) {
    part[((long long)c * kSlices + s) * 2] = t0;
    part[((long long)c * kSlices + s) * 2 + 1] = t1;
  }
}

// forward finalize: batch mean / biased variance -> mean, invstd; running stats
// (torch: running_var takes the unbiased variance, momentum-weighted)
__global__ void bn_train_finalize_kernel(const double* __restrict__ part, int C, long long n, float eps, float momentum,
                                         float* __restrict__ mean, float* __restrict__ invstd, float* running_mean,
                                         float* running_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  for (int s = 0; s < kSlices; ++s) {
    s0 += part[((long long)c * kSlices + s) * 2];
    s1 += part[((long long)c * kSlices + s) * 2 + 1];
  }
  const double mu = s0 / (double)n;
  double var = s1 / (double)n - mu * mu;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mu);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
}

__global__ void bn_eval_stats_kernel(int C, float eps, const float* __restrict__ running_mean,
                                     const float* __restrict__ running_var, float* __restrict__ mean,
                                     float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = running_mean[c];
  invstd[c] = 1.f / sqrtf(running_var[c] + eps);
}

// y = relu((z - mean) * invstd * gamma + beta)  (aten's batch_norm element order)
// grid: (voxel blocks, B * C rows); row r = b * C + c
__global__ void bn_apply_kernel(const float* __restrict__ z, float* __restrict__ y, int C, long long V,
                                const float* __restrict__ mean, const float* __restrict__ invstd,
                                const float* __restrict__ gamma, const float* __restrict__ beta, int relu) {
  const int c = (int)(blockIdx.y % C);
  const float mu = mean[c], is = invstd[c], g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float* zr = z + (long long)blockIdx.y * V;
  float* yr = y + (long long)blockIdx.y * V;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < V; i += (long long)gridDim.x * blockDim.x) {
    const float v = (zr[i] - mu) * is * g + bt;
    yr[i] = relu ? fmaxf(v, 0.f) : v;
  }
}

// backward finalize: dgamma, dbeta and the per-channel coefficients of
// dz = k * (g - mg - xhat * mgx): k = gamma * invstd, mg = dbeta / n, mgx = dgamma / n
// (train); eval: mg = mgx = 0
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ part, int C, long long n, int train,
                                       const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       float* dgamma, float* dbeta, float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  for (int s = 0; s < kSlices; ++s) {
    s0 += part[((long long)c * kSlices + s) * 2];
    s1 += part[((long long)c * kSlices + s) * 2 + 1];
  }
  if (dbeta) dbeta[c] = (float)s0;
  if (dgamma) dgamma[c] = (float)s1;
  coef[3 * c] = (gamma ? gamma[c] : 1.f) * invstd[c];
  coef[3 * c + 1] = train ? (float)(s0 / (double)n) : 0.f;
  coef[3 * c + 2] = train ? (float)(s1 / (double)n) : 0.f;
}

__global__ void bn_bwd_apply_kernel(const BnArgs a, const float* __restrict__ coef, float* __restrict__ dz) {
  const int c = (int)(blockIdx.y % a.C);
  const float mu = a.mean[c], is = a.invstd[c], k = coef[3 * c], mg = coef[3 * c + 1], mgx = coef[3 * c + 2];
  const long long r0 = (long long)blockIdx.y * a.V;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < a.V; v += (long long)gridDim.x * blockDim.x) {
    const long long i = r0 + v;
    float g = a.dy[i];
    if (a.relu && !(a.y[i] > 0.f)) g = 0.f;
    const float xh = (a.z[i] - mu) * is;
    dz[i] = k * (g - mg - xh * mgx);
  }
}


// ---- trilinear resample backward (F.interpolate's, skip_model_3d.py:48,50,162) ----
// The forward is separable (a product of per-axis linear interpolations), so its
// transpose is three 1-D transposed passes (W, then H, then D).  Each pass gathers:
// input index i of the axis collects l0(p) g[p] over the outputs p with i0(p) = i and
// l1(p) g[p] over those with i1(p) = i (axis_index: the forward's own index rule), p
// scanned over a window that covers every such output -- deterministic, no atomics.
__global__ void interp_t_kernel(const float* __restrict__ g, float* __restrict__ out, long long outer, int n_out,
                                int n_in, long long inner, float ratio, int ac) {
  const long long n = outer * n_in * inner;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e % inner;
    const long long t = e / inner;
    const int i = (int)(t % n_in);
    const long long o = t / n_in;
    int p0 = 0, p1 = n_out - 1;
    if (ratio > 0.f) {  // outputs whose source index i0 is i - 1 or i (one output of slack per side)
      const float lo = ac ? ((float)i - 1.f) / ratio : ((float)i - 0.5f) / ratio - 0.5f;
      const float hi = ac ? ((float)i + 1.f) / ratio : ((float)i + 1.5f) / ratio - 0.5f;
      p0 = max(0, (int)floorf(lo) - 1);
      p1 = min(n_out - 1, (int)ceilf(hi) + 1);
    }
    const float* gp = g + o * n_out * inner + r;
    if (n_in == n_out) {  // the forward's identity axis (axis_index: i0 = i1 = o, l0 = 1)
      out[e] = gp[(long long)i * inner];
      continue;
    }
    float s = 0.f;
    for (int p = p0; p <= p1; ++p) {
      const Axis ax = axis_index(ratio, p, n_in, n_out, ac);
      float wgt = 0.f;
      if (ax.i0 == i) wgt += ax.l0;
      if (ax.i1 == i) wgt += ax.l1;
      if (wgt != 0.f) s += wgt * gp[(long long)p * inner];
    }
    out[e] = s;
  }
}

// ---- Disp + DisparityRegression backward (build_model_2d.py:33-42,52-57) ----
// disp = sum_d d p_d, p = softmax(-U), U = trilinear(cost, ac=False): per output pixel
// dU_d = -dout * p_d * (d - disp).  One thread per pixel walks D three times (min, sum,
// then dU), U re-interpolated with the forward's source-index rule; the D part of the
// interpolation's transpose is applied on the fly -- dU_d goes to the two cost planes
// its depth lerp read (i0 with l0, i1 with l1; i0 is non-decreasing in d, so a
// two-value window flushes each plane once, in order) -- and the kernel writes
// dV[b][dd][oh][ow] over the D3 planes instead of dU over maxdisp.
__global__ __launch_bounds__(256) void disp_bwd_kernel(const float* __restrict__ cost, const float* __restrict__ disp,
                                                       const float* __restrict__ dout, float* __restrict__ dV,
                                                       int D3, int H3, int W3, int maxdisp, float rd, float rh,
                                                       float rw) {
  const int Ho = 3 * H3, Wo = 3 * W3;
  const int ow = blockIdx.x * blockDim.x + threadIdx.x;
  if (ow >= Wo) return;
  const int oh = blockIdx.y, b = blockIdx.z;
  const Axis ah = axis_index(rh, oh, H3, Ho, 0), aw = axis_index(rw, ow, W3, Wo, 0);
  const long long HW = (long long)H3 * W3;
  const float* c = cost + (long long)b * D3 * HW;
  auto plane = [&](int d) {
    const float* q = c + d * HW;
    return ah.l0 * (aw.l0 * q[ah.i0 * W3 + aw.i0] + aw.l1 * q[ah.i0 * W3 + aw.i1]) +
           ah.l1 * (aw.l0 * q[ah.i1 * W3 + aw.i0] + aw.l1 * q[ah.i1 * W3 + aw.i1]);
  };
  auto U = [&](const Axis& ad) { return ad.l0 * plane(ad.i0) + ad.l1 * plane(ad.i1); };
  float m = 3.4e38f;
  for (int od = 0; od < maxdisp; ++od) m = fminf(m, U(axis_index(rd, od, D3, maxdisp, 0)));
  float s = 0.f;
  for (int od = 0; od < maxdisp; ++od) s += expf(m - U(axis_index(rd, od, D3, maxdisp, 0)));
  const long long pix = ((long long)b * Ho + oh) * Wo + ow;
  const float g = dout[pix] / s, dsp = disp[pix];
  const long long plane_o = (long long)Ho * Wo;
  float* out = dV + (long long)b * D3 * plane_o + (long long)oh * Wo + ow;
  int lo = 0;
  float a0 = 0.f, a1 = 0.f;  // plane lo, lo + 1
  for (int od = 0; od < maxdisp; ++od) {
    const Axis ad = axis_index(rd, od, D3, maxdisp, 0);
    const float du = -g * expf(m - U(ad)) * ((float)od - dsp);
    while (ad.i0 > lo) {
      out[lo * plane_o] = a0;
      a0 = a1;
      a1 = 0.f;
      ++lo;
    }
    a0 += ad.l0 * du;
    if (ad.i1 != ad.i0)
      a1 += ad.l1 * du;
    else
      a0 += ad.l1 * du;
  }
  for (; lo < D3; ++lo) {
    out[lo * plane_o] = a0;
    a0 = a1;
    a1 = 0.f;
  }
}

// ---- cost-volume backward (retrain/LEAStereo.py:34-48) ----
// cost[b, c, i, h, w] = L[b, c, h, w], cost[b, C + c, i, h, w] = R[b, c, h, w - i] (w >= i):
// dL[b, c, h, w] = sum_{i <= w} dcost[b, c, i, h, w],
// dR[b, c, h, w] = sum_{i < W - w} dcost[b, C + c, i, h, w + i]
__global__ void cost_volume_bwd_kernel(const float* __restrict__ dcost, float* __restrict__ dl,
                                       float* __restrict__ dr, int B, int C, int H, int W, int D3) {
  const long long n = (long long)B * C * H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(e % W);
    long long t = e / W;
    const int h = (int)(t % H);
    t /= H;
    const int c = (int)(t % C), b = (int)(t / C);
    const long long HW = (long long)H * W, vol = (long long)D3 * HW;
    const float* gl = dcost + ((long long)b * 2 * C + c) * vol + (long long)h * W + w;
    const float* gr = dcost + ((long long)b * 2 * C + C + c) * vol + (long long)h * W + w;
    float sl = 0.f, sr = 0.f;
    for (int i = 0; i < D3 && i <= w; ++i) sl += gl[i * HW];
    for (int i = 0; i < D3 && w + i < W; ++i) sr += gr[i * HW + i];
    dl[e] = sl;
    dr[e] = sr;
  }
}

// couts per block: 16 or 32 (MT = 4 held 392 registers: one wave per SIMD)
inline int mt_for(int cout) { return cout <= 16 ? 1 : 2; }

// K split: about 2048 workgroups, at most 256 MB of partials
inline int nsplit_for(int B, int cin, int cout, int D, int H, int W, int k, int kd) {
  const int taps = kd * k * k, ci = k == 3 ? WCfg<3>::CI : WCfg<1>::CI;
  const long long nblk = (long long)((cin + ci - 1) / ci) * ((cout + 16 * mt_for(cout) - 1) / (16 * mt_for(cout)));
  const long long nseg = (long long)B * D * H * ((W + SEG - 1) / SEG);
  long long s = 2048 / nblk;
  const long long per = (long long)NWAVE * cout * cin * taps * 4;
  s = std::min(s, (256LL << 20) / per);
  s = std::min(s, nseg);
  return (int)std::max(1LL, s);
}

inline int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 4096); }
// (voxel blocks, B * C rows) for the per-channel elementwise kernels
inline dim3 row_grid(int B, int C, long long V) {
  const long long rows = (long long)B * C;
  return dim3((unsigned)std::max<long long>(1, std::min<long long>((V + 255) / 256, 4096 / std::min(rows, 4096LL) + 1)),
              (unsigned)rows);
}

}  // namespace grad
}  // namespace lea

using namespace lea;
using namespace lea::grad;

namespace lea {
namespace grad {

// K split over nsplit workgroups per (chunk, cout block); kd = k (3D) or 1 (2D 3x3)
size_t wgrad_ws_bytes(int B, int cin, int cout, int D, int H, int W, int k, int kd) {
  if (B <= 0 || cin <= 0 || cout <= 0 || D <= 0 || H <= 0 || W <= 0 || (k != 1 && k != 3)) return 0;
  const int ns = nsplit_for(B, cin, cout, D, H, W, k, kd);
  return ((size_t)ns * NWAVE + kSumGroups) * cout * cin * kd * k * k * sizeof(float);
}

int wgrad(const char* what, const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes, int B,
          int cin, int cout, int D, int H, int W, int k, int kd, void* stream) {
  LEA_CHECK_ARG(x && dz && dw && workspace, "%s: null pointer", what);
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && D > 0 && H > 0 && W > 0, "%s: bad shape", what);
  LEA_CHECK_ARG(k == 1 || k == 3, "%s: k=%d unsupported", what, k);
  LEA_CHECK_ARG((long long)D * H <= (1LL << 30) / B, "%s: volume too large", what);
  const size_t need = wgrad_ws_bytes(B, cin, cout, D, H, W, k, kd);
  LEA_CHECK_ARG(ws_bytes >= need, "%s: workspace %zu < %zu bytes", what, ws_bytes, need);
  hipStream_t st = as_stream(stream);
  WArgs a;
  a.x = x;
  a.dz = dz;
  a.part = (float*)workspace;
  a.B = B;
  a.cin = cin;
  a.cout = cout;
  a.D = D;
  a.H = H;
  a.W = W;
  a.nwseg = (W + SEG - 1) / SEG;
  a.nseg = B * D * H * a.nwseg;
  a.nsplit = nsplit_for(B, cin, cout, D, H, W, k, kd);
  const int mt = mt_for(cout);
  const int ci = k == 3 ? WCfg<3>::CI : WCfg<1>::CI;
  const dim3 grid((unsigned)a.nsplit, (unsigned)((cin + ci - 1) / ci), (unsigned)((cout + 16 * mt - 1) / (16 * mt)));
  LEA_CHECK_ARG(grid.y <= 65535 && grid.z <= 65535, "%s: grid too large", what);
#define LEA_WGRAD(KS, KD, MT) \
  if (k == KS && kd == KD && mt == MT) wgrad_kernel<KS, KD, MT><<<grid, 256, 0, st>>>(a);
  LEA_WGRAD(3, 3, 1) LEA_WGRAD(3, 3, 2) LEA_WGRAD(1, 1, 1) LEA_WGRAD(1, 1, 2) LEA_WGRAD(3, 1, 1) LEA_WGRAD(3, 1, 2)
#undef LEA_WGRAD
  int rc = launch_status(what);
  if (rc) return rc;
  const long long n = (long long)cout * cin * kd * k * k;
  const int np = a.nsplit * NWAVE, G = std::min(kSumGroups, np);
  float* const part2 = a.part + (long long)np * n;
  sum_partials_stage1<<<dim3((unsigned)((n + 63) / 64), (unsigned)G), 256, 0, st>>>(a.part, part2, n, np);
  rc = launch_status(what);
  if (rc) return rc;
  sum_partials_stage2<<<grid_for(n), 256, 0, st>>>(part2, dw, n, G);
  return launch_status(what);
}

}  // namespace grad
}  // namespace lea

extern "C" size_t lea_conv3d_wgrad_workspace_bytes(int B, int cin, int cout, int D, int H, int W, int k) {
  return wgrad_ws_bytes(B, cin, cout, D, H, W, k, k);
}

extern "C" int lea_conv3d_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes, int B,
                                int cin, int cout, int D, int H, int W, int k, void* stream) {
  clear_error();
  return wgrad("lea_conv3d_wgrad", x, dz, dw, workspace, ws_bytes, B, cin, cout, D, H, W, k, k, stream);
}

extern "C" size_t lea_conv2d_wgrad_workspace_bytes(int B, int cin, int cout, int H, int W) {
  return wgrad_ws_bytes(B, cin, cout, 1, H, W, 3, 1);
}

extern "C" int lea_conv2d_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes, int B,
                                int cin, int cout, int H, int W, void* stream) {
  clear_error();
  return wgrad("lea_conv2d_wgrad", x, dz, dw, workspace, ws_bytes, B, cin, cout, 1, H, W, 3, 1, stream);
}

extern "C" int lea_conv3d_flip_weights(const float* w, float* wt, int cout, int cin, int k, void* stream) {
  LEA_CHECK_ARG(w && wt && w != wt, "lea_conv3d_flip_weights: null or aliased pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0 && (k == 1 || k == 3), "lea_conv3d_flip_weights: bad shape");
  const long long n = (long long)cout * cin * k * k * k;
  flip_weights_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(w, wt, cout, cin, k);
  return launch_status("lea_conv3d_flip_weights");
}

extern "C" size_t lea_bn_workspace_bytes(int C) {
  return C > 0 ? (size_t)C * kSlices * 2 * sizeof(double) + (size_t)C * 3 * sizeof(float) : 0;
}

extern "C" int lea_bn_forward_f32(const float* z, float* y, int B, int C, int64_t V, const float* gamma,
                                  const float* beta, float* running_mean, float* running_var, float momentum,
                                  float eps, int training, unsigned flags, float* mean, float* invstd,
                                  void* workspace, void* stream) {
  lea::clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_bn_forward_f32");
  LEA_CHECK_ARG(z && y && mean && invstd, "lea_bn_forward_f32: null pointer");
  LEA_CHECK_ARG(B > 0 && C > 0 && V > 0 && (long long)B * C <= 65535, "lea_bn_forward_f32: bad shape");
  LEA_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "lea_bn_forward_f32: running stats pair");
  LEA_CHECK_ARG(training || running_mean, "lea_bn_forward_f32: eval mode needs the running stats");
  LEA_CHECK_ARG(!training || workspace, "lea_bn_forward_f32: train mode needs the workspace");
  LEA_CHECK_ARG(eps > 0.f && momentum >= 0.f && momentum <= 1.f, "lea_bn_forward_f32: eps/momentum");
  hipStream_t st = as_stream(stream);
  if (training) {
    BnArgs a{z, nullptr, nullptr, nullptr, nullptr, B, C, V, 0};
    bn_moments_kernel<kMomentsZ><<<dim3(kSlices, C), 256, 0, st>>>(a, (double*)workspace);
    int rc = launch_status("lea_bn_forward_f32(moments)");
    if (rc) return rc;
    bn_train_finalize_kernel<<<(C + 63) / 64, 64, 0, st>>>((const double*)workspace, C, (long long)B * V, eps,
                                                           momentum, mean, invstd, running_mean, running_var);
  } else {
    bn_eval_stats_kernel<<<(C + 63) / 64, 64, 0, st>>>(C, eps, running_mean, running_var, mean, invstd);
  }
  int rc = launch_status("lea_bn_forward_f32(stats)");
  if (rc) return rc;
  bn_apply_kernel<<<row_grid(B, C, V), 256, 0, st>>>(z, y, C, V, mean, invstd, gamma, beta, (flags & LEA_RELU) ? 1 : 0);
  return launch_status("lea_bn_forward_f32(apply)");
}

extern "C" int lea_bn_backward_f32(const float* dy, const float* y, const float* z, float* dz, int B, int C,
                                   int64_t V, const float* gamma, const float* mean, const float* invstd,
                                   int training, unsigned flags, float* dgamma, float* dbeta, void* workspace,
                                   void* stream) {
  lea::clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_bn_backward_f32");
  LEA_CHECK_ARG(dy && z && dz && mean && invstd && workspace, "lea_bn_backward_f32: null pointer");
  LEA_CHECK_ARG(!(flags & LEA_RELU) || y, "lea_bn_backward_f32: LEA_RELU needs y");
  LEA_CHECK_ARG(B > 0 && C > 0 && V > 0 && (long long)B * C <= 65535, "lea_bn_backward_f32: bad shape");
  hipStream_t st = as_stream(stream);
  BnArgs a{z, dy, y, mean, invstd, B, C, V, (flags & LEA_RELU) ? 1 : 0};
  double* part = (double*)workspace;
  float* coef = (float*)(part + (long long)C * kSlices * 2);
  bn_moments_kernel<kMomentsGrad><<<dim3(kSlices, C), 256, 0, st>>>(a, part);
  int rc = launch_status("lea_bn_backward_f32(moments)");
  if (rc) return rc;
  bn_bwd_finalize_kernel<<<(C + 63) / 64, 64, 0, st>>>(part, C, (long long)B * V, training ? 1 : 0, gamma, invstd,
                                                       dgamma, dbeta, coef);
  rc = launch_status("lea_bn_backward_f32(finalize)");
  if (rc) return rc;
  bn_bwd_apply_kernel<<<row_grid(B, C, V), 256, 0, st>>>(a, coef, dz);
  return launch_status("lea_bn_backward_f32(apply)");
}

extern "C" size_t lea_resample3d_backward_workspace_bytes(int B, int C, int Di, int Hi, int Wi, int Do, int Ho,
                                                        int Wo) {
  if (B <= 0 || C <= 0 || Di <= 0 || Hi <= 0 || Wi <= 0 || Do <= 0 || Ho <= 0 || Wo <= 0) return 0;
  return (size_t)B * C * ((size_t)Do * Ho * Wi + (size_t)Do * Hi * Wi) * sizeof(float);
}

extern "C" int lea_resample3d_trilinear_backward(const float* dy, float* dx, void* workspace, size_t ws_bytes, int B,
                                                 int C, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                                 int align_corners, void* stream) {
  LEA_CHECK_ARG(dy && dx && workspace && dy != dx, "lea_resample3d_trilinear_backward: null or aliased pointer");
  const size_t need = lea_resample3d_backward_workspace_bytes(B, C, Di, Hi, Wi, Do, Ho, Wo);
  LEA_CHECK_ARG(need > 0, "lea_resample3d_trilinear_backward: bad shape");
  LEA_CHECK_ARG(ws_bytes >= need, "lea_resample3d_trilinear_backward: workspace %zu < %zu bytes", ws_bytes, need);
  hipStream_t st = as_stream(stream);
  const int ac = align_corners ? 1 : 0;
  float* gw = (float*)workspace;                      // [B C Do Ho Wi]
  float* gh = gw + (size_t)B * C * Do * Ho * Wi;      // [B C Do Hi Wi]
  const long long bc = (long long)B * C;
  interp_t_kernel<<<grid_for(bc * Do * Ho * Wi), 256, 0, st>>>(dy, gw, bc * Do * Ho, Wo, Wi, 1, axis_ratio(Wi, Wo, ac), ac);
  int rc = launch_status("lea_resample3d_trilinear_backward(w)");
  if (rc) return rc;
  interp_t_kernel<<<grid_for(bc * Do * Hi * Wi), 256, 0, st>>>(gw, gh, bc * Do, Ho, Hi, Wi, axis_ratio(Hi, Ho, ac), ac);
  rc = launch_status("lea_resample3d_trilinear_backward(h)");
  if (rc) return rc;
  interp_t_kernel<<<grid_for(bc * Di * Hi * Wi), 256, 0, st>>>(gh, dx, bc, Do, Di, (long long)Hi * Wi,
                                                               axis_ratio(Di, Do, ac), ac);
  return launch_status("lea_resample3d_trilinear_backward(d)");
}

extern "C" int lea_disparity_regression_backward(const float* cost, const float* disp, const float* dout, float* dU,
                                                 int B, int D3, int H3, int W3, int maxdisp, void* stream) {
  LEA_CHECK_ARG(cost && disp && dout && dU, "lea_disparity_regression_backward: null pointer");
  LEA_CHECK_ARG(B > 0 && D3 > 0 && H3 > 0 && W3 > 0 && maxdisp > 0 && B <= 65535 && 3 * H3 <= 65535,
                "lea_disparity_regression_backward: bad shape");
  const dim3 grid((unsigned)((3 * W3 + 255) / 256), (unsigned)(3 * H3), (unsigned)B);
  disp_bwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(cost, disp, dout, dU, D3, H3, W3, maxdisp,
                                                      axis_ratio(D3, maxdisp, 0), axis_ratio(H3, 3 * H3, 0),
                                                      axis_ratio(W3, 3 * W3, 0));
  return launch_status("lea_disparity_regression_backward");
}

extern "C" int lea_build_cost_volume_backward(const float* dcost, float* dleft, float* dright, int B, int C, int H,
                                              int W, int D3, void* stream) {
  LEA_CHECK_ARG(dcost && dleft && dright && dleft != dright, "lea_build_cost_volume_backward: null pointer");
  LEA_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0 && D3 > 0, "lea_build_cost_volume_backward: bad shape");
  const long long n = (long long)B * C * H * W;
  cost_volume_bwd_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(dcost, dleft, dright, B, C, H, W, D3);
  return launch_status("lea_build_cost_volume_backward");
}
