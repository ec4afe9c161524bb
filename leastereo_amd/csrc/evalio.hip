// Input standardisation and disparity metrics on the device:
// the host steps either side of LEAStereo.forward.
//
//  * lea_standardize_crop_u8: predict.py:162-184 (load_data: per image channel
//    (x - mean) / std with whole-image float64 statistics, population std, stored
//    float32) fused with predict.py:144-159 (test_transform: zero-pad top-left up to
//    the crop, or centre-crop).  The statistics are exact: sum x and sum x^2 of the
//    uint8 samples are integers (64-bit atomics, order-free), mean = S1 / N and
//    var = (N S2 - S1^2) / N^2 evaluated from them, so the only rounding left is
//    the float64 -> float32 store, as in the reference.
//  * lea_disparity_metrics: evaluation.py:287-307 (EPE over disp in [0.001, maxdisp],
//    optional `round() + z_shift` of evaluation.py:169) and utils/metrics.py:6-46
//    (3-px error and bad-N with the reference's int64 abs_diff array: the float
//    difference is truncated toward zero, NaN / out-of-range become INT64_MIN).
//    Per-workgroup partials in a caller workspace, then a fixed-order final pass:
//    bit-reproducible from run to run.
// Both are HBM-bound streaming passes (bytes in DESIGN.md §4).
#include <cmath>

#include "common.h"

namespace lea {

// ---------------------------------------------------------------- standardise
constexpr int kStatThreads = 256;

// grid (G, 2B): blockIdx.y = image (0..B-1 left, B..2B-1 right).  The image is
// read as a stream of 16-byte words of interleaved samples; byte i of the stream
// is channel i % pix_stride (channels >= 3, e.g. PNG alpha, are skipped).
__global__ __launch_bounds__(kStatThreads) void u8_stats_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int B, long long npix,
    int pix_stride, unsigned long long* __restrict__ sums /* [2B][3][2] */) {
  const int img = blockIdx.y;
  const long long nbytes = npix * pix_stride;
  const uint8_t* src = (img < B ? left + (long long)img * nbytes : right + (long long)(img - B) * nbytes);
  // per-thread partials: at most 2^23 pixels per thread (host bounds G) -> the
  // 32-bit sums of uint8 and of their squares (<= 2^16 each) cannot overflow
  unsigned s1[4] = {0, 0, 0, 0};
  unsigned long long s2[4] = {0, 0, 0, 0};
  const long long nvec = nbytes / 16;
  const bool aligned = ((uintptr_t)src & 15) == 0;
  const long long nv = aligned ? nvec : 0;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < nv;
       v += (long long)gridDim.x * blockDim.x) {
    const uint4 q = reinterpret_cast<const uint4*>(src)[v];
    const unsigned wd[4] = {q.x, q.y, q.z, q.w};
    int ch = (int)((v * 16) % pix_stride);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const unsigned x = (wd[j / 4] >> (8 * (j % 4))) & 0xFFu;
      // channel select without dynamic register indexing
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c == ch) {
          s1[c] += x;
          s2[c] += x * x;
        }
      ch = (ch + 1 == pix_stride) ? 0 : ch + 1;
    }
  }
  for (long long i = nv * 16 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nbytes;
       i += (long long)gridDim.x * blockDim.x) {  // tail (or an unaligned image)
    const unsigned x = src[i];
    const int ch = (int)(i % pix_stride);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c == ch) {
        s1[c] += x;
        s2[c] += x * x;
      }
  }
  __shared__ unsigned long long red[2][3][kStatThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    unsigned long long a = s1[c], b2 = s2[c];
    for (int o = kWave / 2; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      b2 += __shfl_xor(b2, o);
    }
    if (lane == 0) {
      red[0][c][wave] = a;
      red[1][c][wave] = b2;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int c = threadIdx.x % 3, k = threadIdx.x / 3;
    unsigned long long t = 0;
    for (int w = 0; w < kStatThreads / kWave; ++w) t += red[k][c][w];
    atomicAdd(sums + ((long long)img * 3 + c) * 2 + k, t);
  }
}

// predict.py:173-183 for one channel: the float32 value of (x - mean) / std for
// each of the 256 possible uint8 samples (float64 arithmetic, one rounding at the
// store, as the reference's assignment into a float32 array)
__device__ __forceinline__ float standardized(unsigned long long S1, unsigned long long S2,
                                              long long npix, int x) {
  const double n = (double)npix;
  const double mean = (double)S1 / n;
  // N*S2 - S1^2 >= 0 exactly in 128-bit integers, then rounded to double
  const unsigned __int128 num = (unsigned __int128)(unsigned long long)npix * S2 -
                                (unsigned __int128)S1 * S1;
  const double numd = (double)(unsigned long long)(num >> 64) * 18446744073709551616.0 +
                      (double)(unsigned long long)num;
  const double sd = sqrt(numd / (n * n));
  return (float)(((double)x - mean) / sd);
}

// out[b][c][y][x] over the crop; grid (ceil(ch*cw / 1024), 2B).  The 3 x 256 value
// table of this image lives in LDS; a thread maps 4 consecutive crop pixels of a
// row and stores one float4 per channel plane.
__global__ __launch_bounds__(256) void u8_standardize_kernel(
    const uint8_t* __restrict__ left, const uint8_t* __restrict__ right, int B, int H, int W,
    int pix_stride, const unsigned long long* __restrict__ sums, float* __restrict__ out_l,
    float* __restrict__ out_r, int ch, int cw, int pad) {
  const int img = blockIdx.y;
  const bool is_left = img < B;
  const int b = is_left ? img : img - B;
  __shared__ float lut[3][256];
  for (int e = threadIdx.x; e < 3 * 256; e += blockDim.x) {
    const int c = e / 256;
    lut[c][e % 256] = standardized(sums[((long long)img * 3 + c) * 2],
                                   sums[((long long)img * 3 + c) * 2 + 1], (long long)H * W, e % 256);
  }
  __syncthreads();
  const uint8_t* src = (is_left ? left : right) + (long long)b * H * W * pix_stride;
  float* dst = (is_left ? out_l : out_r) + (long long)b * 3 * ch * cw;
  const long long plane = (long long)ch * cw;
  // test_transform geometry: pad (h <= ch and w <= cw) puts the image at the
  // bottom-right of a zero crop; otherwise start = int((h - ch) / 2)
  const int oy = pad ? ch - H : -((H - ch) / 2);
  const int ox = pad ? cw - W : -((W - cw) / 2);
  const int qw = (cw + 3) / 4;  // float4 columns per crop row
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < ch * qw; t += gridDim.x * blockDim.x) {
    const int y = t / qw, x0 = (t - y * qw) * 4;
    const int sy = y - oy;
    float v[3][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sx = x0 + k - ox;
      const bool in = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
      const uint8_t* p = src + ((long long)sy * W + sx) * pix_stride;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c][k] = in ? lut[c][p[c]] : 0.f;
    }
    if ((cw & 3) == 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        *reinterpret_cast<float4*>(dst + c * plane + (long long)y * cw + x0) =
            make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (x0 + k < cw)
#pragma unroll
          for (int c = 0; c < 3; ++c) dst[c * plane + (long long)y * cw + x0 + k] = v[c][k];
    }
  }
}

// ---------------------------------------------------------------- metrics
constexpr int kMetThreads = 256;
constexpr int kMetFields = 8;

struct MetricArgs {
  const float* pred;
  long long pbs;
  const float* gt;
  long long gbs;
  unsigned char* correct;  // optional [B, H*W] 3-px correct mask
  double* partial;         // [B][G][kMetFields]
  int npix;
  float maxdisp;
  int round_pred, z_shift;
  int thr[3];
};

// utils/metrics.py:14-17: abs_diff = np.full(shape, 10000) is an int64 array, so
// `abs_diff[mask] = np.abs(true - pred)` stores the float32 difference truncated
// toward zero (x86 cvttss2si: NaN and |x| >= 2^63 give INT64_MIN)
__device__ __forceinline__ long long trunc_i64(float d) {
  if (!(fabsf(d) < 9.2233720368547758e18f)) return (long long)0x8000000000000000ULL;
  return (long long)d;
}

struct MetricAcc {
  double sum;       // sum |pred - gt| over the EPE mask
  unsigned n[7];    // n_eval, (unused), n_valid, n_correct3, n_le_thr1..3
};

__device__ __forceinline__ void metric_pixel(const MetricArgs& a, float pv, float g,
                                             MetricAcc& m, unsigned char* correct_out) {
  if (a.round_pred) pv = rintf(pv) + (float)a.z_shift;  // evaluation.py:169, half-to-even
  // evaluation.py:287-288: mask = (disp >= 0.001) & (disp <= maxdisp) (float32 compares)
  if (g >= 0.001f && g <= a.maxdisp) {
    m.n[0] += 1;
    m.sum += (double)fabsf(pv - g);
  }
  // utils/metrics.py:6-8 validity, :16-19 correct, :41-43 bad-N
  const bool valid = (g < a.maxdisp) && (g > 0.001f);
  const long long ad = valid ? trunc_i64(fabsf(g - pv)) : 10000LL;
  const float g5 = g * 0.05f;
  const bool ok3 = ad < 3 || (double)ad < (double)g5;
  m.n[2] += valid;
  m.n[3] += ok3;
#pragma unroll
  for (int k = 0; k < 3; ++k) m.n[4 + k] += (ad <= a.thr[k]);
  if (correct_out) *correct_out = ok3 ? 1 : 0;
}

// grid (G, B); a thread takes 4 consecutive pixels per step (float4 loads)
__global__ __launch_bounds__(kMetThreads) void metrics_partial_kernel(const MetricArgs a) {
  const int b = blockIdx.y;
  const float* pr = a.pred + (long long)b * a.pbs;
  const float* gt = a.gt + (long long)b * a.gbs;
  unsigned char* cm = a.correct ? a.correct + (long long)b * a.npix : nullptr;
  MetricAcc m;
  m.sum = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) m.n[k] = 0;
  const bool vec = ((((uintptr_t)pr) | ((uintptr_t)gt)) & 15) == 0;
  const int nq = vec ? a.npix / 4 : 0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
    const float4 p4 = reinterpret_cast<const float4*>(pr)[q];
    const float4 g4 = reinterpret_cast<const float4*>(gt)[q];
    unsigned char c[4];
    metric_pixel(a, p4.x, g4.x, m, &c[0]);
    metric_pixel(a, p4.y, g4.y, m, &c[1]);
    metric_pixel(a, p4.z, g4.z, m, &c[2]);
    metric_pixel(a, p4.w, g4.w, m, &c[3]);
    if (cm) *reinterpret_cast<uchar4*>(cm + 4 * q) = make_uchar4(c[0], c[1], c[2], c[3]);
  }
  for (int p = nq * 4 + blockIdx.x * blockDim.x + threadIdx.x; p < a.npix;
       p += gridDim.x * blockDim.x)
    metric_pixel(a, pr[p], gt[p], m, cm ? cm + p : nullptr);
  // fixed-order block reduction (wave shuffles, then waves in order)
  __shared__ double red[kMetFields][kMetThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < kMetFields; ++k) {
    double v = k == 1 ? m.sum : (k == 7 ? 0.0 : (double)m.n[k]);
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[k][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < kMetFields) {
    double t = 0;
    for (int w = 0; w < kMetThreads / kWave; ++w) t += red[threadIdx.x][w];
    a.partial[((long long)b * gridDim.x + blockIdx.x) * kMetFields + threadIdx.x] = t;
  }
}

// one workgroup per pair: thread t sums field t % 8 over partial rows t / 8,
// t / 8 + 32, ...; then a fixed-order tree over the 32 threads of each field
__global__ __launch_bounds__(256) void metrics_final_kernel(const double* __restrict__ partial,
                                                            int G, double* __restrict__ out) {
  const int b = blockIdx.x, t = threadIdx.x;
  const double* p = partial + (long long)b * G * kMetFields;
  double v = 0;
  for (int e = t; e < G * kMetFields; e += 256) v += p[e];
  __shared__ double red[256];
  red[t] = v;
  __syncthreads();
  for (int o = 128; o >= kMetFields; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t < kMetFields) out[(long long)b * kMetFields + t] = red[t];
}

inline int metric_blocks(long long npix) {
  const long long per = (long long)kMetThreads * 16;
  long long g = (npix + per - 1) / per;
  return (int)(g < 1 ? 1 : (g > 512 ? 512 : g));
}

}  // namespace lea

extern "C" size_t lea_standardize_workspace_bytes(int B) {
  return B > 0 ? (size_t)B * 2 * 3 * 2 * sizeof(unsigned long long) : 0;
}

extern "C" int lea_standardize_crop_u8(const void* left, const void* right, int B, int H, int W,
                                       int pix_stride, float* out_left, float* out_right,
                                       int crop_h, int crop_w, void* workspace, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(left && right && out_left && out_right && workspace,
                "lea_standardize_crop_u8: null pointer");
  LEA_CHECK_ARG(B > 0 && H > 0 && W > 0 && crop_h > 0 && crop_w > 0,
                "lea_standardize_crop_u8: bad shape B=%d H=%d W=%d crop %dx%d", B, H, W, crop_h,
                crop_w);
  LEA_CHECK_ARG(pix_stride >= 3 && pix_stride <= 4,
                "lea_standardize_crop_u8: pixel stride %d (RGB = 3, RGBA = 4)", pix_stride);
  LEA_CHECK_ARG((long long)H * W < (1LL << 31) && (long long)crop_h * crop_w < (1LL << 31),
                "lea_standardize_crop_u8: image too large");
  const bool pad = H <= crop_h && W <= crop_w;
  // predict.py:150-158: the crop branch slices [start, start + crop) and copies it
  // into a [crop] array, which fails unless both sides are at least the crop
  LEA_CHECK_ARG(pad || (H >= crop_h && W >= crop_w),
                "test_transform: a %dx%d image neither fits a %dx%d crop nor covers it "
                "(the reference's copy into the crop fails)", H, W, crop_h, crop_w);
  hipStream_t st = as_stream(stream);
  const long long npix = (long long)H * W;
  if (hipMemsetAsync(workspace, 0, lea_standardize_workspace_bytes(B), st) != hipSuccess)
    return launch_status("lea_standardize_crop_u8 (workspace clear)");
  long long g = (npix + kStatThreads * 16 - 1) / (kStatThreads * 16);
  g = g > 1024 ? 1024 : g;
  // every thread must see < 2^23 pixels so its 32-bit sum of uint8 cannot overflow
  const long long gmin = (npix + ((long long)kStatThreads << 23) - 1) / ((long long)kStatThreads << 23);
  g = g < gmin ? gmin : g;
  u8_stats_kernel<<<dim3((unsigned)g, 2 * B), kStatThreads, 0, st>>>(
      (const uint8_t*)left, (const uint8_t*)right, B, npix, pix_stride,
      (unsigned long long*)workspace);
  int rc = launch_status("lea_standardize_crop_u8 (stats)");
  if (rc) return rc;
  const long long quads = (long long)crop_h * ((crop_w + 3) / 4);
  const int gx = (int)((quads + 256 * 2 - 1) / (256 * 2));
  u8_standardize_kernel<<<dim3(gx, 2 * B), 256, 0, st>>>(
      (const uint8_t*)left, (const uint8_t*)right, B, H, W, pix_stride,
      (const unsigned long long*)workspace, out_left, out_right, crop_h, crop_w, pad ? 1 : 0);
  return launch_status("lea_standardize_crop_u8");
}

extern "C" size_t lea_disparity_metrics_workspace_bytes(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  return (size_t)B * lea::metric_blocks((long long)H * W) * lea::kMetFields * sizeof(double);
}

extern "C" int lea_disparity_metrics(const float* pred, int64_t pred_bstride, const float* gt,
                                     int64_t gt_bstride, int B, int H, int W, float maxdisp,
                                     int round_pred, int z_shift, int thr1, int thr2, int thr3,
                                     unsigned char* correct, double* out, void* workspace,
                                     void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(pred && gt && out && workspace, "lea_disparity_metrics: null pointer");
  LEA_CHECK_ARG(B > 0 && H > 0 && W > 0 && (long long)H * W < (1LL << 31),
                "lea_disparity_metrics: bad shape B=%d H=%d W=%d", B, H, W);
  MetricArgs a;
  a.pred = pred;
  a.pbs = pred_bstride;
  a.gt = gt;
  a.gbs = gt_bstride;
  a.correct = correct;
  a.partial = (double*)workspace;
  a.npix = H * W;
  a.maxdisp = maxdisp;
  a.round_pred = round_pred;
  a.z_shift = z_shift;
  a.thr[0] = thr1;
  a.thr[1] = thr2;
  a.thr[2] = thr3;
  const int G = metric_blocks(a.npix);
  hipStream_t st = as_stream(stream);
  metrics_partial_kernel<<<dim3(G, B), kMetThreads, 0, st>>>(a);
  int rc = launch_status("lea_disparity_metrics");
  if (rc) return rc;
  metrics_final_kernel<<<B, 256, 0, st>>>(a.partial, G, out);
  return launch_status("lea_disparity_metrics (final)");
}
