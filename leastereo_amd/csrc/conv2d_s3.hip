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
#include <algorithm>

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

// ---- backward (train.py:130-178 through new_model_2d.py:94) ----
// The tiling above makes the transposed conv a gather with one tap per input pixel:
// input row y is read only by output row oy = (y + 1) / 3 at kernel row kh = (y + 1) % 3
// (columns alike), so
//   dx[b][ci][y][x] = sum_co w[co][ci][kh(y)][kw(x)] * dz[b][co][oy(y)][ox(x)]
// (0 where oy = Ho: the last row when Hi % 3 == 0 is read by no output; columns alike).
// One thread per input pixel and 16 channels.
constexpr int kS3CiBlock = 16;

__global__ __launch_bounds__(256) void conv2d_s3_dgrad_kernel(const float* __restrict__ dz, const float* __restrict__ w,
                                                              float* __restrict__ dx, int cin, int cout, int Hi,
                                                              int Wi, int Ho, int Wo) {
  const int b = blockIdx.z, ci0 = blockIdx.y * kS3CiBlock;
  const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (long long)Hi * Wi) return;
  const int y = (int)(pix / Wi), x = (int)(pix - (long long)y * Wi);
  const int oy = (y + 1) / 3, ox = (x + 1) / 3, t = ((y + 1) % 3) * 3 + (x + 1) % 3;
  const bool read = oy < Ho && ox < Wo;
  const float* g = dz + ((long long)b * cout * Ho + (read ? oy : 0)) * Wo + (read ? ox : 0);
  const long long HWo = (long long)Ho * Wo;
  float acc[kS3CiBlock];
#pragma unroll
  for (int j = 0; j < kS3CiBlock; ++j) acc[j] = 0.f;
  for (int co = 0; co < (read ? cout : 0); ++co) {
    const float gv = g[co * HWo];
    const float* wc = w + (long long)co * cin * 9 + t;
#pragma unroll
    for (int j = 0; j < kS3CiBlock; ++j)
      if (ci0 + j < cin) acc[j] = fmaf(wc[(ci0 + j) * 9], gv, acc[j]);
  }
  float* o = dx + ((long long)b * cin + ci0) * Hi * Wi + pix;
#pragma unroll
  for (int j = 0; j < kS3CiBlock; ++j)
    if (ci0 + j < cin) o[(long long)j * Hi * Wi] = acc[j];
}

// dw[co][ci][kh][kw] = sum_{b, oy, ox} dz[b][co][oy][ox] * x[b][ci][3 oy + kh - 1][3 ox + kw - 1]:
// workgroup (K slice s, 16-channel chunk, 16-cout block) walks 64-pixel tiles of its slice,
// staging dz[16][64] and the 16 x 9 patch values per pixel in LDS ([pixel][element]: the
// lanes of a read take consecutive elements, distinct banks); thread e owns elements
// e + 256 k of the block's 16 x 144, accumulates over its tiles and writes one partial;
// a second kernel sums the slices in order (deterministic).
constexpr int kS3Tile = 64, kS3Elems = kS3CoBlock * kS3CiBlock * 9, kS3Per = kS3Elems / 256;
static_assert(kS3Elems % 256 == 0, "elements per thread");

__global__ __launch_bounds__(256) void conv2d_s3_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                              float* __restrict__ part, int B, int cin, int cout,
                                                              int Hi, int Wi, int Ho, int Wo, int ntile) {
  __shared__ float xs[kS3Tile][kS3CiBlock * 9 + 1];
  __shared__ float gs[kS3Tile][kS3CoBlock + 1];
  const int tid = threadIdx.x, s = blockIdx.x, ns = gridDim.x;
  const int ci0 = blockIdx.y * kS3CiBlock, co0 = blockIdx.z * kS3CoBlock;
  const long long HWo = (long long)Ho * Wo, HWi = (long long)Hi * Wi, npix = (long long)B * HWo;
  float acc[kS3Per];
#pragma unroll
  for (int k = 0; k < kS3Per; ++k) acc[k] = 0.f;
  for (int tl = s; tl < ntile; tl += ns) {
    const long long p0 = (long long)tl * kS3Tile;
    __syncthreads();
    for (int e = tid; e < kS3Tile * kS3CiBlock * 9; e += 256) {
      const int j = e / (kS3CiBlock * 9), r = e - j * (kS3CiBlock * 9), c = ci0 + r / 9, t = r % 9;
      const long long p = p0 + j;
      float v = 0.f;
      if (p < npix && c < cin) {
        const int b = (int)(p / HWo), q = (int)(p - (long long)b * HWo), oy = q / Wo, ox = q - oy * Wo;
        const int yy = 3 * oy + t / 3 - 1, xx = 3 * ox + t % 3 - 1;
        if ((unsigned)yy < (unsigned)Hi && (unsigned)xx < (unsigned)Wi)
          v = x[((long long)b * cin + c) * HWi + (long long)yy * Wi + xx];
      }
      xs[j][r] = v;
    }
    for (int e = tid; e < kS3Tile * kS3CoBlock; e += 256) {
      const int j = e % kS3Tile, co = co0 + e / kS3Tile;
      const long long p = p0 + j;
      float v = 0.f;
      if (p < npix && co < cout) {
        const int b = (int)(p / HWo);
        v = dz[((long long)b * cout + co) * HWo + (p - (long long)b * HWo)];
      }
      gs[j][e / kS3Tile] = v;
    }
    __syncthreads();
    for (int j = 0; j < kS3Tile; ++j) {
#pragma unroll
      for (int k = 0; k < kS3Per; ++k) {
        const int e = tid + 256 * k, co = e / (kS3CiBlock * 9), r = e - co * (kS3CiBlock * 9);
        acc[k] = fmaf(gs[j][co], xs[j][r], acc[k]);
      }
    }
  }
  // partial s: [cout][cin][9] slots of this block's (co, ci) range
#pragma unroll
  for (int k = 0; k < kS3Per; ++k) {
    const int e = tid + 256 * k, co = co0 + e / (kS3CiBlock * 9), r = e % (kS3CiBlock * 9), c = ci0 + r / 9;
    if (co < cout && c < cin) part[((long long)s * cout + co) * cin * 9 + (long long)c * 9 + r % 9] = acc[k];
  }
}

__global__ void conv2d_s3_wgrad_sum_kernel(const float* __restrict__ part, float* __restrict__ dw, long long n, int ns) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < ns; ++s) v += part[(long long)s * n + i];
    dw[i] = v;
  }
}

inline int s3_wgrad_split(int B, int Ho, int Wo) {
  const long long ntile = ((long long)B * Ho * Wo + kS3Tile - 1) / kS3Tile;
  return (int)std::max(1LL, std::min(ntile, 256LL));
}

}  // namespace lea

extern "C" int lea_conv2d_s3_bnrelu(const void* x, int64_t x_bstride, const float* w,
                                    const float* scale, const float* shift, void* y,
                                    int64_t y_bstride, int B, int cin, int cout, int Hi, int Wi,
                                    unsigned flags, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_conv2d_s3_bnrelu");
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

extern "C" int lea_conv2d_s3_backward_data(const float* dz, const float* w, float* dx, int B, int cin, int cout,
                                           int Hi, int Wi, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(dz && w && dx && dz != dx, "lea_conv2d_s3_backward_data: null or aliased pointer");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && Hi > 0 && Wi > 0 && B <= 65535 &&
                    (cin + kS3CiBlock - 1) / kS3CiBlock <= 65535 && (long long)cin * Hi * Wi < (1LL << 31),
                "lea_conv2d_s3_backward_data: bad shape B=%d cin=%d cout=%d Hi=%d Wi=%d", B, cin, cout, Hi, Wi);
  const int Ho = (Hi - 1) / 3 + 1, Wo = (Wi - 1) / 3 + 1;
  dim3 grid((unsigned)(((long long)Hi * Wi + 255) / 256), (cin + kS3CiBlock - 1) / kS3CiBlock, B);
  conv2d_s3_dgrad_kernel<<<grid, 256, 0, as_stream(stream)>>>(dz, w, dx, cin, cout, Hi, Wi, Ho, Wo);
  return launch_status("lea_conv2d_s3_backward_data");
}

extern "C" size_t lea_conv2d_s3_wgrad_workspace_bytes(int B, int cin, int cout, int Hi, int Wi) {
  using namespace lea;
  if (B <= 0 || cin <= 0 || cout <= 0 || Hi <= 0 || Wi <= 0) return 0;
  const int Ho = (Hi - 1) / 3 + 1, Wo = (Wi - 1) / 3 + 1;
  return (size_t)s3_wgrad_split(B, Ho, Wo) * cout * cin * 9 * sizeof(float);
}

extern "C" int lea_conv2d_s3_wgrad(const float* x, const float* dz, float* dw, void* workspace, size_t ws_bytes,
                                   int B, int cin, int cout, int Hi, int Wi, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(x && dz && dw && workspace, "lea_conv2d_s3_wgrad: null pointer");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && Hi > 0 && Wi > 0 && (long long)B * cin * Hi * Wi < (1LL << 40),
                "lea_conv2d_s3_wgrad: bad shape");
  const size_t need = lea_conv2d_s3_wgrad_workspace_bytes(B, cin, cout, Hi, Wi);
  LEA_CHECK_ARG(ws_bytes >= need, "lea_conv2d_s3_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  const int Ho = (Hi - 1) / 3 + 1, Wo = (Wi - 1) / 3 + 1;
  const int ns = s3_wgrad_split(B, Ho, Wo);
  const int ntile = (int)(((long long)B * Ho * Wo + kS3Tile - 1) / kS3Tile);
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)ns, (cin + kS3CiBlock - 1) / kS3CiBlock, (cout + kS3CoBlock - 1) / kS3CoBlock);
  conv2d_s3_wgrad_kernel<<<grid, 256, 0, st>>>(x, dz, (float*)workspace, B, cin, cout, Hi, Wi, Ho, Wo, ntile);
  const int rc = launch_status("lea_conv2d_s3_wgrad");
  if (rc) return rc;
  const long long n = (long long)cout * cin * 9;
  conv2d_s3_wgrad_sum_kernel<<<(unsigned)std::min<long long>((n + 255) / 256, 1024), 256, 0, st>>>(
      (const float*)workspace, dw, n, ns);
  return launch_status("lea_conv2d_s3_wgrad(sum)");
}
