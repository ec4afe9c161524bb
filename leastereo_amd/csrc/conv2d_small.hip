// Feature-net cell ConvBR2d 3x3 / s1 / p1 with few channels (cin <= 16, cout <= 32):
// models/operations_2d.py:31-47 as the 2D cells of retrain/new_model_2d.py:41-75 use it
// (8 channels at 1/3 resolution, 16 at 1/6, sibling groups up to 32 outputs).
//
// These convs are 0.1-0.6 GFLOP on a few-MB map: the DMA / MFMA engine's staging pipeline
// (4-channel chunks, a K of 36 per chunk) spent 9-17 us per launch on them, latency, not
// work.  Here a workgroup stages its (TH + 2) x 34 input halo of every channel in LDS once
// and each thread runs the whole 9 * cin dot product for one pixel and 8 output channels on
// the VALU.  The weights come from the same packed buffer the MFMA engine reads
// (PackCfg<3, MT, 1>: [chunk][tap][ci % 4][COP] with the 16-column swizzle of odd rows when
// COP % 32 == 0), staged once per workgroup as [ci][tap][co] and read as wave-uniform
// 16-byte LDS broadcasts (scalar loads of them -- 72-144 dependent s_loads per wave --
// ran 3-4x slower than the engine).
//
// Workgroup = 256 threads = 32 columns x TH rows x NG groups of 8 output channels
// (TH = 8 / NG), so the waves of one workgroup share the halo and every wave's 8 couts are
// uniform (NG = 1, 2, 4 for cout <= 8, 16, 32).  Same epilogue as the engine: folded BN,
// ReLU, then the residual (the cell's sum / skip term).
#include <algorithm>

#include "common.h"
#include "conv3d_impl.h"

namespace lea {

constexpr int kSmallTW = 32;         // output columns per workgroup
constexpr int kSmallRS = kSmallTW + 2;  // staged row stride (floats)

template <int CIN, int NG>
__global__ __launch_bounds__(256) void conv2d_small_kernel(const ConvArgs a) {
  constexpr int TH = 8 / NG;
  constexpr int MT = NG == 4 ? 2 : 1;
  using P = PackCfg<3, MT, 1>;
  constexpr int PL = (TH + 2) * kSmallRS;  // staged floats per channel
  constexpr int CO8 = NG * 8;              // output channels per workgroup
  __shared__ float xs[CIN * PL];
  __shared__ __attribute__((aligned(16))) float ws[CIN * 9 * CO8];  // [ci][tap][co]
  __shared__ float ss[2 * CO8];  // folded BN scale / shift of the workgroup's couts
  const int tid = threadIdx.x;
  const int tx = tid & 31;
  const int rest = tid >> 5;
  const int ty = rest % TH;
  const int cg = __builtin_amdgcn_readfirstlane(rest / TH);  // wave-uniform: 64 lanes = 2 rests
  const int b = blockIdx.z;
  const int w0 = blockIdx.x * kSmallTW, h0 = blockIdx.y * TH;
  const long long HW = (long long)a.H * a.W;
  const float* xb = a.x + (long long)b * a.xbs;
  // every load of the stage in flight at once (a rolled loop waited for each in turn)
  float xv[(CIN * PL + 255) / 256];
#pragma unroll
  for (int k = 0; k < (CIN * PL + 255) / 256; ++k) {
    const int e = tid + 256 * k;
    const int ci = e / PL, r = e - ci * PL;
    const int rr = r / kSmallRS, cc = r - rr * kSmallRS;
    const int h = h0 - 1 + rr, w = w0 - 1 + cc;
    const bool ok = e < CIN * PL && ci < a.cin && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
    // branch-free: every lane loads an in-range address, the padding lanes select 0
    const int cic = min(ci, a.cin - 1), hc = min(max(h, 0), a.H - 1), wc = min(max(w, 0), a.W - 1);
    const float v = xb[cic * HW + (long long)hc * a.W + wc];
    xv[k] = ok ? v : 0.f;
  }
  float wv[(CIN * 9 * CO8 + 255) / 256];
#pragma unroll
  for (int k = 0; k < (CIN * 9 * CO8 + 255) / 256; ++k) {
    const int e = min(tid + 256 * k, CIN * 9 * CO8 - 1);
    const int co = e % CO8, q = e / CO8, tap = q % 9, ci = q / 9;
    const int ch = ci / P::CIN_B, cb = ci % P::CIN_B;
    const int col = (P::SWZ && (cb & 1)) ? (co ^ 16) : co;
    wv[k] = a.wp[((ch * 9 + tap) * P::CIN_B + cb) * P::COP + col];
  }
  if (tid < 2 * CO8) {
    const int coc = min(tid % CO8, a.cout - 1);
    ss[tid] = a.scale ? (tid < CO8 ? a.scale[coc] : a.shift[coc]) : (tid < CO8 ? 1.f : 0.f);
  }
#pragma unroll
  for (int k = 0; k < (CIN * PL + 255) / 256; ++k)
    if (tid + 256 * k < CIN * PL) xs[tid + 256 * k] = xv[k];
#pragma unroll
  for (int k = 0; k < (CIN * 9 * CO8 + 255) / 256; ++k)
    if (tid + 256 * k < CIN * 9 * CO8) ws[tid + 256 * k] = wv[k];
  __syncthreads();
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const float* xp = xs + ty * kSmallRS + tx;
  const float4* wq = reinterpret_cast<const float4*>(ws) + cg * 2;  // this wave's 8 couts
  // one channel per iteration (unrolled, the compiler hoisted every LDS read: 512 VGPRs)
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float v = xp[ci * PL + (tap / 3) * kSmallRS + tap % 3];
      // one address per wave: LDS broadcast
      const float4 wa = wq[(ci * 9 + tap) * (CO8 / 4)], wb = wq[(ci * 9 + tap) * (CO8 / 4) + 1];
      const float wr[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(wr[j], v, acc[j]);
    }
  }
  const int h = h0 + ty, w = w0 + tx;
  // lea_conv2d_bnrelu_pair: this wave's 8 couts belong to the second conv (uniform: csplit % 8 == 0)
  const bool second = a.csplit > 0 && cg * 8 >= a.csplit;
  const bool relu = a.flags & LEA_RELU, resid = (a.flags & LEA_RESIDUAL) && !second;
  const long long pix = (long long)min(h, a.H - 1) * a.W + min(w, a.W - 1);
  // the residuals' loads all issued before the first use (clamped, in range)
  float rv[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int coc = min(cg * 8 + j, a.cout - 1);
    sc[j] = ss[cg * 8 + j];  // (staged: scalar loads of them were sunk below the stores)
    sh[j] = ss[CO8 + cg * 8 + j];
    rv[j] = resid ? a.res[(long long)b * a.rbs + coc * HW + pix] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = acc[j];
    v = v * sc[j] + sh[j];
    if (relu) v = fmaxf(v, 0.f);
    acc[j] = resid ? v + rv[j] : v;
  }
  // stores last: none of the loads above may be ordered after one (y may alias them)
  if (h >= a.H || w >= a.W) return;
  float* yp = second ? a.y2 + (long long)b * a.y2bs + pix - (long long)a.csplit * HW : a.y + (long long)b * a.ybs + pix;
  if (cg * 8 + 8 <= a.cout) {  // (uniform) the whole group: one block of 8 stores
#pragma unroll
    for (int j = 0; j < 8; ++j) yp[(cg * 8 + j) * HW] = acc[j];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (cg * 8 + j < a.cout) yp[(cg * 8 + j) * HW] = acc[j];
  }
}

int g_conv2d_small = 1;  // lea_conv2d_set_small

bool conv2d_small_ok(int cin, int cout) { return g_conv2d_small && cin <= 16 && cout <= 32; }

static int ng_of(int cout) { return cout <= 8 ? 1 : cout <= 16 ? 2 : 4; }

const char* conv2d_small_name(int cin, int cout) {
  static thread_local char name[64];
  snprintf(name, sizeof(name), "conv2d_small_kernel<%d, %d>", (cin + 3) / 4 * 4, ng_of(cout));
  return name;
}

int run_conv2d_small(const ConvArgs& a, int B, hipStream_t st) {
  const int ng = ng_of(a.cout), cin4 = (a.cin + 3) / 4 * 4, th = 8 / ng;
  LEA_CHECK_ARG(B <= 65535 && (a.H + th - 1) / th <= 65535, "lea_conv2d: grid too large");
  const dim3 grid((a.W + kSmallTW - 1) / kSmallTW, (a.H + th - 1) / th, B);
#define LEA_SMALL2D(CI, G)                                                      \
  if (cin4 == CI && ng == G) {                                                  \
    conv2d_small_kernel<CI, G><<<grid, 256, 0, st>>>(a);                        \
    return launch_status("lea_conv2d(small)");                                  \
  }
  LEA_SMALL2D(4, 1) LEA_SMALL2D(4, 2) LEA_SMALL2D(4, 4)
  LEA_SMALL2D(8, 1) LEA_SMALL2D(8, 2) LEA_SMALL2D(8, 4)
  LEA_SMALL2D(12, 1) LEA_SMALL2D(12, 2) LEA_SMALL2D(12, 4)
  LEA_SMALL2D(16, 1) LEA_SMALL2D(16, 2) LEA_SMALL2D(16, 4)
#undef LEA_SMALL2D
  set_error("lea_conv2d(small): cin=%d cout=%d", a.cin, a.cout);
  return LEA_E_UNSUPPORTED;
}

}  // namespace lea

extern "C" int lea_conv2d_set_small(int on) {
  lea::clear_error();
  if (on != 0 && on != 1) {
    lea::set_error("lea_conv2d_set_small: on=%d", on);
    return LEA_E_INVALID;
  }
  lea::g_conv2d_small = on;
  return 0;
}

extern "C" int lea_conv2d_bnrelu_pair(const void* x, int64_t x_bstride, const float* w_packed,
                                      const float* scale, const float* shift, const void* residual,
                                      int64_t r_bstride, void* y, int64_t y_bstride, void* y2, int64_t y2_bstride,
                                      int B, int cin, int cout, int c1, int H, int W, unsigned flags,
                                      void* stream) {
  using namespace lea;
  clear_error();
  ConvArgs a{};
  a.x = (const float*)x;
  a.xbs = x_bstride;
  a.cin1 = cin;
  a.wp = w_packed;
  a.scale = scale;
  a.shift = shift;
  a.res = (const float*)residual;
  a.rbs = r_bstride;
  a.y = (float*)y;
  a.ybs = y_bstride;
  a.y2 = (float*)y2;
  a.y2bs = y2_bstride;
  a.csplit = c1;
  a.cin = cin;
  a.cout = cout;
  a.D = 1;
  a.H = H;
  a.W = W;
  a.flags = flags;
  LEA_CHECK_ARG(a.x && a.wp && a.y && a.y2, "lea_conv2d_bnrelu_pair: null pointer");
  LEA_CHECK_ARG((a.scale == nullptr) == (a.shift == nullptr),
                "lea_conv2d_bnrelu_pair: scale/shift must both be set or both NULL");
  LEA_CHECK_FLAGS(flags, LEA_RELU | LEA_RESIDUAL, "lea_conv2d_bnrelu_pair");
  LEA_CHECK_ARG(!(flags & LEA_RESIDUAL) || a.res, "lea_conv2d_bnrelu_pair: LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && cin > 0 && H > 0 && W > 0 && c1 > 0 && c1 < cout && c1 % 8 == 0,
                "lea_conv2d_bnrelu_pair: bad shape B=%d cin=%d cout=%d c1=%d H=%d W=%d", B, cin, cout, c1, H, W);
  LEA_CHECK_ARG((long long)(cout + 63) * H * W < (1LL << 31), "lea_conv2d_bnrelu_pair: plane too large");
  LEA_CHECK_ARG(a.x != a.y && a.x != a.y2, "lea_conv2d_bnrelu_pair: input aliases an output");
  if (cin > 16 || cout > 32) {  // the few-channel tile only (conv2d_small_ok's shapes, always on here)
    set_error("lea_conv2d_bnrelu_pair: cin=%d cout=%d beyond the few-channel tile", cin, cout);
    return LEA_E_UNSUPPORTED;
  }
  return run_conv2d_small(a, B, as_stream(stream));
}

extern "C" const char* lea_conv2d_kernel_name_cin(int B, int cin, int cout, int H, int W) {
  if (B <= 0 || cin <= 0 || cout <= 0 || H <= 0 || W <= 0) return nullptr;
  if (lea::conv2d_small_ok(cin, cout)) return lea::conv2d_small_name(cin, cout);
  return lea_conv2d_kernel_name(B, cout, H, W);
}
