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
// Separable evaluation, two launches (r01: one 27-tap trilinear gather per voxel
// issued 216 loads per output and ran at 0.4 TB/s):
//   pass 1  Y[d][kh,kw](hi, wi) = sum_kd  lerp_d(Q[kd,kh,kw])(d + kd - 1)   low-res h, w
//   pass 2  out(d, h, w)        = sum_kh,kw  bilerp(Y[d][kh,kw])(h + kh - 1, w + kw - 1)
// (taps outside the output volume skipped), i.e. 6 loads per Y element and 36 per
// output voxel.  Y (B*cout*Do*9*Hi*Wi floats) lives in a caller-provided workspace
// (lea_tapsum_workspace_bytes).  Same sums in a different association order.
#include "common.h"

using bf16x8_t = __attribute__((ext_vector_type(8))) __bf16;

namespace lea {

// pass 1: grid (quads of one low-res plane, (b, co, d, kh*3+kw)); float4 when Wi % 4 == 0
template <bool VEC>
__global__ __launch_bounds__(256) void tapsum_dpass_f32(const float* __restrict__ q, long long qbs,
                                                        float* __restrict__ ws, int cout, int Di,
                                                        int Hi, int Wi, int Do, float rd) {
#pragma clang fp contract(off)
  int r = blockIdx.y;  // ((b * cout + co) * Do + d) * 9 + khw
  const int khw = r % 9;
  r /= 9;
  const int d = r % Do;
  r /= Do;
  const int co = r % cout;
  const int b = r / cout;
  const long long HWi = (long long)Hi * Wi;
  const long long vol = HWi * Di;
  const float* qb = q + (long long)b * qbs + ((long long)co * 27 + khw) * vol;
  float* yo = ws + (long long)blockIdx.y * HWi;
  const int n = VEC ? (int)(HWi / 4) : (int)HWi;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float acc[VEC ? 4 : 1] = {};
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      const int pd = d + kd - 1;
      if ((unsigned)pd >= (unsigned)Do) continue;
      const Axis ad = axis_index(rd, pd, Di, Do, 1);
      const float* q0 = qb + (long long)kd * 9 * vol + ad.i0 * HWi;
      const float* q1 = qb + (long long)kd * 9 * vol + ad.i1 * HWi;
      if constexpr (VEC) {
        const float4 a = reinterpret_cast<const float4*>(q0)[i];
        const float4 c = reinterpret_cast<const float4*>(q1)[i];
        acc[0] += ad.l0 * a.x + ad.l1 * c.x;
        acc[1] += ad.l0 * a.y + ad.l1 * c.y;
        acc[2] += ad.l0 * a.z + ad.l1 * c.z;
        acc[3] += ad.l0 * a.w + ad.l1 * c.w;
      } else {
        acc[0] += ad.l0 * q0[i] + ad.l1 * q1[i];
      }
    }
    if constexpr (VEC)
      reinterpret_cast<float4*>(yo)[i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    else
      yo[i] = acc[0];
  }
}

// pass 1 with q in the bf16 c8 layout (dtype LEA_BF16): one thread per low-res
// voxel and output plane d computes all 9 (kh, kw) partial sums; the 9 channels
// co*27 + kd*9 + (0..8) of one kd span exactly two 16-byte channel words, so each
// (kd, source plane) costs two vector loads.  OFF = (co*27 + kd*9) % 8 is uniform
// per workgroup and selects a specialised unpacking.
template <int OFF>
__device__ __forceinline__ void tapsum_acc9(float (&acc)[9], const bf16x8_t& a0, const bf16x8_t& a1,
                                            const bf16x8_t& b0, const bf16x8_t& b1, float l0, float l1) {
#pragma clang fp contract(off)
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int c = OFF + k;
    const float v0 = c < 8 ? (float)a0[c] : (float)a1[c - 8];
    const float v1 = c < 8 ? (float)b0[c] : (float)b1[c - 8];
    acc[k] += l0 * v0 + l1 * v1;
  }
}

__global__ __launch_bounds__(256) void tapsum_dpass_c8(const __bf16* __restrict__ q, long long qbs,
                                                       float* __restrict__ ws, int cout, int Di,
                                                       int Hi, int Wi, int Do, float rd) {
  const int r = blockIdx.y;  // (b * cout + co) * Do + d
  const int d = r % Do;
  const int bc = r / Do;
  const int co = bc % cout, b = bc / cout;
  const long long HWi = (long long)Hi * Wi;
  const long long vol = HWi * Di;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HWi) return;
  const bf16x8_t* qw = reinterpret_cast<const bf16x8_t*>(q + (long long)b * qbs);
  float acc[9] = {};
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int pd = d + kd - 1;
    if ((unsigned)pd >= (unsigned)Do) continue;
    const Axis ad = axis_index(rd, pd, Di, Do, 1);
    const int cb = co * 27 + kd * 9;
    const bf16x8_t* blk0 = qw + (long long)(cb / 8) * vol;
    const bf16x8_t* blk1 = blk0 + vol;  // next channel word (always exists: 27*cout padded to 8)
    const bf16x8_t a0 = blk0[ad.i0 * HWi + i], a1 = blk1[ad.i0 * HWi + i];
    const bf16x8_t b0 = blk0[ad.i1 * HWi + i], b1 = blk1[ad.i1 * HWi + i];
    switch (cb % 8) {
      case 0: tapsum_acc9<0>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 1: tapsum_acc9<1>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 2: tapsum_acc9<2>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 3: tapsum_acc9<3>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 4: tapsum_acc9<4>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 5: tapsum_acc9<5>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      case 6: tapsum_acc9<6>(acc, a0, a1, b0, b1, ad.l0, ad.l1); break;
      default: tapsum_acc9<7>(acc, a0, a1, b0, b1, ad.l0, ad.l1);
    }
  }
  float* yo = ws + (long long)r * 9 * HWi + i;
#pragma unroll
  for (int k = 0; k < 9; ++k) yo[k * HWi] = acc[k];
}

// pass 2: one workgroup per output row (b, co, d, h); lanes along w
__global__ __launch_bounds__(512) void tapsum_hwpass_f32(
    const float* __restrict__ ws, float* __restrict__ y, long long ybs, int cout, int Hi, int Wi,
    int Do, int Ho, int Wo, float rh, float rw, const float* __restrict__ scale,
    const float* __restrict__ shift, unsigned flags) {
#pragma clang fp contract(off)
  const int row = blockIdx.x;  // ((b * cout + co) * Do + d) * Ho + h
  const int h = row % Ho;
  const int plane = row / Ho;  // (b * cout + co) * Do + d
  const int co = (plane / Do) % cout;
  const int b = plane / (Do * cout);
  const int d = plane % Do;
  const long long HWi = (long long)Hi * Wi;
  const float* yp = ws + (long long)plane * 9 * HWi;
  Axis ah[3];
  bool hok[3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int p = h + kh - 1;
    hok[kh] = (unsigned)p < (unsigned)Ho;
    ah[kh] = axis_index(rh, hok[kh] ? p : 0, Hi, Ho, 1);
  }
  for (int w = threadIdx.x; w < Wo; w += blockDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int p = w + kw - 1;
      if ((unsigned)p >= (unsigned)Wo) continue;
      const Axis aw = axis_index(rw, p, Wi, Wo, 1);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        if (!hok[kh]) continue;
        const float* t = yp + (long long)(kh * 3 + kw) * HWi;
        const float* r0 = t + (long long)ah[kh].i0 * Wi;
        const float* r1 = t + (long long)ah[kh].i1 * Wi;
        acc += ah[kh].l0 * (aw.l0 * r0[aw.i0] + aw.l1 * r0[aw.i1]) +
               ah[kh].l1 * (aw.l0 * r1[aw.i0] + aw.l1 * r1[aw.i1]);
      }
    }
    if (scale) acc = acc * scale[co] + shift[co];
    if (flags & LEA_RELU) acc = fmaxf(acc, 0.f);
    y[(long long)b * ybs + (((long long)co * Do + d) * Ho + h) * Wo + w] = acc;
  }
}

// pass 2's output phase: R output rows (h0..h1) of plane (b, co, d) from the staged rows
// [9][nrmax][Wi] (low-res rows r_lo..), 36 LDS corner values per output
__device__ __forceinline__ void tapsum_rows_out(const float* __restrict__ rows, float* __restrict__ y, long long ybs,
                                                int b, int co, int d, int h0, int h1, int r_lo, bool over, int nrmax,
                                                int Wi, int Do, int Ho, int Wo, float rh, float rw, int Hi,
                                                const float* __restrict__ scale, const float* __restrict__ shift,
                                                unsigned flags) {
#pragma clang fp contract(off)
  const float sc = scale ? scale[co] : 1.f, sh = scale ? shift[co] : 0.f;
  const int cells = (h1 - h0) * Wo;
  for (int t = threadIdx.x; t < cells; t += blockDim.x) {
    const int h = h0 + t / Wo, w = t % Wo;
    Axis ah[3];
    bool hok[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int p = h + kh - 1;
      hok[kh] = (unsigned)p < (unsigned)Ho;
      ah[kh] = axis_index(rh, hok[kh] ? p : 0, Hi, Ho, 1);
    }
    float acc = 0.f;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int p = w + kw - 1;
      if ((unsigned)p >= (unsigned)Wo) continue;
      const Axis aw = axis_index(rw, p, Wi, Wo, 1);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        if (!hok[kh]) continue;
        const float* tm = rows + (kh * 3 + kw) * nrmax * Wi;
        const float* r0 = tm + (over ? 0 : ah[kh].i0 - r_lo) * Wi;
        const float* r1 = tm + (over ? 0 : ah[kh].i1 - r_lo) * Wi;
        acc += ah[kh].l0 * (aw.l0 * r0[aw.i0] + aw.l1 * r0[aw.i1]) +
               ah[kh].l1 * (aw.l0 * r1[aw.i0] + aw.l1 * r1[aw.i1]);
      }
    }
    if (scale) acc = acc * sc + sh;
    if (flags & LEA_RELU) acc = fmaxf(acc, 0.f);
    y[(long long)b * ybs + (((long long)co * Do + d) * Ho + h) * Wo + w] = over ? __builtin_nanf("") : acc;
  }
}

// pass 2, row-staged (r03): a workgroup owns R output rows of one plane; the <= nrmax
// low-res rows of the 9 (kh, kw) maps they read are copied into LDS once (coalesced),
// then every output sums its 36 corner values from LDS instead of gathering them through
// the L1 (36 loads per output).  Same expression and order as tapsum_hwpass_f32: the two
// produce identical bits.
__global__ __launch_bounds__(256) void tapsum_hwpass_rows_f32(
    const float* __restrict__ ws, float* __restrict__ y, long long ybs, int cout, int Hi, int Wi,
    int Do, int Ho, int Wo, float rh, float rw, const float* __restrict__ scale,
    const float* __restrict__ shift, unsigned flags, int R, int nrmax) {
#pragma clang fp contract(off)
  extern __shared__ float rows[];  // [9][nrmax][Wi]
  const int plane = blockIdx.y;    // (b * cout + co) * Do + d
  const int co = (plane / Do) % cout;
  const int b = plane / (Do * cout);
  const int d = plane % Do;
  const int h0 = blockIdx.x * R;
  const int h1 = min(h0 + R, Ho);
  const int r_lo = axis_index(rh, max(h0 - 1, 0), Hi, Ho, 1).i0;
  const int r_hi = axis_index(rh, min(h1, Ho - 1), Hi, Ho, 1).i1;
  // nrmax = the host's exact bound (staged_rows); past it: NaN outputs, never unstaged rows
  const bool over = r_hi - r_lo + 1 > nrmax;
  const int nr = over ? 0 : r_hi - r_lo + 1;
  const long long HWi = (long long)Hi * Wi;
  const float* yp = ws + (long long)plane * 9 * HWi + (long long)r_lo * Wi;
  const int n1 = nr * Wi;
  // eight loads in flight per batch (r04: the rolled loop waited for each load in turn)
  for (int e0 = threadIdx.x; e0 < 9 * n1; e0 += 8 * blockDim.x) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = min(e0 + j * (int)blockDim.x, 9 * n1 - 1);
      const int k = e / n1, r = e - k * n1;
      v[j] = yp[(long long)k * HWi + r];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = e0 + j * (int)blockDim.x;
      if (e < 9 * n1) {
        const int k = e / n1, r = e - k * n1;
        rows[k * nrmax * Wi + r] = v[j];
      }
    }
  }
  __syncthreads();
  tapsum_rows_out(rows, y, ybs, b, co, d, h0, h1, r_lo, over, nrmax, Wi, Do, Ho, Wo, rh, rw, Hi, scale, shift, flags);
}

// passes 1 + 2 in one launch (r05): a workgroup computes the pass-1 values of the <= nrmax
// low-res rows its R output rows read, for all 9 (kh, kw) maps, straight into LDS (same
// expression and kd order as tapsum_dpass_f32 / _c8: identical bits), then runs pass 2's
// output phase -- the 9-map workspace never goes through HBM.  Workgroups walk d fastest
// within (b, co, row block), XCD-contiguous, so the Q planes neighbouring d values share stay
// in L2.  C8: q in the bf16 c8 layout; else f32 NCDHW (VEC: float4 along Wi).
template <bool C8, bool VEC>
__global__ __launch_bounds__(256) void tapsum_fused(const void* __restrict__ qv, long long qbs,
                                                    float* __restrict__ y, long long ybs, int cout, int Di,
                                                    int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh,
                                                    float rw, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, unsigned flags, int R,
                                                    int nrmax, int nhb, int nblk) {
#pragma clang fp contract(off)
  extern __shared__ float rows[];  // [9][nrmax][Wi]
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int d = lin % Do;
  const int hb = (lin / Do) % nhb;
  const int bc = lin / (Do * nhb);  // b * cout + co
  const int co = bc % cout, b = bc / cout;
  const int h0 = hb * R;
  const int h1 = min(h0 + R, Ho);
  const int r_lo = axis_index(rh, max(h0 - 1, 0), Hi, Ho, 1).i0;
  const int r_hi = axis_index(rh, min(h1, Ho - 1), Hi, Ho, 1).i1;
  const bool over = r_hi - r_lo + 1 > nrmax;
  const int nr = over ? 0 : r_hi - r_lo + 1;
  const long long HWi = (long long)Hi * Wi;
  const long long vol = HWi * Di;
  Axis ad[3];
  bool dok[3];
#pragma unroll
  for (int kd = 0; kd < 3; ++kd) {
    const int pd = d + kd - 1;
    dok[kd] = (unsigned)pd < (unsigned)Do;
    ad[kd] = axis_index(rd, dok[kd] ? pd : 0, Di, Do, 1);
  }
  if constexpr (C8) {
    const bf16x8_t* qw = reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const __bf16*>(qv) + (long long)b * qbs);
    for (int e = threadIdx.x; e < nr * Wi; e += blockDim.x) {
      const long long pos = (long long)r_lo * Wi + e;  // (row r_lo + e / Wi, column e % Wi)
      float acc[9] = {};
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        if (!dok[kd]) continue;
        const int cb = co * 27 + kd * 9;
        const bf16x8_t* blk0 = qw + (long long)(cb / 8) * vol;
        const bf16x8_t* blk1 = blk0 + vol;
        const bf16x8_t a0 = blk0[ad[kd].i0 * HWi + pos], a1 = blk1[ad[kd].i0 * HWi + pos];
        const bf16x8_t b0 = blk0[ad[kd].i1 * HWi + pos], b1 = blk1[ad[kd].i1 * HWi + pos];
        switch (cb % 8) {
          case 0: tapsum_acc9<0>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 1: tapsum_acc9<1>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 2: tapsum_acc9<2>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 3: tapsum_acc9<3>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 4: tapsum_acc9<4>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 5: tapsum_acc9<5>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          case 6: tapsum_acc9<6>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1); break;
          default: tapsum_acc9<7>(acc, a0, a1, b0, b1, ad[kd].l0, ad[kd].l1);
        }
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) rows[k * nrmax * Wi + e] = acc[k];
    }
  } else {
    const float* qb = reinterpret_cast<const float*>(qv) + (long long)b * qbs + (long long)co * 27 * vol;
    constexpr int V = VEC ? 4 : 1;
    for (int e = threadIdx.x; e < nr * Wi / V; e += blockDim.x) {
      const long long pos = (long long)r_lo * Wi + (long long)e * V;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float acc[V] = {};
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          if (!dok[kd]) continue;
          const float* q0 = qb + (long long)(kd * 9 + k) * vol + ad[kd].i0 * HWi + pos;
          const float* q1 = qb + (long long)(kd * 9 + k) * vol + ad[kd].i1 * HWi + pos;
          if constexpr (VEC) {
            const float4 a = *reinterpret_cast<const float4*>(q0);
            const float4 c = *reinterpret_cast<const float4*>(q1);
            acc[0] += ad[kd].l0 * a.x + ad[kd].l1 * c.x;
            acc[1] += ad[kd].l0 * a.y + ad[kd].l1 * c.y;
            acc[2] += ad[kd].l0 * a.z + ad[kd].l1 * c.z;
            acc[3] += ad[kd].l0 * a.w + ad[kd].l1 * c.w;
          } else {
            acc[0] += ad[kd].l0 * q0[0] + ad[kd].l1 * q1[0];
          }
        }
#pragma unroll
        for (int j = 0; j < V; ++j) rows[k * nrmax * Wi + e * V + j] = acc[j];
      }
    }
  }
  __syncthreads();
  tapsum_rows_out(rows, y, ybs, b, co, d, h0, h1, r_lo, over, nrmax, Wi, Do, Ho, Wo, rh, rw, Hi, scale, shift, flags);
}

}  // namespace lea

// lea_tapsum_set_rows: 2 (default, r05) = passes 1 + 2 fused (tapsum_fused), 1 = the
// row-staged pass 2 after pass 1 through the workspace, each when R output rows' sources fit
// 64 KB of LDS; 0 = pass 1, then one workgroup per output row gathering through the L1
static int g_tapsum_rows = 2;
extern "C" int lea_tapsum_set_rows(int on) {
  lea::clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 2, "lea_tapsum_set_rows: %d", on);
  g_tapsum_rows = on;
  return 0;
}

static int hwpass(const float* ws, void* y, int64_t y_bstride, int B, int cout, int Hi, int Wi, int Do,
                  int Ho, int Wo, const float* scale, const float* shift, unsigned flags, hipStream_t st) {
  using namespace lea;
  const float rh = axis_ratio(Hi, Ho, 1), rw = axis_ratio(Wi, Wo, 1);
  if (g_tapsum_rows) {
    for (int R = 8; R >= 2; R /= 2) {
      // rows h0-1 .. h0+R of every block: the exact largest row count (common.h)
      const int nrmax = staged_rows(Hi, Ho, 1, R, 1);
      const size_t lds = (size_t)9 * nrmax * Wi * sizeof(float);
      if (lds > 65536) continue;
      dim3 g((unsigned)((Ho + R - 1) / R), (unsigned)(B * cout * Do));
      tapsum_hwpass_rows_f32<<<g, 256, lds, st>>>(ws, (float*)y, y_bstride, cout, Hi, Wi, Do, Ho, Wo, rh, rw,
                                                  scale, shift, flags, R, nrmax);
      return launch_status("lea_tapsum_upsample");
    }
  }
  const int threads = Wo >= 512 ? 512 : ((Wo + 63) / 64) * 64;  // one row per workgroup
  dim3 g2((unsigned)((long long)B * cout * Do * Ho));
  tapsum_hwpass_f32<<<g2, threads, 0, st>>>(ws, (float*)y, y_bstride, cout, Hi, Wi, Do, Ho, Wo, rh, rw, scale,
                                            shift, flags);
  return launch_status("lea_tapsum_upsample");
}

extern "C" size_t lea_tapsum_workspace_bytes(int B, int cout, int Hi, int Wi, int Do) {
  if (B <= 0 || cout <= 0 || Hi <= 0 || Wi <= 0 || Do <= 0) return 0;
  return (size_t)B * cout * Do * 9 * Hi * Wi * sizeof(float);
}

extern "C" int lea_tapsum_upsample(const void* q, int64_t q_bstride, void* y, int64_t y_bstride,
                                   int B, int cout, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                   const float* scale, const float* shift, unsigned flags,
                                   void* workspace, int dtype, void* stream) {
  // dtype LEA_BF16: q in the bf16 c8 layout (27*cout channels padded to a multiple
  // of 8); y is f32 NCDHW either way (the disparity regression reads f32)
  using namespace lea;
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_tapsum_upsample");
  LEA_CHECK_ARG(q && y && q != y && workspace, "lea_tapsum_upsample: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_tapsum_upsample: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && cout > 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 && Wo > 0,
                "lea_tapsum_upsample: bad shape");
  LEA_CHECK_ARG((long long)B * cout * Do * Ho < (1LL << 31) && (long long)B * cout * Do * 9 <= 65535,
                "lea_tapsum_upsample: grid too large");
  if (dtype != LEA_F32 && dtype != LEA_BF16) {
    set_error("lea_tapsum_upsample: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  hipStream_t st = as_stream(stream);
  float* ws = (float*)workspace;
  const long long HWi = (long long)Hi * Wi;
  const float rd = axis_ratio(Di, Do, 1);
  const bool vec = (HWi % 4) == 0 && ((uintptr_t)q % 16) == 0 && (q_bstride % 4) == 0 &&
                   ((long long)Di * HWi) % 4 == 0 && ((uintptr_t)ws % 16) == 0;
  if (g_tapsum_rows == 2) {
    const float rh = axis_ratio(Hi, Ho, 1), rw = axis_ratio(Wi, Wo, 1);
    for (int R = 8; R >= 2; R /= 2) {
      const int nrmax = staged_rows(Hi, Ho, 1, R, 1);
      const size_t lds = (size_t)9 * nrmax * Wi * sizeof(float);
      if (lds > 65536) continue;
      const int nhb = (Ho + R - 1) / R;
      const long long nb = (long long)B * cout * Do * nhb;
      if (nb >= (1LL << 31)) break;
      const bool v4 = dtype == LEA_F32 && vec && Wi % 4 == 0;
      const dim3 g((unsigned)nb);
      if (dtype == LEA_BF16)
        tapsum_fused<true, false><<<g, 256, lds, st>>>(q, q_bstride, (float*)y, y_bstride, cout, Di, Hi, Wi, Do,
                                                       Ho, Wo, rd, rh, rw, scale, shift, flags, R, nrmax, nhb, (int)nb);
      else if (v4)
        tapsum_fused<false, true><<<g, 256, lds, st>>>(q, q_bstride, (float*)y, y_bstride, cout, Di, Hi, Wi, Do,
                                                       Ho, Wo, rd, rh, rw, scale, shift, flags, R, nrmax, nhb, (int)nb);
      else
        tapsum_fused<false, false><<<g, 256, lds, st>>>(q, q_bstride, (float*)y, y_bstride, cout, Di, Hi, Wi, Do,
                                                        Ho, Wo, rd, rh, rw, scale, shift, flags, R, nrmax, nhb, (int)nb);
      return launch_status("lea_tapsum_upsample");
    }
  }
  if (dtype == LEA_BF16) {
    dim3 g1((unsigned)((HWi + 255) / 256), (unsigned)(B * cout * Do));
    tapsum_dpass_c8<<<g1, 256, 0, st>>>((const __bf16*)q, q_bstride, ws, cout, Di, Hi, Wi, Do, rd);
    const int rc = launch_status("lea_tapsum_upsample");
    if (rc) return rc;
    return hwpass(ws, y, y_bstride, B, cout, Hi, Wi, Do, Ho, Wo, scale, shift, flags, st);
  }
  const long long n = vec ? HWi / 4 : HWi;
  dim3 g1((unsigned)((n + 255) / 256), (unsigned)(B * cout * Do * 9));
  if (vec)
    tapsum_dpass_f32<true><<<g1, 256, 0, st>>>((const float*)q, q_bstride, ws, cout, Di, Hi, Wi, Do, rd);
  else
    tapsum_dpass_f32<false><<<g1, 256, 0, st>>>((const float*)q, q_bstride, ws, cout, Di, Hi, Wi, Do, rd);
  const int rc = launch_status("lea_tapsum_upsample");
  if (rc) return rc;
  return hwpass(ws, y, y_bstride, B, cout, Hi, Wi, Do, Ho, Wo, scale, shift, flags, st);
}
