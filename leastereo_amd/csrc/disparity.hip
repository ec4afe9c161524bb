// Fused disparity regression: trilinear (align_corners=False) upsample of the
// matching-net output by 3 in D, H, W + softmin over D + sum_d d * p_d.
// Replaces models/build_model_2d.py:52-57 (Disp.forward) and :33-42
// (DisparityRegression.forward).  The [B, maxdisp, 3H3, 3W3] volume the reference
// materialises (425 MB at 576x960 D192 fp32) never exists here.
//
// One thread per output pixel (b, oh, ow), 256 consecutive ow per workgroup.
// The bilinear (h, w) weights and four source columns are fixed per pixel, so the
// thread walks the D axis once: plane values v[dd] = bilerp(cost[dd]) are formed
// on demand (each input plane at most once, d0(od) is monotone), the depth lerp
// gives U[od], and an online softmin (running min m, s = sum e^(m-U), t = sum
// od*e^(m-U), rescaled when m drops) produces disp = t / s.  Reads are the
// 4*D3 cost values per pixel (cache-resident: 3x3 output pixels share them);
// the kernel is bound by the exp/lerp issue, far below HBM time.
#include "common.h"

namespace lea {

struct AxisW {
  int i0, i1;
  float l0, l1;
};

// aten area_pixel_compute_source_index, align_corners=False, clamped at 0.
__device__ __forceinline__ AxisW src_axis(float ratio, int o, int in, int out) {
#pragma clang fp contract(off)
  AxisW a;
  if (in == out) {
    a.i0 = a.i1 = o;
    a.l0 = 1.f;
    a.l1 = 0.f;
    return a;
  }
  float real = ratio * ((float)o + 0.5f) - 0.5f;
  if (real < 0.f) real = 0.f;
  int i = (int)floorf(real);
  if (i > in - 1) i = in - 1;
  float lam = fminf(fmaxf(real - (float)i, 0.f), 1.f);
  a.i0 = i;
  a.i1 = i + ((i < in - 1) ? 1 : 0);
  a.l1 = lam;
  a.l0 = 1.f - lam;
  return a;
}

constexpr int kDispThreads = 256;
constexpr int kDispChunk = 16;  // cost planes fetched per batch of loads

// LDS: the depth axis table (identical for every pixel) and, per thread, one
// batch of bilinearly interpolated cost planes (own column: conflict-free).
// FAST: hardware exp (v_exp_f32 on x*log2e, ~1e-6 relative) for the bf16 path
// (dtype LEA_BF16: its matching cost carries ~1e-2 relative error already); the
// f32 path keeps the accurate expf.
template <bool FAST>
__device__ __forceinline__ float dexp(float x) {
  if constexpr (FAST)
    return __expf(x);
  else
    return expf(x);
}

// expf(x) for x that cannot overflow (the register form's m - U <= rounding above 0):
// the device library's sequence -- x log2(e) split hi / lo, exp2 of the reduced
// argument, ldexp, the underflow select -- without its overflow select (bit-identical)
__device__ __forceinline__ float exp_noovf(float x) {
#pragma clang fp contract(off)
  const float ph = x * 0x1.715476p+0f;
  float pl = fmaf(x, 0x1.715476p+0f, -ph);
  pl = fmaf(x, 0x1.4ae0bep-26f, pl);
  const float rn = __builtin_rintf(ph);
  const float r = __builtin_ldexpf(__builtin_amdgcn_exp2f((ph - rn) + pl), (int)rn);
  return x < -0x1.9fe368p+6f ? 0.f : r;
}

template <bool FAST>
__global__ __launch_bounds__(kDispThreads) void disparity_f32(const float* __restrict__ cost,
                                                              float* __restrict__ disp, int D3,
                                                              int H3, int W3, int maxdisp,
                                                              float rd, float rh, float rw) {
#pragma clang fp contract(off)
  extern __shared__ float lds[];
  AxisW* tab = reinterpret_cast<AxisW*>(lds);                      // [maxdisp]
  float* pv = lds + 4 * maxdisp;                                   // [kDispChunk + 1][threads]
  for (int od = threadIdx.x; od < maxdisp; od += blockDim.x) tab[od] = src_axis(rd, od, D3, maxdisp);
  __syncthreads();
  const int Ho = 3 * H3, Wo = 3 * W3;
  const int ow = blockIdx.x * blockDim.x + threadIdx.x;
  if (ow >= Wo) return;  // no barrier below
  const int oh = blockIdx.y;
  const int b = blockIdx.z;
  const AxisW ah = src_axis(rh, oh, H3, Ho);
  const AxisW aw = src_axis(rw, ow, W3, Wo);
  const long long HW = (long long)H3 * W3;
  const float* base = cost + (long long)b * D3 * HW;
  const float* r0 = base + (long long)ah.i0 * W3;
  const float* r1 = base + (long long)ah.i1 * W3;
  float* col = pv + threadIdx.x;

  float m = 0.f, s = 0.f, t = 0.f;
  int od = 0;
  for (int p0 = 0; p0 < D3; p0 += kDispChunk) {
    // planes p0 .. p0 + kDispChunk (one past: the upper lerp source of the last
    // depth in this batch), all loads issued before the first use
#pragma unroll
    for (int k = 0; k <= kDispChunk; ++k) {
      const int dd = min(p0 + k, D3 - 1);
      const long long o = (long long)dd * HW;
      col[k * kDispThreads] = ah.l0 * (aw.l0 * r0[o + aw.i0] + aw.l1 * r0[o + aw.i1]) +
                              ah.l1 * (aw.l0 * r1[o + aw.i0] + aw.l1 * r1[o + aw.i1]);
    }
    for (; od < maxdisp && tab[od].i0 < p0 + kDispChunk; ++od) {
      const AxisW ad = tab[od];
      const float u = ad.l0 * col[(ad.i0 - p0) * kDispThreads] + ad.l1 * col[(ad.i1 - p0) * kDispThreads];
      if (od == 0) {
        m = u;
        s = 1.f;
        t = 0.f;
      } else if (u < m) {
        const float f = dexp<FAST>(u - m);  // < 1: rescale what was summed against the old min
        s = s * f + 1.f;
        t = t * f + (float)od;
        m = u;
      } else {
        const float e = dexp<FAST>(m - u);
        s += e;
        t += (float)od * e;
      }
    }
  }
  disp[((long long)b * Ho + oh) * Wo + ow] = t / s;
}

// Register form for the configured depths (r03): D3 and maxdisp compile-time, so the
// thread keeps its D3 bilinearly interpolated plane values v[dd] in registers, the
// depth axis (i0, i1, l0, l1 of every od) folds to constants, and the softmin needs
// no running-minimum rescale: every U[od] is a convex combination of two v's, so
// m = min_dd v[dd] <= min_od U[od] and sum_od e^(m - U) >= e^(m - min U) > 0 -- the same
// ratio t / s as the reference's softmax(-U) (max-subtracted), no divergent branch, no LDS.
template <int D3, int MD, bool FAST>
__global__ __launch_bounds__(kDispThreads) void disparity_reg_f32(const float* __restrict__ cost,
                                                                  float* __restrict__ disp, int H3, int W3,
                                                                  float rh, float rw) {
#pragma clang fp contract(off)
  const int Ho = 3 * H3, Wo = 3 * W3;
  const int ow = blockIdx.x * blockDim.x + threadIdx.x;
  if (ow >= Wo) return;
  const int oh = blockIdx.y;
  const int b = blockIdx.z;
  const AxisW ah = src_axis(rh, oh, H3, Ho);
  const AxisW aw = src_axis(rw, ow, W3, Wo);
  const long long HW = (long long)H3 * W3;
  const float* base = cost + (long long)b * D3 * HW;
  const float* r0 = base + (long long)ah.i0 * W3;
  const float* r1 = base + (long long)ah.i1 * W3;
  float v[D3];
#pragma unroll
  for (int dd = 0; dd < D3; ++dd) {
    const long long o = (long long)dd * HW;
    v[dd] = ah.l0 * (aw.l0 * r0[o + aw.i0] + aw.l1 * r0[o + aw.i1]) +
            ah.l1 * (aw.l0 * r1[o + aw.i0] + aw.l1 * r1[o + aw.i1]);
    // 8 planes' loads (32) in flight at a time: issuing all 4 * D3 first took 256 VGPRs
    if (dd % 8 == 7) __builtin_amdgcn_sched_barrier(0);
  }
  float m = v[0];
#pragma unroll
  for (int dd = 1; dd < D3; ++dd) m = fminf(m, v[dd]);
  constexpr float rd = (float)D3 / (float)MD;
  float s = 0.f, t = 0.f;
#pragma unroll
  for (int od = 0; od < MD; ++od) {
    const AxisW ad = src_axis(rd, od, D3, MD);  // constants after unrolling
    const float u = ad.l0 * v[ad.i0] + ad.l1 * v[ad.i1];
    const float e = FAST ? dexp<true>(m - u) : exp_noovf(m - u);
    s += e;
    t += (float)od * e;
  }
  disp[((long long)b * Ho + oh) * Wo + ow] = t / s;
}

// Row-staged form (r05; the default for the configured depths): a workgroup owns 256
// consecutive output columns of one output row, so its pixels read two source rows
// (ah.i0, ah.i1) of every plane over <= kDispCols source columns.  Those are H-lerped once
// into LDS, hl[dd][c] = ah.l0 * row0 + ah.l1 * row1 (coalesced loads, two per value), and
// each thread forms v[dd] = aw.l0 * hl[dd][i0] + aw.l1 * hl[dd][i1] from LDS -- two LDS reads
// per plane instead of four dependent global loads, ~110 fewer VGPRs than the register
// form's load batches (two waves per SIMD there).  H before W: the bilinear weights are
// applied in the other order than disparity_reg_f32 (same values up to fp32 rounding); the
// depth axis and softmin are the register form's.
constexpr int kDispCols = 96;  // >= the source columns of 256 outputs at x3 (88), + slack

// FACT (r06, form 4): the per-pixel phase with D3 exponentials instead of MD.  x3 up-sampling
// along D with align_corners=False puts od = 3k + 1 on plane k and od = 3k, 3k + 2 a third of
// the way towards planes k - 1, k + 1 (clamped at the ends), so with F_k = exp((m - v_k) / 3):
// exp(m - u) = F_{k-1} F_k^2,  F_k^3,  F_k^2 F_{k+1}, summed in the same od order.  The kernel
// is VALU-bound on the exponentials; rolled loops keep it at 32-49 VGPRs.  Not bit-identical
// to the per-od exponentials (a few ulp per term; the oracle bars).
template <int D3, int MD, bool FAST, class Plane>
__device__ __forceinline__ float softmin_fact(const Plane& plane) {
#pragma clang fp contract(off)
  static_assert(MD == 3 * D3, "x3 depth up-sampling");
  // a plain select (no NaN in the planes): fminf's NaN rule let the vectoriser split this loop
  // into per-pair NaN tests and divergent branches
  float m = plane(0);
#pragma unroll 8
  for (int dd = 1; dd < D3; ++dd) {
    const float v = plane(dd);
    m = v < m ? v : m;
  }
  auto fk = [&](int dd) {
    if constexpr (FAST)  // __expf's exp2(x log2 e) with the 1/3 folded into its multiplier
      return __builtin_amdgcn_exp2f((m - plane(dd)) * (0x1.715476p+0f / 3.f));
    else
      return exp_noovf((m - plane(dd)) * 0x1.555556p-2f);
  };
  float s = 0.f, t = 0.f;
  float fp = fk(0), fc = fp;  // F_{k-1}, F_k
  float od = 0.f;             // 3k (exact in float)
#pragma unroll 4
  for (int k = 0; k < D3; ++k) {
    const float fn = k + 1 < D3 ? fk(k + 1) : fc;
    const float f2 = fc * fc;
    const float e1 = f2 * fc;
    const float e0 = k == 0 ? e1 : fp * f2;
    const float e2 = k + 1 < D3 ? f2 * fn : e1;
    s += e0;
    t += od * e0;
    s += e1;
    t += (od + 1.f) * e1;
    s += e2;
    t += (od + 2.f) * e2;
    od += 3.f;
    fp = fc;
    fc = fn;
  }
  return t / s;
}

template <int D3, int MD, bool FAST, bool FACT>
__global__ __launch_bounds__(kDispThreads, 4) void disparity_rows_f32(const float* __restrict__ cost,
                                                                   float* __restrict__ disp, int H3, int W3,
                                                                   float rh, float rw) {
#pragma clang fp contract(off)
  __shared__ float hl[D3 * kDispCols];
  const int Ho = 3 * H3, Wo = 3 * W3;
  const int ow0 = blockIdx.x * blockDim.x;
  const int oh = blockIdx.y;
  const int b = blockIdx.z;
  const AxisW ah = src_axis(rh, oh, H3, Ho);
  const int c_lo = src_axis(rw, ow0, W3, Wo).i0;
  const int c_hi = src_axis(rw, min(ow0 + (int)blockDim.x - 1, Wo - 1), W3, Wo).i1;
  // host: <= kDispCols (Wo = 3 W3); past it the staging is clamped and the outputs are NaN
  const bool over = c_hi - c_lo + 1 > kDispCols;
  const int ncol = min(c_hi - c_lo + 1, kDispCols);
  const long long HW = (long long)H3 * W3;
  const float* base = cost + (long long)b * D3 * HW + c_lo;
  const float* r0 = base + (long long)ah.i0 * W3;
  const float* r1 = base + (long long)ah.i1 * W3;
  for (int e = threadIdx.x; e < D3 * ncol; e += blockDim.x) {
    const int dd = e / ncol, c = e - dd * ncol;
    const long long o = (long long)dd * HW + c;
    hl[dd * kDispCols + c] = ah.l0 * r0[o] + ah.l1 * r1[o];
  }
  __syncthreads();
  const int ow = ow0 + threadIdx.x;
  if (ow >= Wo) return;  // no barrier below
  const AxisW aw = src_axis(rw, ow, W3, Wo);
  const int j0 = min(aw.i0 - c_lo, kDispCols - 1), j1 = min(aw.i1 - c_lo, kDispCols - 1);
  auto plane = [&](int dd) { return aw.l0 * hl[dd * kDispCols + j0] + aw.l1 * hl[dd * kDispCols + j1]; };
  if constexpr (FACT) {
    const float r = softmin_fact<D3, MD, FAST>(plane);
    disp[((long long)b * Ho + oh) * Wo + ow] = over ? __builtin_nanf("") : r;
    return;
  }
  // pass 1: the smallest plane value; pass 2 forms the planes again from LDS in depth order
  // (the register form kept all D3 of them live: two waves per SIMD)
  float m = plane(0);
#pragma unroll
  for (int dd = 1; dd < D3; ++dd) {
    m = fminf(m, plane(dd));
    if (dd % 8 == 7) __builtin_amdgcn_sched_barrier(0);
  }
  constexpr float rd = (float)D3 / (float)MD;
  float s = 0.f, t = 0.f;
  float vlo = plane(0), vhi = plane(D3 > 1 ? 1 : 0);
  int k = 0;  // vlo = plane k, vhi = plane min(k + 1, D3 - 1): constants after unrolling
#pragma clang loop unroll(full)
  for (int od = 0; od < MD; ++od) {
    const AxisW ad = src_axis(rd, od, D3, MD);  // constants after unrolling
    while (k < ad.i0) {
      ++k;
      vlo = vhi;
      vhi = plane(k + 1 < D3 ? k + 1 : D3 - 1);
    }
    const float v1 = ad.i1 == k ? vlo : vhi;
    const float u = ad.l0 * vlo + ad.l1 * v1;
    const float e = FAST ? dexp<true>(m - u) : exp_noovf(m - u);
    s += e;
    t += (float)od * e;
    if (od % 12 == 11) __builtin_amdgcn_sched_barrier(0);
  }
  disp[((long long)b * Ho + oh) * Wo + ow] = over ? __builtin_nanf("") : t / s;
}

// Three-row form (r06): output rows 3k, 3k + 1, 3k + 2 read source rows
// k - 1, k, k + 1 only (x3 up-sampling, align_corners=False), so one workgroup of 3 x 256
// threads owns 256 columns of all three: every raw source value is loaded ONCE (three loads
// per staged element, for three H-lerped rows) instead of twice by each of three row
// workgroups (six), and the row-position arithmetic is paid once per element.  Each output
// row's LDS row is ah.l0 * row(ah.i0) + ah.l1 * row(ah.i1) with that row's own weights -- the
// two-row kernel's expression, so every output is bit-identical to disparity_rows_f32; the
// per-pixel phase is that kernel's.  LDS 3 * D3 * kDispCols floats (74 KB at D3 = 64: two
// workgroups, 24 waves per CU).
constexpr int kDisp3Threads = 3 * kDispThreads;

template <int D3, int MD, bool FAST, bool FACT>
__global__ __launch_bounds__(kDisp3Threads) void disparity_rows3_f32(const float* __restrict__ cost,
                                                                   float* __restrict__ disp, int H3, int W3,
                                                                   float rh, float rw) {
#pragma clang fp contract(off)
  __shared__ float hl[3][D3 * kDispCols];
  const int Ho = 3 * H3, Wo = 3 * W3;
  const int ow0 = blockIdx.x * kDispThreads;
  const int k = blockIdx.y;  // source row k: output rows 3k .. 3k + 2
  const int b = blockIdx.z;
  const AxisW a0 = src_axis(rh, 3 * k, H3, Ho), a1 = src_axis(rh, 3 * k + 1, H3, Ho),
              a2 = src_axis(rh, 3 * k + 2, H3, Ho);
  // the staged raw rows: lo = min of the three rows' i0 (k - 1, or 0 at the top), lo + 1, lo + 2
  // clamped to the map; every i0 / i1 of the three rows lies in [lo, lo + 2] (x3: k - 1 .. k + 1)
  const int lo = min(a0.i0, min(a1.i0, a2.i0));
  const int r1 = min(lo + 1, H3 - 1), r2 = min(lo + 2, H3 - 1);
  const int c_lo = src_axis(rw, ow0, W3, Wo).i0;
  const int c_hi = src_axis(rw, min(ow0 + kDispThreads - 1, Wo - 1), W3, Wo).i1;
  const bool over = c_hi - c_lo + 1 > kDispCols ||
                    max(a0.i1, max(a1.i1, a2.i1)) > lo + 2;  // host-checked; NaN rather than a wrong row
  const int ncol = min(c_hi - c_lo + 1, kDispCols);
  const long long HW = (long long)H3 * W3;
  const float* base = cost + (long long)b * D3 * HW + c_lo;
  const float* p0 = base + (long long)lo * W3;
  const float* p1 = base + (long long)r1 * W3;
  const float* p2 = base + (long long)r2 * W3;
  // row i of the map as one of the three staged values (workgroup-uniform selects)
  auto pick = [&](int i, float v0, float v1, float v2) { return i == lo ? v0 : (i == lo + 1 ? v1 : v2); };
  for (int e = threadIdx.x; e < D3 * ncol; e += kDisp3Threads) {
    const int dd = e / ncol, c = e - dd * ncol;
    const long long o = (long long)dd * HW + c;
    const float v0 = p0[o], v1 = p1[o], v2 = p2[o];
    const int s = dd * kDispCols + c;
    hl[0][s] = a0.l0 * pick(a0.i0, v0, v1, v2) + a0.l1 * pick(a0.i1, v0, v1, v2);
    hl[1][s] = a1.l0 * pick(a1.i0, v0, v1, v2) + a1.l1 * pick(a1.i1, v0, v1, v2);
    hl[2][s] = a2.l0 * pick(a2.i0, v0, v1, v2) + a2.l1 * pick(a2.i1, v0, v1, v2);
  }
  __syncthreads();
  const int row = __builtin_amdgcn_readfirstlane(threadIdx.x / kDispThreads);  // wave-uniform
  const int ow = ow0 + (int)threadIdx.x % kDispThreads;
  const int oh = 3 * k + row;
  if (ow >= Wo) return;  // no barrier below
  const float* h = hl[row];
  const AxisW aw = src_axis(rw, ow, W3, Wo);
  const int j0 = min(aw.i0 - c_lo, kDispCols - 1), j1 = min(aw.i1 - c_lo, kDispCols - 1);
  auto plane = [&](int dd) { return aw.l0 * h[dd * kDispCols + j0] + aw.l1 * h[dd * kDispCols + j1]; };
  if constexpr (FACT) {
    const float r = softmin_fact<D3, MD, FAST>(plane);
    disp[((long long)b * Ho + oh) * Wo + ow] = over ? __builtin_nanf("") : r;
    return;
  }
  float m = plane(0);
#pragma unroll
  for (int dd = 1; dd < D3; ++dd) {
    m = fminf(m, plane(dd));
    if (dd % 8 == 7) __builtin_amdgcn_sched_barrier(0);
  }
  constexpr float rd = (float)D3 / (float)MD;
  float s = 0.f, t = 0.f;
  float vlo = plane(0), vhi = plane(D3 > 1 ? 1 : 0);
  int kk = 0;  // vlo = plane kk, vhi = plane min(kk + 1, D3 - 1): constants after unrolling
#pragma clang loop unroll(full)
  for (int od = 0; od < MD; ++od) {
    const AxisW ad = src_axis(rd, od, D3, MD);  // constants after unrolling
    while (kk < ad.i0) {
      ++kk;
      vlo = vhi;
      vhi = plane(kk + 1 < D3 ? kk + 1 : D3 - 1);
    }
    const float v1 = ad.i1 == kk ? vlo : vhi;
    const float u = ad.l0 * vlo + ad.l1 * v1;
    const float e = FAST ? dexp<true>(m - u) : exp_noovf(m - u);
    s += e;
    t += (float)od * e;
    if (od % 12 == 11) __builtin_amdgcn_sched_barrier(0);
  }
  disp[((long long)b * Ho + oh) * Wo + ow] = over ? __builtin_nanf("") : t / s;
}

}  // namespace lea

// lea_disparity_set_register_form: 4 (default, r06) = form 3 with D3 exponentials per pixel
// instead of maxdisp (softmin_mean's FACT; the two-row kernel at D3 = 88 likewise), 3 = the three-row staged kernel (C2 69.5 -> 68.3,
// C4 275.6 -> 266.4 us; not at D3 = 88), 2 (r05) = the row-staged kernel for the configured
// (D3, maxdisp), 1 = the register kernel for them, 0 = the online-softmin kernel everywhere
// (A/B and tests)
static int g_disp_reg = 4;
extern "C" int lea_disparity_set_register_form(int on) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 4, "lea_disparity_set_register_form: %d", on);
  g_disp_reg = on;
  return 0;
}

extern "C" int lea_disparity_regression(const void* cost, float* disp, int B, int D3, int H3,
                                        int W3, int maxdisp, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(cost && disp, "lea_disparity_regression: null pointer");
  LEA_CHECK_ARG(B > 0 && D3 > 0 && H3 > 0 && W3 > 0 && maxdisp > 0,
                "lea_disparity_regression: bad shape B=%d D3=%d H3=%d W3=%d maxdisp=%d", B, D3, H3,
                W3, maxdisp);
  LEA_CHECK_ARG(3 * H3 <= 65535 && B <= 65535, "lea_disparity_regression: grid too large");
  if (dtype != LEA_F32 && dtype != LEA_BF16) {
    set_error("lea_disparity_regression: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const int Wo = 3 * W3;
  const size_t lds = (size_t)4 * maxdisp * sizeof(float) + (size_t)(kDispChunk + 1) * kDispThreads * sizeof(float);
  LEA_CHECK_ARG(lds <= 65536, "lea_disparity_regression: maxdisp %d too large", maxdisp);
  dim3 block(kDispThreads);
  dim3 grid((Wo + kDispThreads - 1) / kDispThreads, 3 * H3, B);
  const float rh = (float)H3 / (float)(3 * H3), rw = (float)W3 / (float)(3 * W3);
  const bool fast = dtype == LEA_BF16;
#define LEA_DISP_REG(D3_, MD_)                                                                          \
  if (D3 == D3_ && maxdisp == MD_) {                                                                   \
    auto k_ = fast ? disparity_reg_f32<D3_, MD_, true> : disparity_reg_f32<D3_, MD_, false>;            \
    k_<<<grid, block, 0, as_stream(stream)>>>((const float*)cost, disp, H3, W3, rh, rw);                 \
    return launch_status("lea_disparity_regression");                                                  \
  }
  // the row-staged forms: 256 outputs of a row read <= kDispCols source columns (Wo = 3 W3)
  const bool cols_ok = (256LL * W3 + Wo - 1) / Wo + 2 <= kDispCols;
#define LEA_DISP_ROWS3(D3_, MD_)                                                                        \
  if (D3 == D3_ && maxdisp == MD_) {                                                                   \
    auto k_ = fact ? (fast ? disparity_rows3_f32<D3_, MD_, true, true> : disparity_rows3_f32<D3_, MD_, false, true>)   \
                   : (fast ? disparity_rows3_f32<D3_, MD_, true, false> : disparity_rows3_f32<D3_, MD_, false, false>); \
    k_<<<dim3((Wo + kDispThreads - 1) / kDispThreads, H3, B), kDisp3Threads, 0, as_stream(stream)>>>(   \
        (const float*)cost, disp, H3, W3, rh, rw);                                                     \
    return launch_status("lea_disparity_regression");                                                  \
  }
  // (88, 264) -- config 5 -- keeps the two-row kernel: three rows' LDS (101 KB) leave one
  // workgroup per CU there (213 -> 260 us, profiles/r06_disp_probe.txt)
  const bool fact = g_disp_reg == 4;
  if (g_disp_reg >= 3 && cols_ok) {
    LEA_DISP_ROWS3(4, 12) LEA_DISP_ROWS3(8, 24) LEA_DISP_ROWS3(16, 48) LEA_DISP_ROWS3(32, 96)
    LEA_DISP_ROWS3(64, 192)
  }
#undef LEA_DISP_ROWS3
  const bool rows_ok = g_disp_reg >= 2 && cols_ok;
#define LEA_DISP_ROWS(D3_, MD_)                                                                         \
  if (D3 == D3_ && maxdisp == MD_) {                                                                   \
    auto k_ = fact ? (fast ? disparity_rows_f32<D3_, MD_, true, true> : disparity_rows_f32<D3_, MD_, false, true>)   \
                   : (fast ? disparity_rows_f32<D3_, MD_, true, false> : disparity_rows_f32<D3_, MD_, false, false>); \
    k_<<<grid, block, 0, as_stream(stream)>>>((const float*)cost, disp, H3, W3, rh, rw);                 \
    return launch_status("lea_disparity_regression");                                                  \
  }
  if (rows_ok) {
    LEA_DISP_ROWS(4, 12) LEA_DISP_ROWS(8, 24) LEA_DISP_ROWS(16, 48) LEA_DISP_ROWS(32, 96) LEA_DISP_ROWS(64, 192)
    LEA_DISP_ROWS(88, 264)
  }
#undef LEA_DISP_ROWS
  if (g_disp_reg) {
    // (88, 264) -- config 5 -- stays on the LDS kernel: its 88 plane values take all 256
    // VGPRs, one wave per SIMD (r03: 0.388 vs 0.380 ms); at (64, 192): 0.125 -> 0.081 ms
    LEA_DISP_REG(4, 12) LEA_DISP_REG(8, 24) LEA_DISP_REG(16, 48) LEA_DISP_REG(32, 96) LEA_DISP_REG(64, 192)
  }
#undef LEA_DISP_REG
  auto kern = dtype == LEA_BF16 ? disparity_f32<true> : disparity_f32<false>;
  kern<<<grid, block, lds, as_stream(stream)>>>(
      (const float*)cost, disp, D3, H3, W3, maxdisp, (float)D3 / (float)maxdisp,
      (float)H3 / (float)(3 * H3), (float)W3 / (float)(3 * W3));
  return launch_status("lea_disparity_regression");
}
