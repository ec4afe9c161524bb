// ConvBR3d (Conv3d k in {1,3}, stride 1, pad k/2, no bias -> folded BN -> ReLU
// [-> + residual]) as an implicit GEMM on the gfx950 fp32 matrix cores.
// Replaces models/operations_3d.py:31-47 for every ConvBR of the matching net
// (retrain/skip_model_3d.py), the cell's pairwise sums (LEA_RESIDUAL,
// skip_model_3d.py:69), the skip-fusion concat (two input sources,
// skip_model_3d.py:150,155) and -- in the resampling variant -- the trilinear
// level change that precedes every cell preprocess (skip_model_3d.py:44-53).
//
// GEMM view (per batch b, output plane d):
//     Y[co][v] = sum_{ci, tap} Wt[co][ci][tap] * X[ci][v + off(tap)]
// M = cout (blocks of <= 64 per workgroup, 16-row MFMA tiles), N = voxels
// (16-wide runs along W, coalesced NCDHW), K = cin * k^3.
// MFMA = v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulate):
//     A (lane l) = Wt[co = 16*mt + (l & 15)][k = l >> 4]
//     B (lane l) = X [k = l >> 4][v = 16*nt + (l & 15)]
//     D (lane l, reg r) = Y[co = 16*mt + 4*(l >> 4) + r][v = l & 15]
// so the epilogue stores 16 consecutive w per cout row (64-B segments).
//
// Workgroup = 4 waves = a TH x TW voxel tile of one output plane, all couts of
// its block.  K is streamed in chunks of CIN_B input channels staged in LDS; every
// wave then runs k^3 * CIN_B/4 k-steps of MT x NT MFMAs whose operands are single
// ds_read_b32 at per-lane base + compile-time offset.  LDS strides keep each
// 32-lane read group on 32 distinct banks (the two k-rows of a half-wave sit 16
// banks apart: strides = 16 mod 32).
//
// Two staging engines:
//  * conv3d_dma_kernel (k=3, the MFMA-bound layers): the input halo block is
//    fetched by LDS-DMA (`buffer_load_dword ... lds`) through one buffer resource
//    per input channel.  The per-lane source offsets are computed once per
//    workgroup; voxels outside the volume get an offset beyond the resource's
//    num_records, so the hardware range check returns 0 -- the conv's zero
//    padding costs no VALU.  Weights arrive by `global_load_lds_dwordx4`.  Two
//    LDS stages: chunk c+1's DMA is in flight while chunk c's MFMAs run; one
//    vmcnt(0) + barrier per chunk.  (Register staging spent 2-7 VALU
//    instructions per MFMA on index math and saturated VALU issue: r01 PMC.)
//  * conv3d_reg_kernel (k=1, and the RESAMPLE variant for k in {1,3}): register
//    staged; with RESAMPLE each staged value is the trilinear (align_corners=True)
//    interpolation of the low/high-resolution input at the output voxel, so the
//    resampled volume is never written to HBM.
#pragma once
#include "common.h"

namespace lea {

constexpr int kConvWaves = 4;
constexpr int kConvThreads = kConvWaves * kWave;

using f32x4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;
using lds_void = __attribute__((address_space(3))) void;

// Row stride of the staged weight block / packed weights, congruent 16 mod 32
// so lanes 0-15 and 16-31 of one ds_read_b32 fall on disjoint banks.
__host__ __device__ constexpr int cout_stride(int cop) { return (cop % 32 == 0) ? cop + 16 : cop; }
__host__ __device__ constexpr int round_16mod32(int n) {
  return (n % 32 <= 16) ? n + (16 - n % 32) : n + (48 - n % 32);
}

struct ConvArgs {
  const float* x;   // source 1: input channels [0, cin1)
  long long xbs;
  const float* x2;  // source 2: input channels [cin1, cin) (virtual concat)
  long long x2bs;
  int cin1;
  const float* wp;
  const float* scale;
  const float* shift;
  const float* res;
  long long rbs;
  float* y;
  long long ybs;
  int cin, cout, D, H, W;  // conv (= output) volume
  int Di, Hi, Wi;          // stored input volume (RESAMPLE variant)
  float rd, rh, rw;        // align_corners=True source ratios (RESAMPLE variant)
  int tiles_w, ncob;
  int ntiles, ndz, nblk;   // DMA engine's 1-D grid: tiles x depth groups x (B * ncob)
  unsigned flags;
  int spw;                 // W x D Winograd engine: depth pairs walked per workgroup (0 = 1)
  unsigned* dbg;           // diagnostic builds only (LEA_EXP_STAMPS): per-wave phase cycles
  // lea_conv2d_bnrelu_pair (few-channel 2D tile): couts [csplit, cout) go to y2 (no residual)
  float* y2;
  long long y2bs;
  int csplit;
  long long uoff;          // F(2,3) x F(2,3) tile (conv3d_wino22.hip): U section of the packed weights
  int grp;                 // F(4,3) x F(4,3) tile: block order (0 = linear; g = groups of g x g tiles)
};

// KD = kernel depth: KS for the 3D convs, 1 for the feature net's 2D 3x3 convs
// (a 2D conv is the D = 1 case of a (1, 3, 3) kernel).
template <int KS, int MT, int KD = KS>
struct PackCfg {
  static constexpr int KT = KD * KS * KS;
  static constexpr int CIN_B = (KS == 3) ? 4 : 32;
  static constexpr int COP = MT * 16;
  static constexpr int COPS = COP;  // row stride of a staged weight row (floats)
  // Rows 32 or 64 wide (stride = 0 mod 32 banks): odd input-channel rows are
  // stored with 16-column halves swapped, so the two k-rows of a half-wave read
  // disjoint banks without padding (16- and 48-wide rows are already 16 mod 32).
  static constexpr bool SWZ = (COP % 32) == 0;
  static constexpr int CHUNK = KT * CIN_B * COPS;  // floats per K chunk
};

// Column of this lane's A element of m-tile m inside a staged weight row.
template <int KS, int MT>
__device__ __forceinline__ int a_col(int m, int kq, int n) {
  return ((PackCfg<KS, MT>::SWZ ? (m ^ (kq & 1)) : m) * 16) + n;
}

template <int KS, int MT, int NT, int TW, int TD = 1, int KD = KS>
struct TileCfg : PackCfg<KS, MT, KD> {
  using P = PackCfg<KS, MT, KD>;
  static constexpr int PAD = KS / 2;
  static constexpr int NTILES = kConvWaves * NT;
  static constexpr int TPR = TW / 16;  // 16-voxel N tiles per row
  static constexpr int TH = NTILES / TPR;
  static_assert(NTILES % TPR == 0, "tile rows");
  static constexpr int RH = TH + KS - 1;
  static constexpr int RW = TW + KS - 1;
  static constexpr int PLANE = RH * RW;
  static constexpr int PLANES = KD + TD - 1;       // input planes feeding TD output planes
  static constexpr int IMG = PLANES * PLANE;       // staged floats per input channel
  static constexpr int CIS = round_16mod32(IMG);   // LDS stride between input channels
  static constexpr int XS = P::CIN_B * CIS;
  static constexpr int WS = P::CHUNK;
  static constexpr int STAGE = XS + WS;            // floats (multiple of 16: 64-B aligned)
  static_assert(XS % 16 == 0 && WS % 16 == 0, "16-byte aligned LDS regions");
};

// ----------------------------------------------------------------- MFMA main loop
// One K chunk from an LDS stage: KS^3 taps x CIN_B/4 k-steps x (MT x NT) MFMAs.
template <int KS, int MT, int NT, int TW, int TD, int KD = KS>
__device__ __forceinline__ void mfma_chunk(const float* xs, const float* ws, const int (&xoff)[NT],
                                           const int (&woff)[MT], f32x4 (&acc)[TD][MT][NT]) {
  using C = TileCfg<KS, MT, NT, TW, TD, KD>;
  constexpr int CIN_B = C::CIN_B;
#pragma unroll
  for (int s = 0; s < CIN_B / 4; ++s) {
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) {
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const int tap = (kd * KS + kh) * KS + kw;
          float av[MT], bv[TD][NT];
#pragma unroll
          for (int m = 0; m < MT; ++m) av[m] = ws[woff[m] + (tap * CIN_B + 4 * s) * C::COPS];
#pragma unroll
          for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int j = 0; j < NT; ++j)
              bv[t][j] = xs[xoff[j] + 4 * s * C::CIS + (t + kd) * C::PLANE + kh * C::RW + kw];
#pragma unroll
          for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
              for (int j = 0; j < NT; ++j)
                acc[t][m][j] =
                    __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[t][j], acc[t][m][j], 0, 0, 0);
        }
      }
    }
  }
}

// Folded-BN affine, ReLU, residual, masked store of the MT x NT accumulator tiles.
template <int KS, int MT, int NT, int TW, int TD>
__device__ __forceinline__ void epilogue(const ConvArgs& a, const f32x4 (&acc)[TD][MT][NT], int b,
                                         int co0, int d0, int h0, int w0, int wave, int lane) {
  using C = TileCfg<KS, MT, NT, TW, TD>;
  const long long HW = (long long)a.H * a.W;
  const long long DHW = HW * a.D;
  const bool relu = a.flags & LEA_RELU;
  const bool resid = a.flags & LEA_RESIDUAL;
  const int kq = lane >> 4, n = lane & 15;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + m * 16 + kq * 4 + r;
      if (co >= a.cout) continue;
      const float sc = a.scale ? a.scale[co] : 1.f;
      const float sh = a.shift ? a.shift[co] : 0.f;
#pragma unroll
      for (int t = 0; t < TD; ++t) {
        const int d = d0 + t;
        if (d >= a.D) continue;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int g = wave * NT + j;
          const int h = h0 + g / C::TPR;
          const int w = w0 + (g % C::TPR) * 16 + n;
          if (h >= a.H || w >= a.W) continue;
          const long long o = (long long)co * DHW + (long long)d * HW + (long long)h * a.W + w;
          float v = acc[t][m][j][r] * sc + sh;
          if (relu) v = fmaxf(v, 0.f);
          if (resid) v += a.res[(long long)b * a.rbs + o];
          a.y[(long long)b * a.ybs + o] = v;
        }
      }
    }
  }
}

// DMA-engine epilogue.  Output addressing is one per-lane 32-bit element offset
// (host checks cout*D*H*W < 2^31) plus per-element offsets that are uniform across
// the wave, and tiles that lie wholly inside the volume and the cout block skip
// the per-element masks: on the small-K cell layers the r01 epilogue (64-bit
// index math and four compares per stored value) was ~1 VALU op per MFMA.
// Epilogue operands -- folded BN of this lane's couts and, under LEA_RESIDUAL with
// RES, the residual of every voxel it stores -- are loaded at the start of the
// workgroup so their latency hides under the main loop (accumulating cell ops were
// ~25% slower when the residual was read in the store phase).
template <int MT, int NT, int TD, bool RES>
struct EpiRegs {
  float sc[MT][4], sh[MT][4];
  float rv[RES ? TD : 1][RES ? MT : 1][RES ? NT : 1][4];
};

// KD = 4 marks the depth-paired layout (couts <= 8): accumulator row 8t + c is
// output channel c of plane d0 + t (see conv3d_dma_kernel).
template <int KS, int MT, int NT, int TW, int TD, int KD = KS>
struct EpiGeom {
  using C = TileCfg<KS, MT, NT, TW, TD>;
  static constexpr bool DP = KD == 4;
  int HW, DHW, W;
  int base;       // element offset (in one batch) of this lane's (m, r, t, j) = 0 output
  int wave;
  bool interior;  // the whole tile is inside the volume and the cout block
  int co0, d0, h0, w0, kq, n;
  __device__ EpiGeom(const ConvArgs& a, int co0_, int d0_, int h0_, int w0_, int wave_, int lane)
      : co0(co0_), d0(d0_), h0(h0_), w0(w0_) {
    HW = a.H * a.W;
    DHW = HW * a.D;
    W = a.W;
    wave = wave_;
    kq = lane >> 4;
    n = lane & 15;
    const int g0 = wave * NT;
    const int cq = DP ? (kq & 1) * 4 : kq * 4, dq = DP ? (kq >> 1) : 0;
    base = (co0 + cq) * DHW + (d0 + dq) * HW + (h0 + g0 / C::TPR) * a.W + w0 + (g0 % C::TPR) * 16 + n;
    interior = co0 + (DP ? 8 : C::COP) <= a.cout && d0 + (DP ? 2 : TD) <= a.D && h0 + C::TH <= a.H &&
               w0 + TW <= a.W;
  }
  __device__ int cout_of(int m, int r) const {  // output channel of accumulator row (m, r)
    return co0 + m * 16 + (DP ? (kq & 1) * 4 : kq * 4) + r;
  }
  // offset of element (m, r, t, j) relative to base: uniform across the wave
  __device__ int rel(int m, int r, int t, int j) const {
    const int g0 = wave * NT, g = g0 + j;
    return (m * 16 + r) * DHW + t * HW + (g / C::TPR - g0 / C::TPR) * W +
           ((g % C::TPR) - (g0 % C::TPR)) * 16;
  }
  __device__ bool inside(const ConvArgs& a, int m, int r, int t, int j) const {
    const int g = wave * NT + j;
    return cout_of(m, r) < a.cout && d0 + t + (DP ? (kq >> 1) : 0) < a.D && h0 + g / C::TPR < a.H &&
           w0 + (g % C::TPR) * 16 + n < a.W;
  }
};

template <int KS, int MT, int NT, int TW, int TD, bool RES, int KD>
__device__ __forceinline__ void epi_prefetch(const ConvArgs& a, EpiRegs<MT, NT, TD, RES>& e,
                                             const EpiGeom<KS, MT, NT, TW, TD, KD>& g, int b) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = g.cout_of(m, r);
      const bool cv = co < a.cout;
      e.sc[m][r] = (cv && a.scale) ? a.scale[co] : 1.f;
      e.sh[m][r] = (cv && a.shift) ? a.shift[co] : 0.f;
    }
  if constexpr (RES) {
    const bool resid = a.flags & LEA_RESIDUAL;
    const float* rb = a.res + (long long)b * a.rbs + g.base;
#pragma unroll
    for (int t = 0; t < TD; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            e.rv[t][m][j][r] =
                (resid && (g.interior || g.inside(a, m, r, t, j))) ? rb[g.rel(m, r, t, j)] : 0.f;
  }
}

template <int KS, int MT, int NT, int TW, int TD, bool RES, int KD>
__device__ __forceinline__ void epilogue_dma(const ConvArgs& a, const f32x4 (&acc)[TD][MT][NT],
                                             const EpiRegs<MT, NT, TD, RES>& e,
                                             const EpiGeom<KS, MT, NT, TW, TD, KD>& g, int b) {
  const bool relu = a.flags & LEA_RELU;
  const bool resid = a.flags & LEA_RESIDUAL;
  float* yb = a.y + (long long)b * a.ybs + g.base;
  const float* rb = a.res + (long long)b * a.rbs + g.base;
  auto value = [&](int m, int r, int t, int j) {
    float v = acc[t][m][j][r] * e.sc[m][r] + e.sh[m][r];
    if (relu) v = fmaxf(v, 0.f);
    if (resid) {
      if constexpr (RES)
        v += e.rv[t][m][j][r];
      else
        v += rb[g.rel(m, r, t, j)];
    }
    return v;
  };
  if (g.interior) {
#pragma unroll
    for (int t = 0; t < TD; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) yb[g.rel(m, r, t, j)] = value(m, r, t, j);
  } else {
#pragma unroll
    for (int t = 0; t < TD; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (g.inside(a, m, r, t, j)) yb[g.rel(m, r, t, j)] = value(m, r, t, j);
  }
}

// ------------------------------------------------------------- LDS-DMA engine (k=3)
// CV: the input is LEAStereo's cost volume (retrain/LEAStereo.py:34-48), never
// materialised -- x / x2 are the left / right feature maps [B, cin1, H, W] and the
// staged value of channel c < cin1 at (disparity d, h, w) is left[c][h][w], of
// channel cin1 + c right[c][h][w - d], both 0 for w < d: per lane two offset sets
// (left, right) whose out-of-range entries make the buffer load return the zero.
// KD = 4 (MT = 1, TD = 1): depth-paired tile for convs with <= 8 output channels.
// The 16 MFMA rows hold output channels 0..7 of TWO planes d0, d0+1; the four
// staged input planes p = 0..3 each feed both, through paired weight rows
// W'[p][8t + c] = W[c][kd = p - t] (zero outside 0..2), packed by
// pack_weights_dp_kernel.  36 k-steps per plane pair instead of 2 x 27 on
// half-empty 16-row tiles: 1.5x fewer MFMAs for the 8->8 cell ops.
template <int MT, int NT, int TW, int TD, int KD = 3, bool CV = false>
__global__ __launch_bounds__(kConvThreads, 2) void conv3d_dma_kernel(const ConvArgs a) {
  using C = TileCfg<3, MT, NT, TW, TD, KD>;
  static_assert(KD != 4 || (MT == 1 && TD == 1), "depth pairing is an MT=1, TD=1 tile");
  constexpr int DSTEP = KD == 4 ? 2 : TD;      // output planes per workgroup
  constexpr int DOFF = KD == 4 ? 1 : KD / 2;   // staged plane 0 = output plane d0 - DOFF
  constexpr int XSLOTS = (C::IMG + 63) / 64;  // 256-B DMA pieces per channel image
  constexpr int XSLOTS_W = (XSLOTS + kConvWaves - 1) / kConvWaves;
  constexpr int WSLOTS = (C::WS + 255) / 256;  // 1-KB DMA pieces of the weight chunk
  constexpr int WSLOTS_W = (WSLOTS + kConvWaves - 1) / kConvWaves;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: blocks are dealt round-robin to the 8 XCDs, so block id i
  // becomes position (i % 8) * ceil(N/8) + i / 8 of a (batch/cout-block, tile,
  // depth group) walk with the depth group fastest -- every XCD then runs whole
  // depth columns of neighbouring tiles, whose shared input planes and halo rows
  // stay in its L2 (speed only: any placement is correct).
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int dz = lin % a.ndz;
  const int tile = (lin / a.ndz) % a.ntiles;
  const int bc = lin / (a.ndz * a.ntiles);
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * TW;
  const int d0 = dz * DSTEP;
  const int b = bc / a.ncob;
  const int co0 = (bc - b * a.ncob) * C::COP;
  const int nchunks = (a.cin + C::CIN_B - 1) / C::CIN_B;
  const float* wp = a.wp + (long long)(co0 / C::COP) * nchunks * C::WS;
  const int HW = a.H * a.W;  // host checks D*H*W*4 < 2^32
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;

  // Per-lane byte offsets of this wave's DMA pieces inside one channel volume;
  // identical for every channel and chunk.  Outside the volume -> beyond nrec -> 0.
  unsigned voff[XSLOTS_W], voffr[CV ? XSLOTS_W : 1];
#pragma unroll
  for (int t = 0; t < XSLOTS_W; ++t) {
    const int e = (wave + kConvWaves * t) * 64 + lane;
    unsigned v = 0xFFFFFFF0u, vr = 0xFFFFFFF0u;
    if (e < C::IMG) {
      const int kd = e / C::PLANE;
      const int r = e - kd * C::PLANE;
      const int rr = r / C::RW;
      const int cc = r - rr * C::RW;
      const int d = d0 + kd - DOFF, h = h0 + rr - 1, w = w0 + cc - 1;
      if ((unsigned)d < (unsigned)a.D && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
        if constexpr (CV) {
          if (w >= d) {
            v = (unsigned)(h * a.W + w) * 4u;
            vr = (unsigned)(h * a.W + w - d) * 4u;
          }
        } else {
          v = (unsigned)(d * HW + h * a.W + w) * 4u;
        }
      }
    }
    voff[t] = v;
    if constexpr (CV) voffr[t] = vr;
  }

  auto issue = [&](int ch, float* st) {
    const float* wsrc = wp + (long long)ch * C::WS;
    float* wdst = st + C::XS;
#pragma unroll
    for (int t = 0; t < WSLOTS_W; ++t) {
      const int j = wave + kConvWaves * t;
      if (j < WSLOTS && j * 256 + lane * 4 < C::WS)
        __builtin_amdgcn_global_load_lds(wsrc + j * 256 + lane * 4, (lds_void*)(wdst + j * 256), 16, 0, 0);
    }
#pragma unroll
    for (int ci = 0; ci < C::CIN_B; ++ci) {
      const int c = ch * C::CIN_B + ci;
      const float* base = a.x;
      unsigned n = 0;
      const long long cvol = CV ? (long long)HW : (long long)HW * a.D;  // channel stride
      const unsigned crec = CV ? (unsigned)HW * 4u : nrec;
      if (c < a.cin1) {
        base = a.x + (long long)b * a.xbs + (long long)c * cvol;
        n = crec;
      } else if (c < a.cin) {
        base = a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * cvol;
        n = crec;
      }
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
      // uniform (chunks never straddle cin1 in CV); an arithmetic select -- a ?:
      // between two register arrays becomes a pointer select into scratch
      const unsigned rmask = (CV && c >= a.cin1) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int t = 0; t < XSLOTS_W; ++t) {
        const int j = wave + kConvWaves * t;
        unsigned vo = voff[t];
        if constexpr (CV) vo = voff[t] ^ ((voff[t] ^ voffr[t]) & rmask);
        if (j < XSLOTS && j * 64 + lane < C::IMG)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(st + ci * C::CIS + j * 64), 4,
                                                   vo, 0, 0, 0);
      }
    }
  };

  const int kq = lane >> 4;
  const int n = lane & 15;
  int xoff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int g = wave * NT + j;
    xoff[j] = kq * C::CIS + (g / C::TPR) * C::RW + (g % C::TPR) * 16 + n;
  }
  int woff[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) woff[m] = kq * C::COPS + a_col<3, MT>(m, kq, n);

  f32x4 acc[TD][MT][NT];
#pragma unroll
  for (int t = 0; t < TD; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[t][m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, smem);
  // small accumulator tiles (the cell ops, which accumulate) have registers to
  // spare for a prefetched residual; big tiles keep 2 WGs/CU without
  constexpr bool RES = TD * MT * NT <= 8;
  const EpiGeom<3, MT, NT, TW, TD, KD> geo(a, co0, d0, h0, w0, wave, lane);
  EpiRegs<MT, NT, TD, RES> epi;
  epi_prefetch<3, MT, NT, TW, TD, RES, KD>(a, epi, geo, b);
  for (int ch = 0; ch < nchunks; ++ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of chunk ch landed
    __syncthreads();  // ... and everyone's; everyone is done reading chunk ch-1's stage
    if (ch + 1 < nchunks) issue(ch + 1, smem + ((ch + 1) & 1) * C::STAGE);
    const float* xs = smem + (ch & 1) * C::STAGE;
    mfma_chunk<3, MT, NT, TW, TD, KD>(xs, xs + C::XS, xoff, woff, acc);
  }
  epilogue_dma<3, MT, NT, TW, TD, RES, KD>(a, acc, epi, geo, b);
}

// A launch plan: which instantiation runs a given shape (also reported by name).
struct Plan {
  int engine;  // 0 = dma (k3), 1 = 1x1 streaming, 2 = reg resample, 3 = valu (k3, cout <= 2),
               // 4 = dma depth-paired, 5 = resampled 1x1 gather-GEMM
  int mt, nt, tw, td;
};

// DMA engine: one-dimensional grid, decoded (XCD-aware) inside the kernel.
template <typename K>
int launch_dma(K kernel, const ConvArgs& a0, int th, int tw, int td, int B, hipStream_t st) {
  ConvArgs a = a0;
  a.tiles_w = (a.W + tw - 1) / tw;
  a.ntiles = a.tiles_w * ((a.H + th - 1) / th);
  a.ndz = (a.D + td - 1) / td;
  const long long n = (long long)a.ntiles * a.ndz * B * a.ncob;
  LEA_CHECK_ARG(n < (1LL << 31), "lea_conv3d: grid too large");
  a.nblk = (int)n;
  kernel<<<dim3((unsigned)n), kConvThreads, 0, st>>>(a);
  return launch_status("lea_conv3d");
}

// Instantiated DMA-engine tiles, per MT (one translation unit each, conv3d_dma_mt*.hip):
// NT in {1,2,4,8}, TW in {16,32,64} (TW=16 only for NT <= 2), TD in {1,2}, with the
// accumulator tile MT*NT*TD <= 16, minus the tiles whose unrolled operand prefetch
// does not fit 256 VGPRs (two waves per SIMD): <1,8,*,2>, <2,8,*,1>, <4,4,*,1>, <4,2,64,2>.
#define LEA_DMA_TW_ALL(X, MT, NT, TD) X(MT, NT, 16, TD) X(MT, NT, 32, TD) X(MT, NT, 64, TD)
#define LEA_DMA_TW_BIG(X, MT, NT, TD) X(MT, NT, 32, TD) X(MT, NT, 64, TD)
#define LEA_DMA_LIST_1(X)                                                               \
  LEA_DMA_TW_ALL(X, 1, 1, 1) LEA_DMA_TW_ALL(X, 1, 2, 1) LEA_DMA_TW_BIG(X, 1, 4, 1)      \
  LEA_DMA_TW_BIG(X, 1, 8, 1) LEA_DMA_TW_ALL(X, 1, 1, 2) LEA_DMA_TW_ALL(X, 1, 2, 2)      \
  LEA_DMA_TW_BIG(X, 1, 4, 2)
#define LEA_DMA_LIST_2(X)                                                               \
  LEA_DMA_TW_ALL(X, 2, 1, 1) LEA_DMA_TW_ALL(X, 2, 2, 1) LEA_DMA_TW_BIG(X, 2, 4, 1)      \
  LEA_DMA_TW_ALL(X, 2, 1, 2) LEA_DMA_TW_ALL(X, 2, 2, 2) LEA_DMA_TW_BIG(X, 2, 4, 2)
#define LEA_DMA_LIST_3(X)                                                               \
  LEA_DMA_TW_ALL(X, 3, 1, 1) LEA_DMA_TW_ALL(X, 3, 2, 1) LEA_DMA_TW_BIG(X, 3, 4, 1)      \
  LEA_DMA_TW_ALL(X, 3, 1, 2) LEA_DMA_TW_ALL(X, 3, 2, 2)
#define LEA_DMA_LIST_4(X)                                                               \
  LEA_DMA_TW_ALL(X, 4, 1, 1) LEA_DMA_TW_ALL(X, 4, 2, 1) LEA_DMA_TW_ALL(X, 4, 1, 2)      \
  X(4, 2, 16, 2) X(4, 2, 32, 2)

// Cost-volume-input tiles (matching-net stem0): the planner's 8 x 16 / 4 x 16 tiles.
#define LEA_DMA_CV_LIST(X, MT) \
  X(MT, 1, 16, 1, 3) X(MT, 2, 16, 1, 3) X(MT, 1, 16, 2, 3) X(MT, 2, 16, 2, 3)

// 2D (KD = 1) tiles for the feature net: one plane per workgroup.
#define LEA_DMA2D_LIST(X, MT) X(MT, 1, 16, 1, 1) X(MT, 2, 16, 1, 1)
// Depth-paired tiles (KD = 4, couts <= 8; grid steps two planes per workgroup).
#define LEA_DMA_DP_LIST(X) X(1, 1, 16, 1, 4) X(1, 2, 16, 1, 4)

// Per-MT entry points (defined by LEA_DMA_TU in conv3d_dma_mt*.hip).  lds_bytes
// returns 0 for a tile that is not instantiated; run returns LEA_E_UNSUPPORTED.
#define LEA_DMA_DECL(MT)                                                  \
  int dma_lds_bytes_mt##MT(int nt, int tw, int td);                       \
  int run_dma_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st);   \
  int run_dma2d_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st);
#define LEA_DMA_DECL_CV(MT) \
  int run_dma_cv_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st);
LEA_DMA_DECL_CV(1)
LEA_DMA_DECL_CV(2)
LEA_DMA_DECL_CV(3)
LEA_DMA_DECL_CV(4)
#undef LEA_DMA_DECL_CV
int run_dma_dp(const Plan& p, const ConvArgs& a, int B, hipStream_t st);  // conv3d_dma_mt1.hip
// the few-channel 2D 3x3 tile (conv2d_small.hip): eligibility and launch
bool conv2d_small_ok(int cin, int cout);
int run_conv2d_small(const ConvArgs& a, int B, hipStream_t st);
LEA_DMA_DECL(1)
LEA_DMA_DECL(2)
LEA_DMA_DECL(3)
LEA_DMA_DECL(4)
#undef LEA_DMA_DECL

#define LEA_DMA_LDS_CASE(MT, NT, TW, TD) \
  if (nt == NT && tw == TW && td == TD) return 2 * TileCfg<3, MT, NT, TW, TD>::STAGE * 4;
#define LEA_DMA_RUN_CASE(MT, NT, TW, TD)                                                      \
  if (p.nt == NT && p.tw == TW && p.td == TD)                                                 \
    return launch_dma(conv3d_dma_kernel<MT, NT, TW, TD>, a, TileCfg<3, MT, NT, TW, TD>::TH, TW, \
                      TD, B, st);
#define LEA_DMA2D_RUN_CASE(MT, NT, TW, TD, KD)                                           \
  if (p.nt == NT && p.tw == TW && p.td == TD)                                             \
    return launch_dma(conv3d_dma_kernel<MT, NT, TW, TD, KD>,                              \
                      a, TileCfg<3, MT, NT, TW, TD, KD>::TH, TW, TD, B, st);
#define LEA_DMA_DP_RUN_CASE(MT, NT, TW, TD, KD)                                          \
  if (p.nt == NT && p.tw == TW)                                                           \
    return launch_dma(conv3d_dma_kernel<MT, NT, TW, TD, KD>,                              \
                      a, TileCfg<3, MT, NT, TW, TD, KD>::TH, TW, 2, B, st);
#define LEA_DMA_CV_RUN_CASE(MT, NT, TW, TD, KD)                                          \
  if (p.nt == NT && p.tw == TW && p.td == TD)                                             \
    return launch_dma(conv3d_dma_kernel<MT, NT, TW, TD, KD, true>,                        \
                      a, TileCfg<3, MT, NT, TW, TD, KD>::TH, TW, TD, B, st);
#define LEA_DMA_TU(MT)                                                            \
  int dma_lds_bytes_mt##MT(int nt, int tw, int td) {                              \
    LEA_DMA_LIST_##MT(LEA_DMA_LDS_CASE) return 0;                                 \
  }                                                                               \
  int run_dma_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st) {   \
    LEA_DMA_LIST_##MT(LEA_DMA_RUN_CASE)                                           \
    set_error("lea_conv3d: no DMA tile <%d, %d, %d, %d>", MT, p.nt, p.tw, p.td);  \
    return LEA_E_UNSUPPORTED;                                                     \
  }                                                                               \
  int run_dma2d_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st) { \
    LEA_DMA2D_LIST(LEA_DMA2D_RUN_CASE, MT)                                        \
    set_error("lea_conv2d: no DMA tile <%d, %d, %d, 1, 1>", MT, p.nt, p.tw);     \
    return LEA_E_UNSUPPORTED;                                                     \
  }                                                                               \
  int run_dma_cv_mt##MT(const Plan& p, const ConvArgs& a, int B, hipStream_t st) { \
    LEA_DMA_CV_LIST(LEA_DMA_CV_RUN_CASE, MT)                                      \
    set_error("lea_conv3d_costvolume: no tile <%d, %d, %d, %d>", MT, p.nt, p.tw, p.td); \
    return LEA_E_UNSUPPORTED;                                                     \
  }

}  // namespace lea
