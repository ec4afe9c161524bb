// ConvBR3d dispatch and C ABI, plus the register-staged (resampling), 1x1 streaming
// and VALU engines.  The DMA engine and the shared tile machinery live in
// conv3d_impl.h (header comment there describes the GEMM mapping).
#include "conv3d_impl.h"

namespace lea {

// ------------------------------------------------- register-staged engine (+ resample)
template <int KS, int MT, int NT, int TW, bool RS>
__global__ __launch_bounds__(kConvThreads, 2) void conv3d_reg_kernel(const ConvArgs a) {
  using C = TileCfg<KS, MT, NT, TW>;
  constexpr int CIN_B = C::CIN_B;
  __shared__ __attribute__((aligned(16))) float smem[C::STAGE];
  __shared__ Axis tabs[RS ? (KS + C::RH + C::RW) : 1];
  float* xs = smem;
  float* ws = smem + C::XS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tile = blockIdx.x;
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * TW;
  const int d0 = blockIdx.y;
  const int b = blockIdx.z / a.ncob;
  const int co0 = (blockIdx.z - b * a.ncob) * C::COP;
  const int nchunks = (a.cin + CIN_B - 1) / CIN_B;
  const float* wp = a.wp + (long long)(co0 / C::COP) * nchunks * C::WS;
  const long long HW = (long long)a.H * a.W;
  const long long DHW = HW * a.D;
  const long long HWi = (long long)a.Hi * a.Wi;
  const long long DHWi = HWi * a.Di;

  if constexpr (RS) {  // source index/weights of every staged d, h, w (aten align_corners=True)
    for (int i = tid; i < KS + C::RH + C::RW; i += kConvThreads) {
      if (i < KS) {
        const int d = d0 + i - C::PAD;
        tabs[i] = axis_index(a.rd, (unsigned)d < (unsigned)a.D ? d : 0, a.Di, a.D, 1);
      } else if (i < KS + C::RH) {
        const int h = h0 + (i - KS) - C::PAD;
        tabs[i] = axis_index(a.rh, (unsigned)h < (unsigned)a.H ? h : 0, a.Hi, a.H, 1);
      } else {
        const int w = w0 + (i - KS - C::RH) - C::PAD;
        tabs[i] = axis_index(a.rw, (unsigned)w < (unsigned)a.W ? w : 0, a.Wi, a.W, 1);
      }
    }
  }

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
  for (int m = 0; m < MT; ++m) woff[m] = kq * C::COPS + a_col<KS, MT>(m, kq, n);

  f32x4 acc[1][MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[0][m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < nchunks; ++ch) {
    const int c0 = ch * CIN_B;
    __syncthreads();  // previous chunk's reads are done (and the axis tables are ready)
    {
      const float4* src = reinterpret_cast<const float4*>(wp + (long long)ch * C::WS);
      float4* dst = reinterpret_cast<float4*>(ws);
#pragma unroll 4
      for (int i = tid; i < C::WS / 4; i += kConvThreads) dst[i] = src[i];
    }
    // RESAMPLE: 8 gathered loads per staged value; unroll deep enough that a
    // thread keeps ~64 loads in flight (the loop is latency-bound otherwise)
#pragma unroll 8
    for (int i = tid; i < CIN_B * C::IMG; i += kConvThreads) {
      const int ci = i / C::IMG;
      int rem = i - ci * C::IMG;
      const int kd = rem / C::PLANE;
      rem -= kd * C::PLANE;
      const int rr = rem / C::RW;
      const int cc = rem - rr * C::RW;
      const int d = d0 + kd - C::PAD;
      const int h = h0 + rr - C::PAD;
      const int w = w0 + cc - C::PAD;
      const int c = c0 + ci;
      float v = 0.f;
      if ((unsigned)d < (unsigned)a.D && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W &&
          c < a.cin) {
        const float* src = (c < a.cin1) ? a.x + (long long)b * a.xbs + (long long)c * (RS ? DHWi : DHW)
                                        : a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * (RS ? DHWi : DHW);
        if constexpr (RS) {
          const Axis ad = tabs[kd], ah = tabs[KS + rr], aw = tabs[KS + C::RH + cc];
          const float* p00 = src + ad.i0 * HWi + (long long)ah.i0 * a.Wi;
          const float* p01 = src + ad.i0 * HWi + (long long)ah.i1 * a.Wi;
          const float* p10 = src + ad.i1 * HWi + (long long)ah.i0 * a.Wi;
          const float* p11 = src + ad.i1 * HWi + (long long)ah.i1 * a.Wi;
          v = trilerp(ad, ah, aw, p00, p01, p10, p11);
        } else {
          v = src[(long long)d * HW + (long long)h * a.W + w];
        }
      }
      xs[ci * C::CIS + kd * C::PLANE + rr * C::RW + cc] = v;
    }
    __syncthreads();
    mfma_chunk<KS, MT, NT, TW, 1>(xs, ws, xoff, woff, acc);
  }
  epilogue<KS, MT, NT, TW, 1>(a, acc, b, co0, d0, h0, w0, wave, lane);
}

// ------------------------------------- 1x1 of a trilinearly resampled input, gather-GEMM
// The cell preprocess after a level change (skip_model_3d.py:44-53: trilinear
// align_corners=True, then the 1x1 ConvBR) without the resampled tensor and without
// staging: lane (g, n) of a wave forms its own B fragment of v_mfma_f32_16x16x4_f32 --
// input channel 4 s + g of output voxel v0 + n -- from the 8 corners of aten's
// trilinear expression (trilerp: same operands, same order as the register-staged
// engine; the MFMA sums may associate differently), read by buffer loads (padding channels' operands forced to
// 0).  The A fragments (the k = 1 packing of this cout block) sit in LDS.  A wave walks
// `tpw` consecutive 16-voxel tiles of the flat output run; every k-step's loads of a
// 32-channel chunk are issued before its MFMAs.  HBM-bound: the input is read once.
constexpr int kRsMaxCin = 128;
template <int MT>
__global__ __launch_bounds__(256) void conv1x1_rs_f32_kernel(const ConvArgs a, int tpw) {
#pragma clang fp contract(off)
  constexpr int COP = 16 * MT;
  constexpr bool SWZ = (COP % 32) == 0;
  __shared__ __attribute__((aligned(16))) float ws[kRsMaxCin * COP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, n = lane & 15;
  const int b = blockIdx.y / a.ncob, cob = blockIdx.y - b * a.ncob;
  const int co0 = cob * COP;
  const int nch = (a.cin + 31) / 32;  // 32-channel chunks of the packing
  {
    const float4* src = reinterpret_cast<const float4*>(a.wp + (long long)cob * nch * 32 * COP);
    float4* dst = reinterpret_cast<float4*>(ws);
    for (int i = threadIdx.x; i < nch * 32 * COP / 4; i += 256) dst[i] = src[i];
  }
  float sc[MT][4], sh[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * m + 4 * g + r;
      sc[m][r] = (a.scale && co < a.cout) ? a.scale[co] : 1.f;
      sh[m][r] = (a.scale && co < a.cout) ? a.shift[co] : 0.f;
    }
  __syncthreads();
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const int HWo = a.H * a.W;
  const long long vout = (long long)HWo * a.D;
  const unsigned HWi = (unsigned)(a.Hi * a.Wi), vin = HWi * (unsigned)a.Di;  // host: cin * vin * 4 < 2^32
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)b * a.xbs), 0, (int)(unsigned)((long long)a.cin * vin * 4), 0x00020000);
  const long long t0 = ((long long)blockIdx.x * 4 + wave) * tpw;
  for (int tt = 0; tt < tpw; ++tt) {
    const long long v0 = (t0 + tt) * 16;
    if (v0 >= vout) break;
    const long long v = min(v0 + n, vout - 1);
    const int od = (int)(v / HWo), rem = (int)(v - (long long)od * HWo);
    const int oh = rem / a.W, ow = rem - oh * a.W;
    const Axis ad = axis_index(a.rd, od, a.Di, a.D, 1), ah = axis_index(a.rh, oh, a.Hi, a.H, 1),
               aw = axis_index(a.rw, ow, a.Wi, a.W, 1);
    const unsigned r00 = ((unsigned)ad.i0 * HWi + (unsigned)(ah.i0 * a.Wi)) * 4u;
    const unsigned r01 = ((unsigned)ad.i0 * HWi + (unsigned)(ah.i1 * a.Wi)) * 4u;
    const unsigned r10 = ((unsigned)ad.i1 * HWi + (unsigned)(ah.i0 * a.Wi)) * 4u;
    const unsigned r11 = ((unsigned)ad.i1 * HWi + (unsigned)(ah.i1 * a.Wi)) * 4u;
    const unsigned w0 = (unsigned)aw.i0 * 4u, w1 = (unsigned)aw.i1 * 4u;
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
      float c[8][8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int ci = ch * 32 + 4 * s + g;
        const unsigned co = ci < a.cin ? (unsigned)ci * vin * 4u : 0u;  // padding channels: bv = 0 below
        const unsigned rr[4] = {r00, r01, r10, r11};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          c[s][2 * q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, co + rr[q] + w0, 0, 0));
          c[s][2 * q + 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, co + rr[q] + w1, 0, 0));
        }
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float* e = c[s];
        const int ci = ch * 32 + 4 * s + g;
        // padding channels (ci >= cin) read channel 0's voxels: their operand is forced to 0
        // so a non-finite input there cannot reach other outputs through the zero weights
        const float bv = ci >= a.cin ? 0.f :
            ad.l0 * (ah.l0 * (aw.l0 * e[0] + aw.l1 * e[1]) + ah.l1 * (aw.l0 * e[2] + aw.l1 * e[3])) +
            ad.l1 * (ah.l0 * (aw.l0 * e[4] + aw.l1 * e[5]) + ah.l1 * (aw.l0 * e[6] + aw.l1 * e[7]));
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int col = 16 * m + n;
          const float av = ws[ci * COP + ((SWZ && (ci & 1)) ? (col ^ 16) : col)];
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[m], 0, 0, 0);
        }
      }
    }
    // D (lane, r) = out[co0 + 16 m + 4 g + r][v0 + n]
    if (v0 + n < vout) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + 16 * m + 4 * g + r;
          if (co >= a.cout) continue;
          float y = acc[m][r] * sc[m][r] + sh[m][r];
          if (relu) y = fmaxf(y, 0.f);
          const long long o = (long long)co * vout + v0 + n;
          if (resid) y += a.res[(long long)b * a.rbs + o];
          a.y[(long long)b * a.ybs + o] = y;
        }
    }
  }
}

// ---------------------------------------------------------- 1x1x1 streaming engine
// A 1x1 ConvBR is a [cout x cin] x [cin x voxels] GEMM that reads every input
// element exactly once: HBM-bound.  No LDS for X: each lane's B fragment
// (X[ci = 4s + kq][v = v0 + 16j + n]) is loaded straight from global memory
// (16 consecutive floats per 16-lane group), all CIN_B/4 k-steps of a chunk
// issued before its MFMAs so a chunk's loads are in flight together.  Weights of
// the chunk (32 x COPS floats) are staged in LDS.  The volume is treated as a
// flat run of D*H*W voxels.  VEC (r05): lane n owns the NT consecutive voxels v0 + NT n + j
// (column n of tile j) instead of v0 + 16 j + n, so its loads, residual reads and stores are
// NT-float vectors -- 16 lanes cover 64 NT contiguous bytes per instruction instead of 64
// (host: every base, batch stride and D*H*W a multiple of NT floats).  Each output's k-step
// sequence is unchanged: bit-identical.
template <int MT, int NT, bool VEC>
__global__ __launch_bounds__(kConvThreads) void conv1x1_kernel(const ConvArgs a) {
  using P = PackCfg<1, MT>;
  constexpr int CIN_B = P::CIN_B;
  constexpr int KS = CIN_B / 4;
  using vecf = float __attribute__((ext_vector_type(NT)));
  __shared__ __attribute__((aligned(16))) float ws[P::CHUNK];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.y / a.ncob;
  const int co0 = (blockIdx.y - b * a.ncob) * P::COP;
  const int nchunks = (a.cin + CIN_B - 1) / CIN_B;
  const float* wp = a.wp + (long long)(co0 / P::COP) * nchunks * P::CHUNK;
  const long long V = (long long)a.D * a.H * a.W;
  const long long v0 = ((long long)blockIdx.x * kConvWaves + wave) * NT * 16;
  const int kq = lane >> 4, n = lane & 15;
  // voxel of (lane, tile j): VEC v0 + NT n + j, else v0 + 16 j + n
  auto vox = [&](int j) -> long long { return VEC ? v0 + NT * n + j : v0 + j * 16 + n; };
  const bool full = VEC && vox(NT - 1) < V;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < nchunks; ++ch) {
    float bv[KS][NT];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c = ch * CIN_B + 4 * s + kq;
      const float* src = (c < a.cin1) ? a.x + (long long)b * a.xbs + (long long)c * V
                                      : a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * V;
      if (VEC && full && c < a.cin) {
        const vecf t = *reinterpret_cast<const vecf*>(src + vox(0));
#pragma unroll
        for (int j = 0; j < NT; ++j) bv[s][j] = t[j];
      } else {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const long long v = vox(j);
          bv[s][j] = (c < a.cin && v < V) ? src[v] : 0.f;
        }
      }
    }
    __syncthreads();  // previous chunk's weight reads are done
    {
      const float4* src = reinterpret_cast<const float4*>(wp + (long long)ch * P::CHUNK);
      float4* dst = reinterpret_cast<float4*>(ws);
#pragma unroll
      for (int i = tid; i < P::CHUNK / 4; i += kConvThreads) dst[i] = src[i];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float av[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = ws[(4 * s + kq) * P::COPS + a_col<1, MT>(m, kq, n)];
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[s][j], acc[m][j], 0, 0, 0);
    }
  }

  const bool relu = a.flags & LEA_RELU;
  const bool resid = a.flags & LEA_RESIDUAL;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + m * 16 + kq * 4 + r;
      if (co >= a.cout) continue;
      const float sc = a.scale ? a.scale[co] : 1.f;
      const float sh = a.shift ? a.shift[co] : 0.f;
      if (VEC && full) {
        const long long o = (long long)co * V + vox(0);
        vecf val;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          val[j] = acc[m][j][r] * sc + sh;
          if (relu) val[j] = fmaxf(val[j], 0.f);
        }
        if (resid) {
          const vecf rv = *reinterpret_cast<const vecf*>(a.res + (long long)b * a.rbs + o);
#pragma unroll
          for (int j = 0; j < NT; ++j) val[j] += rv[j];
        }
        *reinterpret_cast<vecf*>(a.y + (long long)b * a.ybs + o) = val;
        continue;
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const long long v = vox(j);
        if (v >= V) continue;
        const long long o = (long long)co * V + v;
        float val = acc[m][j][r] * sc + sh;
        if (relu) val = fmaxf(val, 0.f);
        if (resid) val += a.res[(long long)b * a.rbs + o];
        a.y[(long long)b * a.ybs + o] = val;
      }
    }
  }
}

// ------------------------------------------------- VALU engine for cout <= 2 (k=3)
// The head's last_3 (32 -> 1, skip_model_3d.py:132) would use 1/16 of each MFMA's
// rows.  Here every thread owns 2 adjacent output voxels of a 8 x 64 plane tile
// and runs plain FMAs; weights are wave-uniform (scalar loads from the packed
// chunk), the input halo block comes by the same LDS-DMA pieces as the MFMA
// engine (double-buffered), read back as ds_read_b64 pairs.
template <int COUT>
__global__ __launch_bounds__(kConvThreads) void conv3d_valu_kernel(const ConvArgs a) {
  constexpr int TH = 8, TW = 64, RH = TH + 2, RW = TW + 2, PLANE = RH * RW, IMG = 3 * PLANE;
  constexpr int CIN_B = PackCfg<3, 1>::CIN_B;
  constexpr int CIS = (IMG + 15) / 16 * 16;
  constexpr int STAGE = CIN_B * CIS;
  constexpr int XSLOTS = (IMG + 63) / 64;
  constexpr int XSLOTS_W = (XSLOTS + kConvWaves - 1) / kConvWaves;
  constexpr int CHUNK = PackCfg<3, 1>::CHUNK;  // packed layout of mt=1: [tap][ci][16]
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h0 = (blockIdx.x / a.tiles_w) * TH;
  const int w0 = (blockIdx.x % a.tiles_w) * TW;
  const int d0 = blockIdx.y;
  const int b = blockIdx.z;
  const int nchunks = (a.cin + CIN_B - 1) / CIN_B;
  const int HW = a.H * a.W;
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;

  unsigned voff[XSLOTS_W];
#pragma unroll
  for (int t = 0; t < XSLOTS_W; ++t) {
    const int e = (wave + kConvWaves * t) * 64 + lane;
    unsigned v = 0xFFFFFFF0u;
    if (e < IMG) {
      const int kd = e / PLANE;
      const int r = e - kd * PLANE;
      const int rr = r / RW;
      const int cc = r - rr * RW;
      const int d = d0 + kd - 1, h = h0 + rr - 1, w = w0 + cc - 1;
      if ((unsigned)d < (unsigned)a.D && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        v = (unsigned)(d * HW + h * a.W + w) * 4u;
    }
    voff[t] = v;
  }
  auto issue = [&](int ch, float* st) {
#pragma unroll
    for (int ci = 0; ci < CIN_B; ++ci) {
      const int c = ch * CIN_B + ci;
      const float* base = a.x;
      unsigned n = 0;
      if (c < a.cin1) {
        base = a.x + (long long)b * a.xbs + (long long)c * HW * a.D;
        n = nrec;
      } else if (c < a.cin) {
        base = a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * HW * a.D;
        n = nrec;
      }
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
#pragma unroll
      for (int t = 0; t < XSLOTS_W; ++t) {
        const int j = wave + kConvWaves * t;
        if (j < XSLOTS && j * 64 + lane < IMG)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(st + ci * CIS + j * 64), 4,
                                                   voff[t], 0, 0, 0);
      }
    }
  };

  const int row = tid >> 5;        // 0..7
  const int col = (tid & 31) * 2;  // 0..62
  float acc[COUT][2];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc[co][0] = acc[co][1] = 0.f;

  issue(0, smem);
  for (int ch = 0; ch < nchunks; ++ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ch + 1 < nchunks) issue(ch + 1, smem + ((ch + 1) & 1) * STAGE);
    const float* xs = smem + (ch & 1) * STAGE;
    const float* wc = a.wp + (long long)ch * CHUNK;
#pragma unroll
    for (int ci = 0; ci < CIN_B; ++ci) {
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* p = xs + ci * CIS + kd * PLANE + (row + kh) * RW + col;
          const float2 x01 = *reinterpret_cast<const float2*>(p);
          const float2 x23 = *reinterpret_cast<const float2*>(p + 2);
          const float xv[4] = {x01.x, x01.y, x23.x, x23.y};
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int tap = (kd * 3 + kh) * 3 + kw;
#pragma unroll
            for (int co = 0; co < COUT; ++co) {
              const float wv = wc[(tap * CIN_B + ci) * 16 + co];
              acc[co][0] = fmaf(wv, xv[kw], acc[co][0]);
              acc[co][1] = fmaf(wv, xv[kw + 1], acc[co][1]);
            }
          }
        }
      }
    }
  }
  const long long HWl = HW, DHW = (long long)HW * a.D;
  const int h = h0 + row;
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    if (co >= a.cout) continue;
    const float sc = a.scale ? a.scale[co] : 1.f;
    const float sh = a.shift ? a.shift[co] : 0.f;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int w = w0 + col + e;
      if (h >= a.H || w >= a.W) continue;
      const long long o = (long long)co * DHW + (long long)d0 * HWl + (long long)h * a.W + w;
      float v = acc[co][e] * sc + sh;
      if (a.flags & LEA_RELU) v = fmaxf(v, 0.f);
      if (a.flags & LEA_RESIDUAL) v += a.res[(long long)b * a.rbs + o];
      a.y[(long long)b * a.ybs + o] = v;
    }
  }
}

// ------------------------------------------------------------------- weight packing
// Packed layout: [ceil(cout/COP)][ceil(cin/CIN_B)][KS^3][CIN_B][COP], zero outside (cin, cout);
// rows of odd input channels swizzled (PackCfg::SWZ, a_col).
template <int KS, int MT, int KD = KS>
__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ packed,
                                    int cout, int cin, int nchunks, long long total) {
  using P = PackCfg<KS, MT, KD>;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(i % P::COPS);
    long long r = i / P::COPS;
    const int cb = (int)(r % P::CIN_B);
    r /= P::CIN_B;
    const int tap = (int)(r % P::KT);
    r /= P::KT;
    const int ch = (int)(r % nchunks);
    const int co = (int)(r / nchunks) * P::COP + ((P::SWZ && (cb & 1)) ? (col ^ 16) : col);
    const int ci = ch * P::CIN_B + cb;
    float v = 0.f;
    if (co < cout && ci < cin) v = w[((long long)co * cin + ci) * P::KT + tap];
    packed[i] = v;
  }
}

// Depth-paired packing (couts <= 8): [chunk][p = 0..3][kh][kw][CIN_B][16] with
// column 8t + c = W[c][ci][kd = p - t][kh][kw] (zero when kd is outside 0..2).
__global__ void pack_weights_dp_kernel(const float* __restrict__ w, float* __restrict__ packed,
                                       int cout, int cin, int nchunks, long long total) {
  using P = PackCfg<3, 1, 4>;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(i % P::COPS);
    long long r = i / P::COPS;
    const int cb = (int)(r % P::CIN_B);
    r /= P::CIN_B;
    const int tap = (int)(r % P::KT);  // p * 9 + kh * 3 + kw
    const int ch = (int)(r / P::KT);
    const int t = col / 8, co = col % 8;
    const int kd = tap / 9 - t, khw = tap % 9;
    const int ci = ch * P::CIN_B + cb;
    float v = 0.f;
    if (kd >= 0 && kd < 3 && co < cout && ci < cin && ch < nchunks)
      v = w[((long long)co * cin + ci) * 27 + kd * 9 + khw];
    packed[i] = v;
  }
}

// Rows (x16) of the output-channel block a workgroup owns: the smallest of
// 16/32/48 that holds cout, else the 48- or 64-row blocking with less padding.
inline int mt_for(int cout) {
  if (cout <= 16) return 1;
  if (cout <= 32) return 2;
  if (cout <= 48) return 3;
  return ((cout + 47) / 48) * 48 < ((cout + 63) / 64) * 64 ? 3 : 4;
}

template <int KS, int MT, int KD = KS>
size_t packed_floats_t(int cout, int cin) {
  using P = PackCfg<KS, MT, KD>;
  return (size_t)((cout + P::COP - 1) / P::COP) * ((cin + P::CIN_B - 1) / P::CIN_B) * P::CHUNK;
}

// k = 3 convs with 3..8 output channels run depth-paired (conv3d_dma_kernel, KD = 4)
inline bool depth_paired(int cout, int k) { return k == 3 && cout > 2 && cout <= 8; }

size_t packed_floats(int cout, int cin, int k) {
  const int mt = mt_for(cout);
  if (depth_paired(cout, k)) return packed_floats_t<3, 1, 4>(cout, cin);
  if (k == 3)
    return mt == 1 ? packed_floats_t<3, 1>(cout, cin)
           : mt == 2 ? packed_floats_t<3, 2>(cout, cin)
           : mt == 3 ? packed_floats_t<3, 3>(cout, cin) : packed_floats_t<3, 4>(cout, cin);
  return mt == 1 ? packed_floats_t<1, 1>(cout, cin)
         : mt == 2 ? packed_floats_t<1, 2>(cout, cin)
         : mt == 3 ? packed_floats_t<1, 3>(cout, cin) : packed_floats_t<1, 4>(cout, cin);
}

// ------------------------------------------------------------------------- dispatch

// LDS bytes of a double-buffered DMA-engine workgroup (0 if not instantiated).
inline int dma_lds_bytes(int mt, int nt, int tw, int td) {
  switch (mt) {
    case 1: return dma_lds_bytes_mt1(nt, tw, td);
    case 2: return dma_lds_bytes_mt2(nt, tw, td);
    case 3: return dma_lds_bytes_mt3(nt, tw, td);
    default: return dma_lds_bytes_mt4(nt, tw, td);
  }
}

int g_tile_override[3] = {0, 0, 0};

inline bool prefer_tw64(int W) {
  const int w64 = (W + 63) / 64 * 64, w32 = (W + 31) / 32 * 32;
  return (w64 - W) <= (w32 - W) || W >= 1024;
}

// lea_conv3d_set_rs_gather: 1 (default) = the resampled 1x1 convs on the gather-GEMM
// (conv1x1_rs_f32_kernel), 0 = the register-staged engine
int g_rs_gather = 1;

inline Plan make_plan(int B, int cout, int D, int H, int W, int k, bool resample) {
  Plan p;
  p.td = 1;
  p.mt = mt_for(cout);
  // same-box sweep (r02): the gather-GEMM wins on the L1 -> L2 preprocess (64 channels,
  // 61 K output voxels: 35 -> 29.5 us) and loses on the L0 -> L1 ones (32 channels, 491 K:
  // 122 -> 136 us: twice the load instructions of the staged engine's row gathers)
  if (k == 1 && resample && g_rs_gather && (long long)B * D * H * W <= 131072) {
    p.engine = 5;
    p.nt = 0;
    p.tw = 0;
    return p;
  }
  if (k == 1 && !resample) {
    p.engine = 1;
    p.nt = 4;
    p.tw = 0;
    const long long vox = (long long)D * H * W;
    if ((vox + kConvWaves * 64 - 1) / (kConvWaves * 64) * B < 512) p.nt = 2;
    return p;
  }
  if (k == 3 && cout <= 2 && !resample) {
    p.engine = 3;
    p.nt = 0;
    p.tw = 64;
    return p;
  }
  if (depth_paired(cout, k) && !resample) {  // engine 4: two planes x 8 couts per tile
    p.engine = 4;
    p.mt = 1;
    p.tw = 16;
    p.td = 1;
    const long long wgs8 = (long long)((W + 15) / 16) * ((H + 7) / 8) * ((D + 1) / 2) * B;
    p.nt = wgs8 >= 512 ? 2 : 1;
    return p;
  }
  p.engine = resample ? 2 : 0;
  p.tw = prefer_tw64(W) ? 64 : 32;
  p.td = 1;
  if (resample) {
    // register-staged resampling engine; for k = 1 (the level-change preprocess,
    // latency-bound gathers) quarter-height tiles shrink the LDS stage so 8
    // workgroups share a CU and keep more loads in flight
    p.nt = (k == 1) ? (p.mt == 1 ? 2 : 1) : (p.mt == 1 ? 8 : 4);
    return p;
  }
  const long long ncob = (cout + p.mt * 16 - 1) / (p.mt * 16);
  if (g_tile_override[0] > 0) {  // lea_conv3d_set_tile_override (tuning tools)
    p.nt = g_tile_override[0];
    p.tw = g_tile_override[1];
    p.td = g_tile_override[2];
    return p;
  }
  // Tile = 8 rows x 16 columns (NT=2, TW=16) x TD planes for every layer: the r01
  // sweep (tools/conv_sweep.py, profiles/r01_conv_sweep.txt) found it best or within
  // 1% on all nine matching-net layer shapes -- the narrow tile wastes no columns at
  // W = 80/160/320, and 51 KB of LDS lets 3 workgroups share a CU.  Two output
  // planes per workgroup unless that leaves fewer than 1.5 workgroups per CU.
  auto wgs = [&](int nt, int td) {
    const int th = kConvWaves * nt;
    return (long long)((W + 15) / 16) * ((H + th - 1) / th) * ((D + td - 1) / td) * B * ncob;
  };
  p.tw = 16;
  p.nt = 2;
  p.td = wgs(2, 2) >= 384 ? 2 : 1;
  if (p.td == 1 && wgs(2, 1) < 256) p.nt = 1;
  return p;
}

template <typename K>
int launch(K kernel, const ConvArgs& a0, int th, int tw, int B, hipStream_t st, int td = 1) {
  ConvArgs a = a0;
  const long long nt = (long long)((a.W + tw - 1) / tw) * ((a.H + th - 1) / th);
  LEA_CHECK_ARG(nt < (1LL << 31) && a.D <= 65535 && (long long)B * a.ncob <= 65535,
                "lea_conv3d: grid too large");
  a.tiles_w = (a.W + tw - 1) / tw;
  dim3 grid((unsigned)nt, (a.D + td - 1) / td, B * a.ncob);
  kernel<<<grid, kConvThreads, 0, st>>>(a);
  return launch_status("lea_conv3d");
}

#define LEA_TILE_TH(KS, MT, NT, TW) (TileCfg<KS, MT, NT, TW>::TH)

template <int KS, int MT, int NT>
int run_rs(const ConvArgs& a, int tw, int B, hipStream_t st) {
  if (tw == 64) return launch(conv3d_reg_kernel<KS, MT, NT, 64, true>, a, LEA_TILE_TH(KS, MT, NT, 64), 64, B, st);
  return launch(conv3d_reg_kernel<KS, MT, NT, 32, true>, a, LEA_TILE_TH(KS, MT, NT, 32), 32, B, st);
}

int g_1x1_vec = 1;  // lea_conv1x1_set_vector: the NT-float vector form of conv1x1_kernel

template <int MT, int NT>
int launch_1x1(const ConvArgs& a, int B, hipStream_t st) {
  const long long vox = (long long)a.D * a.H * a.W;
  const long long per = kConvWaves * NT * 16;
  const long long gx = (vox + per - 1) / per;
  LEA_CHECK_ARG(gx < (1LL << 31) && (long long)B * a.ncob <= 65535, "lea_conv3d: grid too large");
  // the vector form needs every per-channel and per-batch base on an NT-float boundary
  auto al = [](const void* q) { return q == nullptr || ((uintptr_t)q % (NT * 4)) == 0; };
  const bool vec = g_1x1_vec && vox % NT == 0 && al(a.x) && al(a.x2) && al(a.y) && al(a.res) &&
                   a.xbs % NT == 0 && a.x2bs % NT == 0 && a.ybs % NT == 0 && a.rbs % NT == 0;
  if (vec) conv1x1_kernel<MT, NT, true><<<dim3((unsigned)gx, B * a.ncob), kConvThreads, 0, st>>>(a);
  else conv1x1_kernel<MT, NT, false><<<dim3((unsigned)gx, B * a.ncob), kConvThreads, 0, st>>>(a);
  return launch_status("lea_conv3d");
}

int run_1x1(const Plan& p, const ConvArgs& a, int B, hipStream_t st) {
  if (p.mt == 1) return p.nt == 4 ? launch_1x1<1, 4>(a, B, st) : launch_1x1<1, 2>(a, B, st);
  if (p.mt == 2) return p.nt == 4 ? launch_1x1<2, 4>(a, B, st) : launch_1x1<2, 2>(a, B, st);
  if (p.mt == 3) return p.nt == 4 ? launch_1x1<3, 4>(a, B, st) : launch_1x1<3, 2>(a, B, st);
  return p.nt == 4 ? launch_1x1<4, 4>(a, B, st) : launch_1x1<4, 2>(a, B, st);
}

template <int MT>
int launch_rs_gather(ConvArgs a, int B, hipStream_t st) {
  const long long vout = (long long)a.D * a.H * a.W;
  const long long tiles = (vout + 15) / 16;
  // about 8192 waves over the batch and cout blocks, each walking tpw tiles
  const long long tpw = std::max(1LL, (tiles * B * a.ncob + 8191) / 8192);
  const long long gx = (tiles + 4 * tpw - 1) / (4 * tpw);
  LEA_CHECK_ARG(gx < (1LL << 31) && (long long)B * a.ncob <= 65535, "lea_conv3d: grid too large");
  conv1x1_rs_f32_kernel<MT><<<dim3((unsigned)gx, B * a.ncob), 256, 0, st>>>(a, (int)tpw);
  return launch_status("lea_conv3d(rs gather)");
}

int run_plan(const Plan& p, ConvArgs a, int B, int k, hipStream_t st) {
  a.ncob = (a.cout + p.mt * 16 - 1) / (p.mt * 16);
  if (p.engine == 5) {
    const long long xbytes = (long long)a.cin * a.Di * a.Hi * a.Wi * 4;
    if (a.cin <= kRsMaxCin && a.cin1 == a.cin && xbytes < 0xFFFFFF00LL) {
      if (p.mt == 1) return launch_rs_gather<1>(a, B, st);
      if (p.mt == 2) return launch_rs_gather<2>(a, B, st);
      if (p.mt == 3) return launch_rs_gather<3>(a, B, st);
      return launch_rs_gather<4>(a, B, st);
    }
    // wider inputs than the LDS weight block holds: the register-staged engine
    if (p.mt == 1) return run_rs<1, 1, 2>(a, prefer_tw64(a.W) ? 64 : 32, B, st);
    if (p.mt == 2) return run_rs<1, 2, 1>(a, prefer_tw64(a.W) ? 64 : 32, B, st);
    if (p.mt == 3) return run_rs<1, 3, 1>(a, prefer_tw64(a.W) ? 64 : 32, B, st);
    return run_rs<1, 4, 1>(a, prefer_tw64(a.W) ? 64 : 32, B, st);
  }
  if (p.engine == 3) {
    if (a.cout == 1) return launch(conv3d_valu_kernel<1>, a, 8, 64, B, st);
    return launch(conv3d_valu_kernel<2>, a, 8, 64, B, st);
  }
  if (p.engine == 4) return run_dma_dp(p, a, B, st);
  if (p.engine == 0) {
    if (p.mt == 1) return run_dma_mt1(p, a, B, st);
    if (p.mt == 2) return run_dma_mt2(p, a, B, st);
    if (p.mt == 3) return run_dma_mt3(p, a, B, st);
    return run_dma_mt4(p, a, B, st);
  }
  if (p.engine == 2) {
    if (k == 3) {
      if (p.mt == 1) return run_rs<3, 1, 8>(a, p.tw, B, st);
      if (p.mt == 2) return run_rs<3, 2, 4>(a, p.tw, B, st);
      if (p.mt == 3) return run_rs<3, 3, 4>(a, p.tw, B, st);
      return run_rs<3, 4, 4>(a, p.tw, B, st);
    }
    if (p.mt == 1) return run_rs<1, 1, 2>(a, p.tw, B, st);
    if (p.mt == 2) return run_rs<1, 2, 1>(a, p.tw, B, st);
    if (p.mt == 3) return run_rs<1, 3, 1>(a, p.tw, B, st);
    return run_rs<1, 4, 1>(a, p.tw, B, st);
  }
  // 1x1x1 without resample: streaming engine over the flat voxel run
  return run_1x1(p, a, B, st);
}

thread_local char g_name[96];

const char* plan_name(const Plan& p, int k) {
  if (p.engine == 5)
    snprintf(g_name, sizeof(g_name), "conv1x1_rs_f32_kernel<%d>", p.mt);
  else if (p.engine == 3)
    snprintf(g_name, sizeof(g_name), "conv3d_valu_kernel<%d>", p.mt == 1 ? 1 : 2);
  else if (p.engine == 0)
    snprintf(g_name, sizeof(g_name), "conv3d_dma_kernel<%d, %d, %d, %d, %d, false>", p.mt, p.nt,
             p.tw, p.td, k == 2 ? 1 : 3);
  else if (p.engine == 4)
    snprintf(g_name, sizeof(g_name), "conv3d_dma_kernel<1, %d, %d, 1, 4, false>", p.nt, p.tw);
  else if (p.engine == 2)
    snprintf(g_name, sizeof(g_name), "conv3d_reg_kernel<%d, %d, %d, %d, true>", k, p.mt, p.nt, p.tw);
  else
    snprintf(g_name, sizeof(g_name), "conv1x1_kernel<%d, %d>", p.mt, p.nt);
  return g_name;
}

// ------------------------------------------------------------ 2D 3x3 (feature net)
// The feature net's Conv2d 3x3 / stride 1 / pad 1 (models/operations_2d.py:31-47)
// runs on the DMA engine as the D = 1 case of a (1, 3, 3) kernel.
size_t packed_floats_2d(int cout, int cin) {
  const int mt = mt_for(cout);
  return mt == 1 ? packed_floats_t<3, 1, 1>(cout, cin)
         : mt == 2 ? packed_floats_t<3, 2, 1>(cout, cin)
         : mt == 3 ? packed_floats_t<3, 3, 1>(cout, cin) : packed_floats_t<3, 4, 1>(cout, cin);
}

inline Plan make_plan_2d(int B, int cout, int H, int W) {
  Plan p;
  p.engine = 0;
  p.mt = mt_for(cout);
  p.tw = 16;
  p.td = 1;
  const long long ncob = (cout + p.mt * 16 - 1) / (p.mt * 16);
  const long long wgs8 = (long long)((W + 15) / 16) * ((H + 7) / 8) * B * ncob;
  p.nt = wgs8 >= 512 ? 2 : 1;  // 8 x 16 tiles, or 4 x 16 on small maps
  return p;
}

int conv_common(ConvArgs& a, int B, int k, bool resample, int dtype, void* stream) {
  clear_error();
  LEA_CHECK_ARG(a.x && a.wp && a.y, "lea_conv3d: null pointer");
  LEA_CHECK_ARG((a.scale == nullptr) == (a.shift == nullptr),
                "lea_conv3d: scale/shift must both be set or both NULL");
  LEA_CHECK_FLAGS(a.flags, LEA_RELU | LEA_RESIDUAL, "lea_conv3d");
  LEA_CHECK_ARG(!(a.flags & LEA_RESIDUAL) || a.res, "lea_conv3d: LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && a.cin > 0 && a.cout > 0 && a.D > 0 && a.H > 0 && a.W > 0,
                "lea_conv3d: bad shape B=%d cin=%d cout=%d D=%d H=%d W=%d", B, a.cin, a.cout, a.D,
                a.H, a.W);
  LEA_CHECK_ARG(a.cin1 >= 0 && a.cin1 <= a.cin && (a.cin1 == a.cin || a.x2),
                "lea_conv3d: bad channel split %d/%d", a.cin1, a.cin);
  LEA_CHECK_ARG(k == 1 || k == 3, "lea_conv3d: k=%d unsupported", k);
  LEA_CHECK_ARG((long long)a.D * a.H * a.W * 4 < (1LL << 32) &&
                    (long long)(a.cout + 63) * a.D * a.H * a.W < (1LL << 31),
                "lea_conv3d: volume too large");
  LEA_CHECK_ARG(a.x != a.y && a.x2 != a.y, "lea_conv3d: input aliases output");
  if (resample) {
    LEA_CHECK_ARG(a.Di > 0 && a.Hi > 0 && a.Wi > 0, "lea_conv3d: bad input volume");
    if (depth_paired(a.cout, k)) {
      set_error("lea_conv3d_bnrelu_resampled: k=3 with %d output channels (depth-paired packing) "
                "is not supported", a.cout);
      return LEA_E_UNSUPPORTED;
    }
  }
  if (dtype != LEA_F32) {
    set_error("lea_conv3d: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const Plan p = make_plan(B, a.cout, a.D, a.H, a.W, k, resample);
  return run_plan(p, a, B, k, as_stream(stream));
}

}  // namespace lea

extern "C" const char* lea_conv3d_kernel_name(int B, int cout, int D, int H, int W, int k,
                                              int resample) {
  if (B <= 0 || cout <= 0 || (k != 1 && k != 3) || D <= 0 || H <= 0 || W <= 0) return nullptr;
  return lea::plan_name(lea::make_plan(B, cout, D, H, W, k, resample != 0), k);
}

extern "C" int lea_conv3d_set_rs_gather(int on) {
  lea::clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_set_rs_gather: on=%d", on);
  lea::g_rs_gather = on;
  return 0;
}

extern "C" int lea_conv1x1_set_vector(int on) {
  lea::clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv1x1_set_vector: on=%d", on);
  lea::g_1x1_vec = on;
  return 0;
}

extern "C" int lea_conv3d_set_tile_override(int nt, int tw, int td) {
  lea::clear_error();
  if (nt <= 0) {
    lea::g_tile_override[0] = 0;
    return 0;
  }
  LEA_CHECK_ARG((tw == 16 || tw == 32 || tw == 64) && (td == 1 || td == 2) &&
                    (nt == 1 || nt == 2 || nt == 4 || nt == 8),
                "lea_conv3d_set_tile_override: bad tile nt=%d tw=%d td=%d", nt, tw, td);
  lea::g_tile_override[0] = nt;
  lea::g_tile_override[1] = tw;
  lea::g_tile_override[2] = td;
  return 0;
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
  const long long want = (total + threads - 1) / threads;
  const int grid = (int)(want < 4096 ? want : 4096);
  const int mt = mt_for(cout);
  hipStream_t st = as_stream(stream);
  const int cin_b = k == 3 ? PackCfg<3, 1>::CIN_B : PackCfg<1, 1>::CIN_B;
  const int nchunks = (cin + cin_b - 1) / cin_b;
#define LEA_PACK(KS, MT) \
  pack_weights_kernel<KS, MT><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total)
  if (depth_paired(cout, k)) {
    pack_weights_dp_kernel<<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total);
  } else if (k == 3) {
    if (mt == 1) LEA_PACK(3, 1); else if (mt == 2) LEA_PACK(3, 2); else if (mt == 3) LEA_PACK(3, 3); else LEA_PACK(3, 4);
  } else {
    if (mt == 1) LEA_PACK(1, 1); else if (mt == 2) LEA_PACK(1, 2); else if (mt == 3) LEA_PACK(1, 3); else LEA_PACK(1, 4);
  }
#undef LEA_PACK
  return launch_status("lea_conv3d_pack_weights");
}

extern "C" int lea_conv3d_bnrelu(const void* x, int64_t x_bstride, const void* x2,
                                 int64_t x2_bstride, int cin2, const float* w_packed,
                                 const float* scale, const float* shift, const void* residual,
                                 int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                 int cout, int D, int H, int W, int k, unsigned flags, int dtype,
                                 void* stream) {
  lea::ConvArgs a{};
  a.x = (const float*)x;
  a.xbs = x_bstride;
  a.x2 = (const float*)x2;
  a.x2bs = x2_bstride;
  a.cin1 = cin - cin2;
  a.wp = w_packed;
  a.scale = scale;
  a.shift = shift;
  a.res = (const float*)residual;
  a.rbs = r_bstride;
  a.y = (float*)y;
  a.ybs = y_bstride;
  a.cin = cin;
  a.cout = cout;
  a.D = D;
  a.H = H;
  a.W = W;
  a.flags = flags;
  return lea::conv_common(a, B, k, false, dtype, stream);
}

extern "C" size_t lea_conv2d_packed_floats(int cout, int cin) {
  if (cout <= 0 || cin <= 0) return 0;
  return lea::packed_floats_2d(cout, cin);
}

extern "C" int lea_conv2d_pack_weights(const float* w, float* packed, int cout, int cin,
                                       void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(w && packed, "lea_conv2d_pack_weights: null pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0, "lea_conv2d_pack_weights: bad shape cout=%d cin=%d", cout, cin);
  const long long total = (long long)packed_floats_2d(cout, cin);
  const int threads = 256;
  const long long want = (total + threads - 1) / threads;
  const int grid = (int)(want < 4096 ? want : 4096);
  const int nchunks = (cin + PackCfg<3, 1, 1>::CIN_B - 1) / PackCfg<3, 1, 1>::CIN_B;
  hipStream_t st = as_stream(stream);
  switch (mt_for(cout)) {
    case 1: pack_weights_kernel<3, 1, 1><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total); break;
    case 2: pack_weights_kernel<3, 2, 1><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total); break;
    case 3: pack_weights_kernel<3, 3, 1><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total); break;
    default: pack_weights_kernel<3, 4, 1><<<grid, threads, 0, st>>>(w, packed, cout, cin, nchunks, total);
  }
  return launch_status("lea_conv2d_pack_weights");
}

extern "C" const char* lea_conv2d_kernel_name(int B, int cout, int H, int W) {
  if (B <= 0 || cout <= 0 || H <= 0 || W <= 0) return nullptr;
  return lea::plan_name(lea::make_plan_2d(B, cout, H, W), 2);
}

extern "C" int lea_conv2d_bnrelu(const void* x, int64_t x_bstride, const float* w_packed,
                                 const float* scale, const float* shift, const void* residual,
                                 int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                 int cout, int H, int W, unsigned flags, int dtype, void* stream) {
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
  a.cin = cin;
  a.cout = cout;
  a.D = 1;
  a.H = H;
  a.W = W;
  a.flags = flags;
  LEA_CHECK_ARG(a.x && a.wp && a.y, "lea_conv2d: null pointer");
  LEA_CHECK_ARG((a.scale == nullptr) == (a.shift == nullptr),
                "lea_conv2d: scale/shift must both be set or both NULL");
  LEA_CHECK_FLAGS(flags, LEA_RELU | LEA_RESIDUAL, "lea_conv2d");
  LEA_CHECK_ARG(!(flags & LEA_RESIDUAL) || a.res, "lea_conv2d: LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && H > 0 && W > 0,
                "lea_conv2d: bad shape B=%d cin=%d cout=%d H=%d W=%d", B, cin, cout, H, W);
  LEA_CHECK_ARG((long long)(cout + 63) * H * W < (1LL << 31), "lea_conv2d: plane too large");
  LEA_CHECK_ARG(a.x != a.y, "lea_conv2d: input aliases output");
  if (dtype != LEA_F32) {
    set_error("lea_conv2d: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  hipStream_t st = as_stream(stream);
  if (conv2d_small_ok(cin, cout)) return run_conv2d_small(a, B, st);
  const Plan p = make_plan_2d(B, cout, H, W);
  a.ncob = (cout + p.mt * 16 - 1) / (p.mt * 16);
  switch (p.mt) {
    case 1: return run_dma2d_mt1(p, a, B, st);
    case 2: return run_dma2d_mt2(p, a, B, st);
    case 3: return run_dma2d_mt3(p, a, B, st);
    default: return run_dma2d_mt4(p, a, B, st);
  }
}

extern "C" const char* lea_conv3d_costvolume_kernel_name(int B, int cout, int D3, int H, int W) {
  if (B <= 0 || cout <= 0 || D3 <= 0 || H <= 0 || W <= 0) return nullptr;
  const lea::Plan p = lea::make_plan(B, cout, D3, H, W, 3, false);
  if (p.engine != 0) return nullptr;
  snprintf(lea::g_name, sizeof(lea::g_name), "conv3d_dma_kernel<%d, %d, %d, %d, 3, true>", p.mt, p.nt,
           p.tw, p.td);
  return lea::g_name;
}

extern "C" int lea_conv3d_bnrelu_costvolume(const void* left, const void* right, int64_t f_bstride,
                                            const float* w_packed, const float* scale,
                                            const float* shift, void* y, int64_t y_bstride, int B,
                                            int C, int cout, int D3, int H, int W, unsigned flags,
                                            int dtype, void* stream) {
  using namespace lea;
  clear_error();
  ConvArgs a{};
  a.x = (const float*)left;
  a.xbs = f_bstride;
  a.x2 = (const float*)right;
  a.x2bs = f_bstride;
  a.cin1 = C;
  a.wp = w_packed;
  a.scale = scale;
  a.shift = shift;
  a.y = (float*)y;
  a.ybs = y_bstride;
  a.cin = 2 * C;
  a.cout = cout;
  a.D = D3;
  a.H = H;
  a.W = W;
  a.flags = flags & LEA_RELU;
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_conv3d_bnrelu_costvolume");
  LEA_CHECK_ARG(left && right && w_packed && y && y != left && y != right,
                "lea_conv3d_bnrelu_costvolume: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_conv3d_bnrelu_costvolume: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && C > 0 && cout > 0 && D3 > 0 && H > 0 && W > 0,
                "lea_conv3d_bnrelu_costvolume: bad shape B=%d C=%d cout=%d D3=%d H=%d W=%d", B, C,
                cout, D3, H, W);
  constexpr int kCinB = PackCfg<3, 1>::CIN_B;  // chunks must not straddle left/right
  LEA_CHECK_ARG(C % kCinB == 0, "lea_conv3d_bnrelu_costvolume: C=%d must be a multiple of %d", C,
                kCinB);
  LEA_CHECK_ARG((long long)(cout + 63) * D3 * H * W < (1LL << 31),
                "lea_conv3d_bnrelu_costvolume: volume too large");
  if (dtype != LEA_F32) {
    set_error("lea_conv3d_bnrelu_costvolume: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const Plan p = make_plan(B, cout, D3, H, W, 3, false);
  LEA_CHECK_ARG(p.engine == 0, "lea_conv3d_bnrelu_costvolume: no DMA plan for cout=%d", cout);
  a.ncob = (cout + p.mt * 16 - 1) / (p.mt * 16);
  hipStream_t st = as_stream(stream);
  switch (p.mt) {
    case 1: return run_dma_cv_mt1(p, a, B, st);
    case 2: return run_dma_cv_mt2(p, a, B, st);
    case 3: return run_dma_cv_mt3(p, a, B, st);
    default: return run_dma_cv_mt4(p, a, B, st);
  }
}

extern "C" int lea_conv3d_bnrelu_resampled(const void* x, int64_t x_bstride, int Di, int Hi,
                                           int Wi, const float* w_packed, const float* scale,
                                           const float* shift, const void* residual,
                                           int64_t r_bstride, void* y, int64_t y_bstride, int B,
                                           int cin, int cout, int D, int H, int W, int k,
                                           unsigned flags, int dtype, void* stream) {
  lea::ConvArgs a{};
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
  a.cin = cin;
  a.cout = cout;
  a.D = D;
  a.H = H;
  a.W = W;
  a.Di = Di;
  a.Hi = Hi;
  a.Wi = Wi;
  a.rd = lea::axis_ratio(Di, D, 1);
  a.rh = lea::axis_ratio(Hi, H, 1);
  a.rw = lea::axis_ratio(Wi, W, 1);
  a.flags = flags;
  return lea::conv_common(a, B, k, true, dtype, stream);
}
