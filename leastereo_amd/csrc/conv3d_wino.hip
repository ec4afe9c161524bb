// ConvBR3d k=3 (fp32) with Winograd F(2,3) along W on the fp32 matrix cores.
// Replaces models/operations_3d.py:31-47 for the matching net's 3x3x3 layers, as
// the direct engine (conv3d_impl.h) does, with 2/3 of its MFMA work.
//
// For a pair of outputs y[w], y[w+1] along W and a fixed (kd, kh):
//     y[w + j] = sum_kw g[kw] x[w - 1 + j + kw]
//   = A^T [ (G g) . (B^T x) ],  x = x[w-1 .. w+2],
//     G g  = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2)          (packed, or formed in-kernel)
//     B^T x = (x0 - x2, x1 + x2, x2 - x1, x1 - x3)          (4 VALU adds per lane)
//     A^T m = (m0 + m1 + m2, m1 - m2 - m3)
// so per 2 outputs and (kd, kh) the GEMM does 4 products instead of 6.  All of it
// is fp32: the transforms are exact up to one rounding per add (G's halves are
// exact), the products and sums are the MFMA's fp32.  48-cout blocks form U = G g
// in the kernel from staged g rows (a quarter less LDS for the weight stage, which
// keeps two workgroups per CU); 16/32-cout blocks stage the packed U.
//
// GEMM view per transform point xi in 0..3 and (kd, kh):
//     M_xi[co][pair] += sum_ci U_xi[kd][kh][co][ci] * V_xi[ci][pair]
// on v_mfma_f32_16x16x4_f32: A (lane l) = U_xi[co = 16 m + (l & 15)][ci = l >> 4],
// B (lane l) = V_xi[ci = l >> 4][pair = l & 15] (computed by the lane from 4 staged
// inputs, two ds_read_b64), D (lane, reg r) = M_xi[co = 16 m + 4 (l >> 4) + r][pair].
// The epilogue applies A^T and stores the two outputs of its pair as one float2.
//
// Workgroup = 4 waves over a TH x 32 x TD output tile (TH = 4 NP rows, 16 pairs per
// row) and COP = 16 MT output channels.  K is streamed in chunks of 4 input channels
// (one MFMA K step): the input halo by LDS-DMA (buffer_load_dword ... lds, one
// buffer resource per channel, out-of-range offsets return the zero padding), the
// chunk's weights (9 x 4 (or 3) x 4 x COP floats) by global_load_lds_dwordx4;
// two stages, one vmcnt(0) + barrier per chunk (the direct engine's pipeline).
#include "conv3d_impl.h"

namespace lea {
namespace wino {

constexpr int CIN_B = 4;

// 16-row MFMA tiles per cout block: 16, 32 or 48 couts (48 for 48k couts that are not
// multiples of 32: the L1 16->48 sibling groups would pad a 64-row block by a third)
__host__ __device__ constexpr int mt_of(int cout) {
  return cout <= 16 ? 1 : (cout % 32 != 0 && cout % 48 == 0) ? 3 : 2;
}
__host__ __device__ constexpr int round_32mod64(int n) { return n % 64 <= 32 ? n + (32 - n % 64) : n + (96 - n % 64); }

template <int MT, int NP, int TD>
struct Cfg {
  static constexpr int COP = 16 * MT;
  static constexpr bool SWZ = (COP % 32) == 0;  // odd-ci rows: 16-column halves swapped
  static constexpr int TH = 4 * NP;
  static constexpr int RH = TH + 2, RW = 34;
  static constexpr int PLANE = RH * RW;
  static constexpr int PLANES = TD + 2;
  static constexpr int IMG = PLANES * PLANE;
  // channel stride = 32 mod 64 floats: the two channels of a 32-lane ds_read_b64
  // group read disjoint halves of the 64 banks
  static constexpr int CIS = round_32mod64(IMG);
  static constexpr int XS = CIN_B * CIS;
  // 48-row blocks stage the plain weights g (3 rows per (kd,kh)) and form U = G g in
  // the kernel, so two stages of two workgroups fit the LDS; 16/32-row blocks stage
  // U (4 rows), which saves the per-step VALU (measured 1-2.5 % faster)
  static constexpr bool GW = MT == 3;
  static constexpr int KW_ROWS = GW ? 3 : 4;
  static constexpr int WS = 9 * KW_ROWS * CIN_B * COP;
  static constexpr int STAGE = XS + WS;
  static_assert(XS % 16 == 0 && WS % 16 == 0, "16-byte aligned LDS regions");
};

__device__ __forceinline__ int a_col(int m, int ci, int n, bool swz) { return ((swz ? (m ^ (ci & 1)) : m) * 16) + n; }

template <int MT, int NP, int TD, bool CV>
__global__ __launch_bounds__(kConvThreads, 2) void conv3d_wino_kernel(const ConvArgs a) {
  using C = Cfg<MT, NP, TD>;
  constexpr int XSLOTS = (C::IMG + 63) / 64;
  constexpr int XSLOTS_W = (XSLOTS + kConvWaves - 1) / kConvWaves;
  constexpr int WSLOTS = (C::WS + 255) / 256;
  constexpr int WSLOTS_W = (WSLOTS + kConvWaves - 1) / kConvWaves;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware 1-D order (as conv3d_dma_kernel): each XCD walks a contiguous range
  // of (batch/cout-block, tile, depth group), depth group fastest
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int dz = lin % a.ndz;
  const int tile = (lin / a.ndz) % a.ntiles;
  const int bc = lin / (a.ndz * a.ntiles);
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * 32;
  const int d0 = dz * TD;
  const int b = bc / a.ncob;
  const int cob = bc - b * a.ncob;
  const int co0 = cob * C::COP;
  const int nchunks = a.cin / CIN_B;
  const float* wp = a.wp + (long long)cob * nchunks * C::WS;
  const int HW = a.H * a.W;  // host checks D*H*W*4 < 2^32
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;

  // per-lane byte offsets of this wave's DMA pieces inside one channel volume
  unsigned voff[XSLOTS_W], voffr[CV ? XSLOTS_W : 1];
#pragma unroll
  for (int t = 0; t < XSLOTS_W; ++t) {
    const int e = (wave + kConvWaves * t) * 64 + lane;
    unsigned v = 0xFFFFFFF0u, vr = 0xFFFFFFF0u;
    if (e < C::IMG) {
      const int p = e / C::PLANE;
      const int r = e - p * C::PLANE;
      const int rr = r / C::RW;
      const int cc = r - rr * C::RW;
      const int d = d0 + p - 1, h = h0 + rr - 1, w = w0 + cc - 1;
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
    const long long cvol = CV ? (long long)HW : (long long)HW * a.D;  // channel stride
    const unsigned crec = CV ? (unsigned)HW * 4u : nrec;
#pragma unroll
    for (int ci = 0; ci < CIN_B; ++ci) {
      const int c = ch * CIN_B + ci;
      const float* base = a.x;
      unsigned n = 0;
      if (c < a.cin1) {
        base = a.x + (long long)b * a.xbs + (long long)c * cvol;
        n = crec;
      } else if (c < a.cin) {
        base = a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * cvol;
        n = crec;
      }
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
      const unsigned rmask = (CV && c >= a.cin1) ? 0xFFFFFFFFu : 0u;  // chunks never straddle cin1
#pragma unroll
      for (int t = 0; t < XSLOTS_W; ++t) {
        const int j = wave + kConvWaves * t;
        unsigned vo = voff[t];
        if constexpr (CV) vo = voff[t] ^ ((voff[t] ^ voffr[t]) & rmask);
        if (j < XSLOTS && j * 64 + lane < C::IMG)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(st + ci * C::CIS + j * 64), 4, vo, 0, 0, 0);
      }
    }
  };

  const int ci = lane >> 4, p = lane & 15;
  int xoff[NP];  // staged input column 2p (w0 + 2p - 1) of row (wave NP + j), channel ci
#pragma unroll
  for (int j = 0; j < NP; ++j) xoff[j] = ci * C::CIS + (wave * NP + j) * C::RW + 2 * p;
  int woff[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) woff[m] = ci * C::COP + a_col(m, ci, p, C::SWZ);

  // folded BN of this lane's couts, fetched now so the epilogue does not wait
  float sc[MT][4], sh[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * m + 4 * ci + r;
      const bool cv = co < a.cout;
      sc[m][r] = (cv && a.scale) ? a.scale[co] : 1.f;
      sh[m][r] = (cv && a.shift) ? a.shift[co] : 0.f;
    }

  f32x4 acc[4][TD][MT][NP];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int t = 0; t < TD; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[x][t][m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, smem);
  for (int ch = 0; ch < nchunks; ++ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of chunk ch landed
    __syncthreads();  // ... and everyone's; chunk ch-1's stage is free
    if (ch + 1 < nchunks) issue(ch + 1, smem + ((ch + 1) & 1) * C::STAGE);
    const float* xs = smem + (ch & 1) * C::STAGE;
    const float* ws = xs + C::XS;
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        float vb[TD][NP][4];
#pragma unroll
        for (int t = 0; t < TD; ++t)
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const float* s = xs + xoff[j] + (t + kd) * C::PLANE + kh * C::RW;
            const float2 lo = *reinterpret_cast<const float2*>(s);
            const float2 hi = *reinterpret_cast<const float2*>(s + 2);
            vb[t][j][0] = lo.x - hi.x;
            vb[t][j][1] = lo.y + hi.x;
            vb[t][j][2] = hi.x - lo.y;
            vb[t][j][3] = lo.y - hi.y;
          }
        const float* wk = ws + (kd * 3 + kh) * C::KW_ROWS * CIN_B * C::COP;
        float u[4][MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if constexpr (C::GW) {  // U = G g of this lane's kw row (exact halves)
            const float g0 = wk[woff[m]], g1 = wk[CIN_B * C::COP + woff[m]];
            const float g2 = wk[2 * CIN_B * C::COP + woff[m]];
            const float t = g0 + g2;
            u[0][m] = g0;
            u[1][m] = (t + g1) * 0.5f;
            u[2][m] = (t - g1) * 0.5f;
            u[3][m] = g2;
          } else {
#pragma unroll
            for (int x = 0; x < 4; ++x) u[x][m] = wk[x * CIN_B * C::COP + woff[m]];
          }
        }
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const float (&av)[MT] = u[x];
#pragma unroll
          for (int t = 0; t < TD; ++t)
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
              for (int j = 0; j < NP; ++j)
                acc[x][t][m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], vb[t][j][x], acc[x][t][m][j], 0, 0, 0);
        }
      }
    }
  }

  // epilogue: A^T, folded BN, ReLU, residual; lane stores outputs (w0+2p, w0+2p+1)
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int w = w0 + 2 * p;
#pragma unroll
  for (int t = 0; t < TD; ++t) {
    const int d = d0 + t;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int h = h0 + wave * NP + j;
      if (d >= a.D || h >= a.H || w >= a.W) continue;
      const bool two = w + 1 < a.W;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + 16 * m + 4 * ci + r;
          if (co >= a.cout) continue;
          const float m0 = acc[0][t][m][j][r], m1 = acc[1][t][m][j][r];
          const float m2 = acc[2][t][m][j][r], m3 = acc[3][t][m][j][r];
          float y0 = (m0 + m1) + m2;
          float y1 = (m1 - m2) - m3;
          y0 = y0 * sc[m][r] + sh[m][r];
          y1 = y1 * sc[m][r] + sh[m][r];
          if (relu) {
            y0 = fmaxf(y0, 0.f);
            y1 = fmaxf(y1, 0.f);
          }
          const long long o = (long long)co * DHW + (long long)d * HW + (long long)h * a.W + w;
          float* yp = a.y + (long long)b * a.ybs + o;
          const float* rp = a.res + (long long)b * a.rbs + o;
          const bool vec = two && ((reinterpret_cast<uintptr_t>(yp) | (resid ? reinterpret_cast<uintptr_t>(rp) : 0)) & 7) == 0;
          if (vec) {
            if (resid) {
              const float2 rv = *reinterpret_cast<const float2*>(rp);
              y0 += rv.x;
              y1 += rv.y;
            }
            *reinterpret_cast<float2*>(yp) = make_float2(y0, y1);
          } else {
            if (resid) y0 += rp[0];
            yp[0] = y0;
            if (two) {
              if (resid) y1 += rp[1];
              yp[1] = y1;
            }
          }
        }
    }
  }
}

// weights [cout][cin][3][3][3] -> per (cout block, chunk): [kd*3+kh][row][ci][COP col],
// rows = U_xi = (G g)_xi (computed in double, rounded once) for 16/32-row blocks,
// rows = g[kw] for 48-row blocks (the kernel forms U)
template <int MT>
__global__ void pack_wino_kernel(const float* __restrict__ w, float* __restrict__ packed, int cout,
                                 int cin, int nchunks, long long total) {
  constexpr int COP = 16 * MT;
  constexpr bool SWZ = (COP % 32) == 0;
  constexpr bool GW = MT == 3;
  constexpr int ROWS = GW ? 3 : 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int col = (int)(q % COP); q /= COP;
    const int ci = (int)(q % CIN_B); q /= CIN_B;
    const int row = (int)(q % ROWS); q /= ROWS;
    const int kdkh = (int)(q % 9); q /= 9;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int mm = col / 16, n = col % 16;
    const int m = SWZ ? (mm ^ (ci & 1)) : mm;
    const int co = cb * COP + 16 * m + n;
    const int c = ch * CIN_B + ci;
    float v = 0.f;
    if (co < cout && c < cin) {
      const float* g = w + (((long long)co * cin + c) * 9 + kdkh) * 3;  // [kd][kh][kw]
      if (GW) {
        v = g[row];
      } else {
        const double g0 = g[0], g1 = g[1], g2 = g[2];
        v = row == 0 ? (float)g0 : row == 3 ? (float)g2 : row == 1 ? (float)((g0 + g1 + g2) * 0.5)
                                                                   : (float)((g0 - g1 + g2) * 0.5);
      }
    }
    packed[i] = v;
  }
}

struct Plan {
  int mt, np, td;
};

thread_local int g_override[2] = {0, 0};  // np, td (lea_conv3d_wino_set_tile_override)

inline Plan make_plan(int B, int cout, int D, int H, int W) {
  // r01 sweep (tools/wino_sweep.py, profiles/r01_wino_sweep.txt): 8-row x 2-plane
  // tiles for the 32-channel blocks (stem0/stem1/conv1/conv2: 0.72-0.81x the
  // direct engine's time), 4 x 2 for the 16-channel cells; single planes only when
  // the volume is too shallow to fill the chip.
  Plan p;
  p.mt = mt_of(cout);
  const long long ncob = (cout + 16 * p.mt - 1) / (16 * p.mt);
  auto wgs = [&](int np, int td) {
    return (long long)((W + 31) / 32) * ((H + 4 * np - 1) / (4 * np)) * ((D + td - 1) / td) * B * ncob;
  };
  p.np = (p.mt == 2 && wgs(2, 2) >= 512) ? 2 : 1;  // MT=3: two stages of 8 rows exceed the LDS
  p.td = wgs(p.np, 2) >= 384 ? 2 : 1;
  if (g_override[0] > 0) {
    p.np = g_override[0];
    p.td = g_override[1];
  }
  return p;
}

#define LEA_WINO_CASE(MT, NP, TD, CV)                                                   \
  if (p.mt == MT && p.np == NP && p.td == TD) {                                         \
    a.tiles_w = (a.W + 31) / 32;                                                        \
    a.ntiles = a.tiles_w * ((a.H + 4 * NP - 1) / (4 * NP));                             \
    a.ndz = (a.D + TD - 1) / TD;                                                        \
    const long long n_ = (long long)a.ntiles * a.ndz * B * a.ncob;                      \
    LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino): grid too large");                \
    a.nblk = (int)n_;                                                                   \
    conv3d_wino_kernel<MT, NP, TD, CV><<<dim3((unsigned)n_), kConvThreads, 0, st>>>(a); \
    return launch_status("lea_conv3d(wino)");                                          \
  }
#define LEA_WINO_TILES(CV)                                                                      \
  LEA_WINO_CASE(1, 1, 1, CV) LEA_WINO_CASE(1, 1, 2, CV) LEA_WINO_CASE(1, 2, 1, CV)              \
  LEA_WINO_CASE(1, 2, 2, CV) LEA_WINO_CASE(2, 1, 1, CV) LEA_WINO_CASE(2, 1, 2, CV)              \
  LEA_WINO_CASE(2, 2, 1, CV) LEA_WINO_CASE(2, 2, 2, CV) LEA_WINO_CASE(3, 1, 1, CV)              \
  LEA_WINO_CASE(3, 1, 2, CV)

int run(const Plan& p, ConvArgs a, int B, hipStream_t st, bool cv) {
  a.ncob = (a.cout + 16 * p.mt - 1) / (16 * p.mt);
  if (cv) {
    LEA_WINO_TILES(true)
  } else {
    LEA_WINO_TILES(false)
  }
  set_error("lea_conv3d(wino): no tile mt=%d np=%d td=%d", p.mt, p.np, p.td);
  return LEA_E_UNSUPPORTED;
}

thread_local char g_name[96];

const char* name(const Plan& p, bool cv) {
  snprintf(g_name, sizeof(g_name), "conv3d_wino_kernel<%d, %d, %d, %s>", p.mt, p.np, p.td,
           cv ? "true" : "false");
  return g_name;
}

int common(ConvArgs& a, int B, bool cv, int dtype, void* stream) {
  LEA_CHECK_ARG(a.x && a.wp && a.y, "lea_conv3d(wino): null pointer");
  LEA_CHECK_ARG((a.scale == nullptr) == (a.shift == nullptr),
                "lea_conv3d(wino): scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(!(a.flags & LEA_RESIDUAL) || a.res, "lea_conv3d(wino): LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && a.cin > 0 && a.cout > 0 && a.D > 0 && a.H > 0 && a.W > 0,
                "lea_conv3d(wino): bad shape B=%d cin=%d cout=%d D=%d H=%d W=%d", B, a.cin, a.cout,
                a.D, a.H, a.W);
  LEA_CHECK_ARG(a.cin % CIN_B == 0 && a.cin1 % CIN_B == 0,
                "lea_conv3d(wino): input channels (%d, first source %d) must be multiples of %d",
                a.cin, a.cin1, CIN_B);
  LEA_CHECK_ARG((long long)a.D * a.H * a.W * 4 < (1LL << 32) &&
                    (long long)(a.cout + 31) * a.D * a.H * a.W < (1LL << 31),
                "lea_conv3d(wino): volume too large");
  LEA_CHECK_ARG(a.x != a.y && a.x2 != a.y, "lea_conv3d(wino): input aliases output");
  if (dtype != LEA_F32) {
    set_error("lea_conv3d(wino): dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const Plan p = make_plan(B, a.cout, a.D, a.H, a.W);
  return run(p, a, B, as_stream(stream), cv);
}

}  // namespace wino
}  // namespace lea

using namespace lea;

extern "C" size_t lea_conv3d_wino_packed_floats(int cout, int cin) {
  if (cout <= 0 || cin <= 0 || cin % wino::CIN_B != 0) return 0;
  const int cop = 16 * wino::mt_of(cout);
  const int rows = wino::mt_of(cout) == 3 ? 3 : 4;
  return (size_t)((cout + cop - 1) / cop) * (cin / wino::CIN_B) * 9 * rows * wino::CIN_B * cop;
}

extern "C" int lea_conv3d_wino_pack_weights(const float* w, float* packed, int cout, int cin,
                                            void* stream) {
  clear_error();
  LEA_CHECK_ARG(w && packed, "lea_conv3d_wino_pack_weights: null pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0 && cin % wino::CIN_B == 0,
                "lea_conv3d_wino_pack_weights: unsupported shape cout=%d cin=%d", cout, cin);
  const long long total = (long long)lea_conv3d_wino_packed_floats(cout, cin);
  const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
  hipStream_t st = as_stream(stream);
  switch (wino::mt_of(cout)) {
    case 1: wino::pack_wino_kernel<1><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, total); break;
    case 3: wino::pack_wino_kernel<3><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, total); break;
    default: wino::pack_wino_kernel<2><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, total);
  }
  return launch_status("lea_conv3d_wino_pack_weights");
}

extern "C" const char* lea_conv3d_wino_kernel_name(int B, int cout, int D, int H, int W, int costvolume) {
  if (B <= 0 || cout <= 0 || D <= 0 || H <= 0 || W <= 0) return nullptr;
  return wino::name(wino::make_plan(B, cout, D, H, W), costvolume != 0);
}

extern "C" int lea_conv3d_wino_set_tile_override(int np, int td) {
  clear_error();
  if (np <= 0) {
    wino::g_override[0] = 0;
    return 0;
  }
  LEA_CHECK_ARG((np == 1 || np == 2) && (td == 1 || td == 2),
                "lea_conv3d_wino_set_tile_override: bad tile np=%d td=%d", np, td);
  wino::g_override[0] = np;
  wino::g_override[1] = td;
  return 0;
}

extern "C" int lea_conv3d_bnrelu_wino(const void* x, int64_t x_bstride, const void* x2,
                                      int64_t x2_bstride, int cin2, const float* w_packed,
                                      const float* scale, const float* shift, const void* residual,
                                      int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                      int cout, int D, int H, int W, unsigned flags, int dtype,
                                      void* stream) {
  clear_error();
  ConvArgs a{};
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
  LEA_CHECK_ARG(cin2 >= 0 && cin2 <= cin && (cin2 == 0 || x2), "lea_conv3d_bnrelu_wino: bad second source");
  return wino::common(a, B, false, dtype, stream);
}

extern "C" int lea_conv3d_bnrelu_costvolume_wino(const void* left, const void* right,
                                                 int64_t f_bstride, const float* w_packed,
                                                 const float* scale, const float* shift, void* y,
                                                 int64_t y_bstride, int B, int C, int cout, int D3,
                                                 int H, int W, unsigned flags, int dtype,
                                                 void* stream) {
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
  LEA_CHECK_ARG(left && right && y != left && y != right,
                "lea_conv3d_bnrelu_costvolume_wino: null or aliased pointer");
  return wino::common(a, B, true, dtype, stream);
}
