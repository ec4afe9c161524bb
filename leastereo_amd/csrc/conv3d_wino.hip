// ConvBR3d k=3 (fp32) with Winograd F(2,3) / F(4,3) along W on the fp32 matrix
// cores.  Replaces models/operations_3d.py:31-47 for the matching net's 3x3x3
// layers, as the direct engine (conv3d_impl.h) does, with 2/3 (F(2,3)) or 1/2
// (F(4,3)) of its MFMA work.
//
// For F consecutive outputs y[w .. w+F-1] along W and a fixed (kd, kh):
//     y[w + j] = sum_kw g[kw] x[w - 1 + j + kw]  =  A^T [ (G g) . (B^T x) ],
// x = x[w-1 .. w+F], F + 2 transform points xi.
//   F(2,3): G g  = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2)
//           B^T x = (x0 - x2, x1 + x2, x2 - x1, x1 - x3)
//           A^T m = (m0 + m1 + m2, m1 - m2 - m3)
//   F(4,3) (points 0, +-1, +-2, inf):
//           G g  = (g0/4, -(g0+g1+g2)/6, -(g0-g1+g2)/6, (g0+2g1+4g2)/24, (g0-2g1+4g2)/24, g2)
//           B^T x = (4x0-5x2+x4, -4x1-4x2+x3+x4, 4x1-4x2-x3+x4, -2x1-x2+2x3+x4,
//                    2x1-x2-2x3+x4, 4x1-5x3+x5)
//           A^T m = (m0+m1+m2+m3+m4, m1-m2+2(m3-m4), m1+m2+4(m3+m4), m1-m2+8(m3-m4)+m5)
// so per F outputs and (kd, kh) the GEMM does F+2 products instead of 3F.  All of it
// is fp32: the products and sums are the MFMA's fp32; the transforms add a few
// roundings per value (F(4,3)'s coefficients are larger, its error a few times
// F(2,3)'s -- both far inside the conv tolerance, tests/test_gpu_wino.py).
// U = G' g is formed in the kernel from the staged weights g (3 LDS reads and 4-6
// VALU per row and step; G' = G with each row's constant factor -- 1/4, -1/6, 1/24,
// 1/2 -- moved onto the accumulator M_xi in the epilogue): the weight stage is 3
// rows per (kd, kh) whatever F, which is what keeps two workgroups per CU with
// F(4,3)'s wider halo.
//
// GEMM view per transform point xi and (kd, kh):
//     M_xi[co][group] += sum_ci U_xi[kd][kh][co][ci] * V_xi[ci][group]
// on v_mfma_f32_16x16x4_f32: A (lane l) = U_xi[co = 16 m + (l & 15)][ci = l >> 4],
// B (lane l) = V_xi[ci = l >> 4][group = l & 15] (computed by the lane from F + 2
// staged inputs, F/2 + 1 ds_read_b64), D (lane, reg r) = M_xi[co = 16 m + 4 (l >> 4)
// + r][group].  The epilogue applies A^T and stores the F outputs of its group as
// one float2 / float4.
//
// Workgroup = 4 waves over a TH x F Q x TD output tile (a lane group of 16 covers
// 16/Q rows of Q groups of F outputs; TH = 4 NP 16/Q rows) and COP = 16 MT output
// channels.  K is streamed in chunks of 4
// input channels (one MFMA K step): the input halo by LDS-DMA (buffer_load_dword ...
// lds, one buffer resource per channel, out-of-range offsets return the zero
// padding), the chunk's weights (9 x 3 x 4 x COP floats) by global_load_lds_dwordx4;
// two stages, one vmcnt(0) + barrier per chunk (the direct engine's pipeline).
// Within a chunk the 9 (kd, kh) steps are software-pipelined: LDS reads two steps
// ahead, the V / U transforms one step ahead, so a step's VALU issues under the
// previous step's MFMAs.
#include "wino_common.h"

namespace lea {
namespace wino {

template <int F, int Q, int MT, int NP, int TD, bool H16 = false>
struct Cfg {
  static constexpr bool DP = MT == 0;           // depth-paired (couts <= 8)
  static constexpr int MTE = DP ? 1 : MT;       // 16-row tiles per wave
  static constexpr int TDA = DP ? 1 : TD;       // accumulator sets along D
  static constexpr int NSTEP = DP ? 12 : 9;     // (kd, kh) steps; depth-paired: (staged plane, kh)
  static_assert(!DP || TD == 2, "a depth-paired tile covers two output planes");
  static constexpr int NX = F + 2;              // transform points
  static constexpr int COP = 16 * MTE;
  static constexpr bool SWZ = (COP % 32) == 0;  // odd-ci rows: 16-column halves swapped
  static constexpr int RPG = 16 / Q;            // tile rows per lane group
  static constexpr int TW = F * Q;              // outputs per tile row
  static constexpr int TH = 4 * NP * RPG;
  static constexpr int RH = TH + 2, RW = TW + 2;
  static constexpr int PLANE = RH * RW;
  static constexpr int PLANES = TD + 2;
  static constexpr int IMG = PLANES * PLANE;
  static constexpr int XSLOTS = (IMG + 63) / 64;  // 64-lane DMA pieces per channel
  // channel stride >= whole pieces: the last piece's surplus lanes land in padding,
  // so no piece needs a per-lane exec mask
  static constexpr int CIS = conflict_free_cis<F, Q>(64 * XSLOTS, RW);
  // H16: rows staged as 16-byte blocks from w0 - 4 (RWA = TW + 8 floats), one channel's
  // planes x rows contiguous (PIECES16 pieces of 64 lanes, the last one partial), channel
  // c at CB2(c) == {1, 3, 33, 35}[c] mod 64 dwords: column w0 - 1 at an even dword (the
  // step's ds_read_b64s stay 8-byte aligned) and, for one tile row per lane group
  // (Q = 16), the 32 lanes of a read (16 groups x 2 channels) on 64 distinct banks
  static constexpr int RWA = TW + 8;
  static constexpr int PLANEA = RH * RWA;
  static constexpr int IMGA = PLANES * PLANEA;
  static constexpr int BLK16 = IMGA / 4;
  static constexpr int PIECES16 = (BLK16 + 63) / 64;
  static constexpr int cb2(int c) {
    int base = 1;
    for (int k = 1; k <= c; ++k) {
      const int want = (k & 1 ? 2 : 0) + (k & 2 ? 32 : 0) + 1, lo = base + IMGA;
      base = lo + ((want - lo) % 64 + 64) % 64;
    }
    return base;
  }
  static_assert(!H16 || (Q == 16 && F == 4), "16-byte halo: one tile row per lane group");
  // r04: channel regions of whole pieces (CSH = PIECES16 x 256 floats, 0 mod 64), every base
  // 1 mod 64: column w0 - 1 sits 16-byte aligned, so a lane reads its 6 inputs per (plane,
  // row) as two ds_read_b128, and each b128 lane group ({0-3,12-15,20-27}, ...: two channels'
  // complementary 4-group runs of one row) reads 64 distinct banks.  The float2 reads the
  // compiler paired into ds_read2_b64 (banked mod 32 over 16-lane groups) were 2-way
  // conflicted on the 64-wide row (pq, pq + 8): 5.9 M of 17.7 M LDS cycles per L0 launch
  static constexpr int CSH = PIECES16 * 256;
  static constexpr int cbh(int c) { return 1 + c * CSH; }
  static_assert(!H16 || (CSH % 64 == 0 && RWA % 4 == 0 && PLANEA % 4 == 0), "b128 halo map");
  static constexpr int XS = H16 ? (cbh(CIN_B) + 3) / 4 * 4 : CIN_B * CIS;
  static constexpr int RWX = H16 ? RWA : RW;       // staged row / plane strides the steps read
  static constexpr int PLX = H16 ? PLANEA : PLANE;
  static constexpr int WS = NSTEP * 3 * CIN_B * COP;  // the chunk's weights g[step][kw][ci][co]
  static constexpr int WSLOTS = (WS + 255) / 256;  // 256-float pieces (padded the same way)
  static constexpr int STAGE = XS + 256 * WSLOTS;
  static_assert(XS % 4 == 0 && WS % 4 == 0 && RW % 2 == 0 && PLANE % 2 == 0, "aligned LDS regions and b64 reads");
  static_assert(2 * STAGE * 4 * 2 <= 160 * 1024, "two double-buffered workgroups per CU");
};

template <int F, int Q, int MT, int NP, int TD, bool CV, bool H16 = false, bool FENCE = false>
__global__ __launch_bounds__(kConvThreads, 2) void conv3d_wino_kernel(const ConvArgs a) {
  using C = Cfg<F, Q, MT, NP, TD, H16>;
  static_assert(!(CV && H16), "16-byte halo: plain volumes only");
  constexpr int NX = C::NX;
  constexpr int XSLOTS = C::XSLOTS;
  constexpr int XSLOTS_W = (XSLOTS + kConvWaves - 1) / kConvWaves;
  constexpr int WSLOTS = C::WSLOTS;
  constexpr int WSLOTS_W = (WSLOTS + kConvWaves - 1) / kConvWaves;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE];
  const unsigned lds0 = lds_addr(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware 1-D order (as conv3d_dma_kernel): each XCD walks a contiguous range
  // of (batch/cout-block, tile, depth group), depth group fastest
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  // a workgroup walks spw consecutive depth groups of TD planes (items = groups x
  // chunks through one DMA pipeline), as the W x D engine (conv3d_wino2.hip)
  const int spw = a.spw > 0 ? a.spw : 1;
  const int ngz = (a.ndz + spw - 1) / spw;
  // cout block fastest: the blocks of one (tile, depth group) share its input in the L2
  const int cob = lin % a.ncob;
  const int rest = lin / a.ncob;
  const int gz = rest % ngz;
  const int tile = (rest / ngz) % a.ntiles;
  const int b = rest / (ngz * a.ntiles);
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * C::TW;
  const int dz0 = gz * spw, ngroups = min(spw, a.ndz - dz0);
  const int co0 = cob * C::COP;
  const int nchunks = a.cin / CIN_B;
  const int nitems = ngroups * nchunks;
  const float* wp = a.wp + (long long)cob * nchunks * C::WS;
  const int HW = a.H * a.W;  // host checks D*H*W*4 < 2^32
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;

  // per-lane DMA pieces of this wave inside one channel volume: the (h, w) byte offset
  // once (or OOB), the plane per depth group
  unsigned hwo[XSLOTS_W];
  int pln[XSLOTS_W], wco[CV ? XSLOTS_W : 1];
#pragma unroll
  for (int t = 0; t < XSLOTS_W; ++t) {
    const int e = (wave + kConvWaves * t) * 64 + lane;
    unsigned v = 0xFFFFFFF0u;
    int pl = -1000, wc_ = 0;
    if (e < C::IMG) {
      const int p = e / C::PLANE;
      const int r = e - p * C::PLANE;
      const int rr = r / C::RW;
      const int cc = r - rr * C::RW;
      const int h = h0 + rr - 1, w = w0 + cc - 1;
      if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
        v = (unsigned)(h * a.W + w) * 4u;
        pl = p - 1;
        wc_ = w;
      }
    }
    hwo[t] = v;
    pln[t] = pl;
    if constexpr (CV) wco[t] = wc_;
  }
  unsigned voff[XSLOTS_W], voffr[CV ? XSLOTS_W : 1];
  // H16: piece t of this wave is k = wave + 4 t of the chunk's CIN_B x PIECES16 (channel
  // k / PIECES16, block slot k % PIECES16)
  constexpr int P16 = C::PIECES16, T16 = H16 ? (CIN_B * P16 + kConvWaves - 1) / kConvWaves : 1;
  unsigned hwo16[T16], voff16[T16];
  int pln16[T16];
  bool ok16[T16];
  if constexpr (H16) {
#pragma unroll
    for (int t = 0; t < T16; ++t) {
      const int k = wave + kConvWaves * t, e = 64 * (k % P16) + lane;
      ok16[t] = k < CIN_B * P16 && e < C::BLK16;
      const int p = e / (C::RH * (C::RWA / 4)), r = e - p * (C::RH * (C::RWA / 4));
      const int rr = r / (C::RWA / 4), blk = r - rr * (C::RWA / 4);
      const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;  // W % 4 == 0: a block is all in or all out
      const bool in = ok16[t] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      hwo16[t] = in ? (unsigned)(h * a.W + w) * 4u : 0xFFFFFFF0u;
      pln16[t] = in ? p - 1 : -1000;
    }
  }
  auto set_group = [&](int d0) {  // DMA offsets of the depth group at output planes d0 ..
    if constexpr (H16) {
#pragma unroll
      for (int t = 0; t < T16; ++t) {
        const int d = d0 + pln16[t];
        voff16[t] = (hwo16[t] != 0xFFFFFFF0u && (unsigned)d < (unsigned)a.D)
                        ? hwo16[t] + (unsigned)d * (unsigned)HW * 4u : 0xFFFFFFF0u;
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < XSLOTS_W; ++t) {
      const int d = d0 + pln[t];
      const bool ok = hwo[t] != 0xFFFFFFF0u && (unsigned)d < (unsigned)a.D;
      if constexpr (CV) {  // planes are the feature maps: left (w >= d) / right shifted by d
        const bool okc = ok && wco[t] >= d;
        voff[t] = okc ? hwo[t] : 0xFFFFFFF0u;
        voffr[t] = okc ? hwo[t] - (unsigned)d * 4u : 0xFFFFFFF0u;
      } else {
        voff[t] = ok ? hwo[t] + (unsigned)d * (unsigned)HW * 4u : 0xFFFFFFF0u;
      }
    }
  };

  auto issue = [&](int item, float* st) {
    const int ch = item % nchunks;
    if (ch == 0) set_group((dz0 + item / nchunks) * TD);
    const float* wsrc = wp + (long long)ch * C::WS;
    float* wdst = st + C::XS;
#pragma unroll
    for (int t = 0; t < WSLOTS_W; ++t) {
      const int j = wave + kConvWaves * t;
      if (j < WSLOTS)  // the last piece reads into the next chunk / the buffer's tail pad
        dma_dwordx4(wsrc + j * 256 + lane * 4, lds0 + 4 * (unsigned)(wdst - smem + j * 256));
    }
    const long long cvol = CV ? (long long)HW : (long long)HW * a.D;  // channel stride
    const unsigned crec = CV ? (unsigned)HW * 4u : nrec;
    if constexpr (H16) {
#pragma unroll
      for (int t = 0; t < T16; ++t) {
        const int k = wave + kConvWaves * t, ci = k / P16;
        const int c = ch * CIN_B + ci;
        const float* base = c < a.cin1 ? a.x + (long long)b * a.xbs + (long long)c * cvol
                                       : a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * cvol;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, crec, 0x00020000);
        const int cb = C::cbh(0) + ci * C::CSH;
        if (ok16[t]) dma_dwordx4_buf(rs, voff16[t], lds0 + 4 * (unsigned)(st - smem + cb + (k % P16) * 256));
      }
      return;
    }
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
        if (j < XSLOTS) dma_dword(rs, vo, lds0 + 4 * (unsigned)(st - smem + ci * C::CIS + j * 64));
      }
    }
  };

  const int ci = lane >> 4, p = lane & 15;
  const int pq = p % Q, pr = p / Q;  // output group within the row, row within the lane group
  int xoff[NP];  // staged input column F pq (w0 + F pq - 1) of tile row (wave NP + j) RPG + pr
#pragma unroll
  for (int j = 0; j < NP; ++j)
    xoff[j] = H16 ? C::cbh(ci) + ((wave * NP + j) * C::RPG + pr) * C::RWA + 3 + F * pq
                  : ci * C::CIS + ((wave * NP + j) * C::RPG + pr) * C::RW + F * pq;
  int woff[C::MTE];
#pragma unroll
  for (int m = 0; m < C::MTE; ++m) woff[m] = ci * C::COP + a_col(m, ci, p, C::SWZ);

  // folded BN of this lane's couts, fetched now so the epilogue does not wait
  // (depth-paired: accumulator row 4 ci + r = cout (row & 7) of plane d0 + (row >> 3))
  float sc[C::MTE][4], sh[C::MTE][4];
#pragma unroll
  for (int m = 0; m < C::MTE; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = C::DP ? 4 * (ci & 1) + r : co0 + 16 * m + 4 * ci + r;
      const bool cv = co < a.cout;
      sc[m][r] = (cv && a.scale) ? a.scale[co] : 1.f;
      sh[m][r] = (cv && a.shift) ? a.shift[co] : 0.f;
    }

  f32x4 acc[NX][C::TDA][C::MTE][NP];
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int t = 0; t < C::TDA; ++t)
#pragma unroll
      for (int m = 0; m < C::MTE; ++m)
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[x][t][m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue of one depth group (output planes d0 ..): A^T, folded BN, ReLU, residual;
  // lane stores outputs w0 + F p .. + F - 1
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int w = w0 + F * pq;
  // the buffer-addressed form (wino_common.h, F = 4): residual loads all issued first,
  // every lane the same NST float4 stores (invalid ones out of range: dropped)
  const bool ebuf = F == 4 && (a.flags & kEpiBuf);
  constexpr int NST = C::TDA * NP * C::MTE * 4;
  const int nco = C::DP ? a.cout : min(C::COP, a.cout - co0);
  const __amdgpu_buffer_rsrc_t yrs = block_rsrc(a.y + (long long)b * a.ybs + (long long)co0 * DHW, nco * DHW * 4);
  const __amdgpu_buffer_rsrc_t rrs =
      block_rsrc((resid ? a.res : a.y) + (long long)b * (resid ? a.rbs : a.ybs) + (long long)co0 * DHW, nco * DHW * 4);
  auto epilogue_buf = [&](int d0) {
    unsigned off[C::TDA][NP][C::MTE][4];
#pragma unroll
    for (int t = 0; t < C::TDA; ++t)
#pragma unroll
      for (int j = 0; j < NP; ++j)
#pragma unroll
        for (int m = 0; m < C::MTE; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int d = C::DP ? d0 + (ci >> 1) : d0 + t;
            const int h = h0 + (wave * NP + j) * C::RPG + pr;
            const int cr = C::DP ? 4 * (ci & 1) + r : 16 * m + 4 * ci + r;
            off[t][j][m][r] = (d < a.D && h < a.H && w < a.W && cr < nco)
                                  ? (unsigned)(cr * DHW + (long long)d * HW + h * a.W + w) * 4u
                                  : kEpiOob;
          }
    f32x4 rv[C::TDA][NP][C::MTE][4];
    if (resid) {
#pragma unroll
      for (int t = 0; t < C::TDA; ++t)
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
          for (int m = 0; m < C::MTE; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) rv[t][j][m][r] = buf_load4(rrs, off[t][j][m][r]);
    }
#pragma unroll
    for (int t = 0; t < C::TDA; ++t)
#pragma unroll
      for (int j = 0; j < NP; ++j)
#pragma unroll
        for (int m = 0; m < C::MTE; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            constexpr int X3 = NX > 4 ? 3 : 0, X4 = NX > 4 ? 4 : 0;  // F = 2 never takes this path
            const float m0 = 0.25f * acc[0][t][m][j][r];
            const float m1 = (-1.f / 6.f) * acc[1][t][m][j][r], m2 = (-1.f / 6.f) * acc[2][t][m][j][r];
            const float m3 = (1.f / 24.f) * acc[X3][t][m][j][r], m4 = (1.f / 24.f) * acc[X4][t][m][j][r];
            const float m5 = acc[NX - 1][t][m][j][r];
            const float sp = m1 + m2, sm = m1 - m2, tp = m3 + m4, tm = m3 - m4;
            f32x4 y;
            y[0] = (m0 + sp) + tp;
            y[1] = fmaf(2.f, tm, sm);
            y[2] = fmaf(4.f, tp, sp);
            y[3] = fmaf(8.f, tm, sm) + m5;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float v = y[e] * sc[m][r] + sh[m][r];
              if (relu) v = fmaxf(v, 0.f);
              y[e] = resid ? v + rv[t][j][m][r][e] : v;
            }
            buf_store4(yrs, off[t][j][m][r], y);
          }
  };
  auto epilogue = [&](int d0) {
#pragma unroll
  for (int t = 0; t < C::TDA; ++t) {
    const int d = C::DP ? d0 + (ci >> 1) : d0 + t;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int h = h0 + (wave * NP + j) * C::RPG + pr;
      if (d >= a.D || h >= a.H || w >= a.W) continue;
      const int nv = min(F, a.W - w);  // valid outputs of this group
#pragma unroll
      for (int m = 0; m < C::MTE; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = C::DP ? 4 * (ci & 1) + r : co0 + 16 * m + 4 * ci + r;
          if (co >= a.cout) continue;
          float y[F];
          if constexpr (F == 2) {
            const float m0 = acc[0][t][m][j][r], m1 = 0.5f * acc[1][t][m][j][r];
            const float m2 = 0.5f * acc[2][t][m][j][r], m3 = acc[3][t][m][j][r];
            y[0] = (m0 + m1) + m2;
            y[1] = (m1 - m2) - m3;
          } else {
            const float m0 = 0.25f * acc[0][t][m][j][r];
            const float m1 = (-1.f / 6.f) * acc[1][t][m][j][r], m2 = (-1.f / 6.f) * acc[2][t][m][j][r];
            const float m3 = (1.f / 24.f) * acc[3][t][m][j][r], m4 = (1.f / 24.f) * acc[4][t][m][j][r];
            const float m5 = acc[NX - 1][t][m][j][r];
            const float sp = m1 + m2, sm = m1 - m2, tp = m3 + m4, tm = m3 - m4;
            y[0] = (m0 + sp) + tp;
            y[1] = fmaf(2.f, tm, sm);
            y[F / 2] = fmaf(4.f, tp, sp);
            y[F - 1] = fmaf(8.f, tm, sm) + m5;
          }
#pragma unroll
          for (int e = 0; e < F; ++e) {
            y[e] = y[e] * sc[m][r] + sh[m][r];
            if (relu) y[e] = fmaxf(y[e], 0.f);
          }
          const long long o = (long long)co * DHW + (long long)d * HW + (long long)h * a.W + w;
          float* yp = a.y + (long long)b * a.ybs + o;
          const float* rp = a.res + (long long)b * a.rbs + o;
          const bool vec = nv == F &&
              ((reinterpret_cast<uintptr_t>(yp) | (resid ? reinterpret_cast<uintptr_t>(rp) : 0)) & (4 * F - 1)) == 0;
          if (vec) {
            if constexpr (F == 2) {
              if (resid) {
                const float2 rv = *reinterpret_cast<const float2*>(rp);
                y[0] += rv.x;
                y[1] += rv.y;
              }
              *reinterpret_cast<float2*>(yp) = make_float2(y[0], y[1]);
            } else {
              if (resid) {
                const float4 rv = *reinterpret_cast<const float4*>(rp);
                y[0] += rv.x;
                y[1] += rv.y;
                y[F / 2] += rv.z;
                y[F - 1] += rv.w;
              }
              *reinterpret_cast<float4*>(yp) = make_float4(y[0], y[1], y[F / 2], y[F - 1]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < F; ++e)
              if (e < nv) {
                if (resid) y[e] += rp[e];
                yp[e] = y[e];
              }
          }
        }
    }
  }
  };

  issue(0, smem);
  for (int it = 0; it < nitems; ++it) {
    const int ch = it % nchunks;
    wait_item<NST>(ebuf && ch == 0 && it > 0);  // this wave's pieces of item it landed
    __syncthreads();  // ... and everyone's; item it-1's stage is free
    if (it + 1 < nitems) issue(it + 1, smem + ((it + 1) & 1) * C::STAGE);
    const float* xs = smem + (it & 1) * C::STAGE;
    const float* ws = xs + C::XS;
    // one (kd, kh) step: raw inputs (F + 2 per lane as float2s) and weight rows g.
    // Depth-paired, step (p, kh) reads staged plane p once for both output planes.
    struct StepOps {
      float2 x2[C::TDA][NP][F / 2 + 1];
      float g[3][C::MTE];
    };
    auto load_step = [&](int step, StepOps& o) {
      const int kd = step / 3, kh = step % 3;
#pragma unroll
      for (int t = 0; t < C::TDA; ++t)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const float* sp = xs + xoff[j] + (t + kd) * C::PLX + kh * C::RWX;
          if constexpr (H16) {  // two 16-byte reads (bank map above); inputs 6, 7 unused
            const float4 lo = *reinterpret_cast<const float4*>(sp);
            // volatile keeps the whole second read (narrowed, it would pair into ds_read2_b64)
            typedef const volatile __attribute__((address_space(3))) f32x4 lds_f32x4;
            const f32x4 hi = *(lds_f32x4*)(sp + 4);
            o.x2[t][j][0] = make_float2(lo.x, lo.y);
            o.x2[t][j][1] = make_float2(lo.z, lo.w);
            o.x2[t][j][2] = make_float2(hi[0], hi[1]);
            continue;
          }
#pragma unroll
          for (int q = 0; q <= F / 2; ++q) o.x2[t][j][q] = *reinterpret_cast<const float2*>(sp + 2 * q);
        }
      const float* wk = ws + step * 3 * CIN_B * C::COP;
#pragma unroll
      for (int m = 0; m < C::MTE; ++m)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.g[r][m] = wk[r * CIN_B * C::COP + woff[m]];
    };
    // transforms of one step: V = B^T x per (plane, row) and U = G' g per cout tile,
    // G' = G with its rows' constant factors moved into the epilogue (kScale)
    struct Xf {
      float vb[C::TDA][NP][NX];
      float u[NX][C::MTE];
    };
    auto xform = [&](const StepOps& o, Xf& T) {
#pragma unroll
      for (int t = 0; t < C::TDA; ++t)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const float x0 = o.x2[t][j][0].x, x1 = o.x2[t][j][0].y, x2 = o.x2[t][j][1].x, x3 = o.x2[t][j][1].y;
          if constexpr (F == 2) {
            T.vb[t][j][0] = x0 - x2;
            T.vb[t][j][1] = x1 + x2;
            T.vb[t][j][2] = x2 - x1;
            T.vb[t][j][3] = x1 - x3;
          } else {
            const float x4 = o.x2[t][j][F / 2].x, x5 = o.x2[t][j][F / 2].y;
            const float pa = fmaf(-4.f, x2, x4), pb = fmaf(-4.f, x1, x3);
            const float pc = x4 - x2, pd = 2.f * (x3 - x1);
            T.vb[t][j][0] = fmaf(4.f, x0, fmaf(-5.f, x2, x4));
            T.vb[t][j][1] = pa + pb;
            T.vb[t][j][2] = pa - pb;
            T.vb[t][j][3] = pc + pd;
            T.vb[t][j][4] = pc - pd;
            T.vb[t][j][NX - 1] = fmaf(4.f, x1, fmaf(-5.f, x3, x5));
          }
        }
#pragma unroll
      for (int m = 0; m < C::MTE; ++m) {
        const float g0 = o.g[0][m], g1 = o.g[1][m], g2 = o.g[2][m];
        const float s = g0 + g2;
        T.u[0][m] = g0;
        T.u[1][m] = s + g1;
        T.u[2][m] = s - g1;
        if constexpr (F == 4) {
          const float s4 = fmaf(4.f, g2, g0);
          T.u[3][m] = fmaf(2.f, g1, s4);
          T.u[4][m] = fmaf(-2.f, g1, s4);
        }
        T.u[NX - 1][m] = g2;
      }
    };
    auto mfmas = [&](const Xf& T) {
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int t = 0; t < C::TDA; ++t)
#pragma unroll
          for (int m = 0; m < C::MTE; ++m)
#pragma unroll
            for (int j = 0; j < NP; ++j)
              acc[x][t][m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(T.u[x][m], T.vb[t][j][x], acc[x][t][m][j], 0, 0, 0);
    };
    // software pipeline over the NSTEP steps: LDS reads two steps ahead, transforms one
    // step ahead, so a step's VALU runs under the previous step's MFMAs
    StepOps ops[2];
    Xf xf[2];
    if constexpr (FENCE) {
      // fenced schedule (r04, as the W x D per-lane tile's PV = 5): each step's MFMAs
      // issue as one block, then the next step's transforms and the LDS reads two ahead
      load_step(0, ops[0]);
      xform(ops[0], xf[0]);
      load_step(1, ops[1]);
#pragma unroll
      for (int step = 0; step < C::NSTEP; ++step) {
        __builtin_amdgcn_sched_barrier(0);
        mfmas(xf[step & 1]);
        __builtin_amdgcn_sched_barrier(0);
        if (step + 1 < C::NSTEP) xform(ops[(step + 1) & 1], xf[(step + 1) & 1]);
        if (step + 2 < C::NSTEP) load_step(step + 2, ops[step & 1]);
      }
    } else {
    // scheduler hint: interleave the step's LDS reads / VALU transforms with the MFMAs
    // (same-box sweep r02: -1 to -4 % per layer; iglp_opt(1) and s_setprio gained less)
    __builtin_amdgcn_iglp_opt(0);
    load_step(0, ops[0]);
    load_step(1, ops[1]);
    xform(ops[0], xf[0]);
#pragma unroll
    for (int step = 0; step < C::NSTEP; ++step) {
      if (step + 1 < C::NSTEP) xform(ops[(step + 1) & 1], xf[(step + 1) & 1]);
      if (step + 2 < C::NSTEP) load_step(step + 2, ops[step & 1]);
      mfmas(xf[step & 1]);
    }
    }
    if (ch == nchunks - 1) {  // the depth group's last chunk: its epilogue, fresh accumulators
      if (ebuf)
        epilogue_buf((dz0 + it / nchunks) * TD);
      else
        epilogue((dz0 + it / nchunks) * TD);
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int t = 0; t < C::TDA; ++t)
#pragma unroll
          for (int m = 0; m < C::MTE; ++m)
#pragma unroll
            for (int j = 0; j < NP; ++j) acc[x][t][m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// weights [cout][cin][3][3][3] -> per (cout block, chunk): [kd*3+kh][kw][ci][COP col]
// (the kernel forms U = G g from each staged kw row)
template <int MT>
__global__ void pack_wino_kernel(const float* __restrict__ w, float* __restrict__ packed, int cout,
                                 int cin, int nchunks, long long total) {
  constexpr int COP = 16 * MT;
  constexpr bool SWZ = (COP % 32) == 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int col = (int)(q % COP); q /= COP;
    const int ci = (int)(q % CIN_B); q /= CIN_B;
    const int kw = (int)(q % 3); q /= 3;
    const int kdkh = (int)(q % 9); q /= 9;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int mm = col / 16, n = col % 16;
    const int m = SWZ ? (mm ^ (ci & 1)) : mm;
    const int co = cb * COP + 16 * m + n;
    const int c = ch * CIN_B + ci;
    packed[i] = (co < cout && c < cin) ? w[(((long long)co * cin + c) * 9 + kdkh) * 3 + kw] : 0.f;
  }
}

// depth-paired weights (couts <= 8) -> per chunk: [p * 3 + kh][kw][ci][8 t + c] =
// W[c][ci][kd = p - t][kh][kw] (zero outside kd in 0..2): staged plane p feeds
// output plane d0 + t through tap kd = p - t
__global__ void pack_wino_dp_kernel(const float* __restrict__ w, float* __restrict__ packed, int cout,
                                    int cin, int nchunks, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int col = (int)(q % 16); q /= 16;
    const int ci = (int)(q % CIN_B); q /= CIN_B;
    const int kw = (int)(q % 3); q /= 3;
    const int step = (int)(q % 12); q /= 12;
    const int ch = (int)q;  // >= nchunks in the tail pad
    const int co = col & 7, kd = step / 3 - (col >> 3), kh = step % 3;
    const int c = ch * CIN_B + ci;
    packed[i] = (ch < nchunks && co < cout && c < cin && kd >= 0 && kd <= 2)
                    ? w[(((long long)co * cin + c) * 9 + kd * 3 + kh) * 3 + kw]
                    : 0.f;
  }
}

struct Plan {
  int f, q, mt, np, td;
  bool d2;   // two-dimensional engine (conv3d_wino2.hip) with tile p2
  Plan2 p2;
  bool h16;  // 1-D engine: halo staged as 16-byte pieces (plan_halo16)
};

int g_override[3] = {0, 0, 0};  // np, td, f (lea_conv3d_wino_set_tile_override)
// lea_conv3d_wino_set_variant: 0 = the planner's choice (5), 1 = F(4,3)-along-W engine only,
// 2..4 = the W x D engine's tiles where it applies (2: four waves, one cout tile each;
// 3: eight waves; 4: two cout tiles per wave at one wave per SIMD), 5..7 = the same
// with the inputs transformed once per chunk into LDS (32-cout blocks; 16-cout blocks
// keep 2)
int g_variant = 0;
int g_spw = 0;  // lea_conv3d_wino2_set_walk: depth pairs per workgroup (0 = planner)
// lea_conv3d_wino_set_small_cout: couts <= 8 packed / planned as 16-row blocks for the
// W x D engine (1) or depth-paired for the 1-D engine (0, the default: r02 sweep, L0 8->8
// 175 us depth-paired vs 210 us on the W x D engine's half-empty 16-row block)
int g_small16 = 0;
// lea_conv3d_wino_set_block48: 48k-cout layers as 48-row blocks of the 1-D engine (1) or
// as 32-row blocks of the W x D engine, the last one padded (0)
int g_block48 = 1;
int g_epibuf = 1;  // lea_conv3d_wino_set_epi_buf
int g_halo16 = 1;  // lea_conv3d_wino2_set_halo16
int g_pipe = 1;    // lea_conv3d_wino2_set_pipeline
int g_wpre = 1;    // lea_conv3d_wino2p_set_wpre (r06: -0.7 % on the kernel, bit-identical)
int g_fence = 1;   // lea_conv3d_wino_set_fence: the depth-paired 16-byte-halo tile's fenced schedule (r04 default)
int g_lane16 = 2;  // lea_conv3d_wino2_set_lane_halo16 (2: the fenced step schedule, PV = 5; r04 default)
// lea_conv3d_wino_set_w22: layers on the F(2,3) x F(2,3) tile (conv3d_wino22.hip): 0 none (LEA_PAIR_SUM
// always), 1 the 16-cout layers, 2 every cout <= 32
int g_w22 = 0;
inline int host_mt(int cout) {
  if (g_small16 && cout <= 8) return 1;
  const int mt = mt_of(cout);
  return (mt == 3 && !g_block48) ? 2 : mt;
}
// the staged g rows of every (cout block, chunk) + one 256-float tail (the kernels stage
// whole 256-float pieces per chunk), in floats
inline long long staged_floats(int cout, int cin) {
  const int mt = host_mt(cout), cop = cop_of(mt), nstep = mt == 0 ? 12 : 9;
  return (long long)((cout + cop - 1) / cop) * (cin / CIN_B) * nstep * 3 * CIN_B * cop + 256;
}
// packed layout: the staged rows; (32-cout blocks) the pipelined F(4,3) x F(2,3) tile's per-lane
// copies; (16- and 32-cout blocks) the F(4,3) x F(4,3) tile's per-lane copy, in 32-cout blocks
// (conv3d_wino44.hip, r06); (couts <= 32) the F(2,3) x F(2,3) tile's U
inline bool has_u22(int cout) { return cout <= 32; }
inline bool has_l44(int cout) { return host_mt(cout) == 1 || host_mt(cout) == 2; }
inline long long l44_offset(int cout, int cin) {
  return staged_floats(cout, cin) + (host_mt(cout) == 2 ? lane_weights_floats(cout, cin) : 0);
}
inline long long u22_offset(int cout, int cin) {
  return l44_offset(cout, cin) + (has_l44(cout) ? lane44_floats(cout, cin) : 0);
}

// W x D engine tile for variant v (2..4), or nullptr-equivalent (q = 0) when the
// layer's cout block has no such tile (couts <= 8 and the 48-row blocks stay 1-D)
inline Plan2 plan2(int v, int mt, int q) {
  Plan2 t{0, 0, 0, 0, 0, 0, 0};
  if (mt != 1 && mt != 2) return t;
  if (v >= 5) {
    t.pv = mt == 2 ? 1 : 0;
    v -= 3;
  }
  t.q = q;
  t.mte = 1;
  t.wc = mt;
  t.nw = 4;
  t.occ = 2;
  if (v == 3 && mt == 2) t.nw = 8;
  if (v == 4 && mt == 2) {
    t.wc = 1;
    t.mte = 2;
    t.occ = 1;
  }
  if (t.q == 16 && t.wc == 2 && t.nw == 4) t.q = 8;  // 64-wide rows would leave a 2-row tile
  if (t.pv) t.q = 8;  // the transformed 64-wide halo does not fit beside the stages
  return t;
}

inline Plan make_plan(int B, int cout, int D, int H, int W) {
  // r01 sweeps (tools/wino_sweep.py, profiles/r01_wino_sweep*.txt): F(4,3) on
  // 64-wide tile rows where they waste little of W (the L0 volumes), else on
  // 32-wide row pairs (L1, L2), F(2,3) for the 48-row blocks (their LDS budget);
  // two output planes per workgroup unless the volume is too shallow to fill the chip.
  Plan p;
  p.h16 = false;
  p.mt = host_mt(cout);
  const long long ncob = (cout + cop_of(p.mt) - 1) / cop_of(p.mt);
  auto fits = [&](int tw) { return (W + tw - 1) / tw * tw * 10 <= W * 11; };  // <= 10 % padding
  p.f = 2;
  p.q = 16;
  if (p.mt != 3) {
    p.f = 4;
    if (!fits(64)) p.q = 8;  // F(4,3) over 32-wide row pairs: F(2,3)'s tile width, 3/4 its MFMAs
  } else if (fits(32)) {
    p.f = 4;  // 48-row blocks: row pairs one plane deep fit the LDS (F(2,3) otherwise)
    p.q = 8;
  }
  auto wgs = [&](int np, int td) {
    const int tw = p.f * p.q, th = 4 * np * (16 / p.q);
    return (long long)((W + tw - 1) / tw) * ((H + th - 1) / th) * ((D + td - 1) / td) * B * ncob;
  };
  p.np = (p.f == 2 && p.mt == 2 && wgs(2, 2) >= 512) ? 2 : 1;
  p.td = (wgs(p.np, 2) >= 384 && !(p.mt == 3 && p.f == 4)) ? 2 : 1;
  if (g_override[0] > 0) {
    p.np = g_override[0];
    p.td = g_override[1];
    if (g_override[2] > 0) {
      p.f = g_override[2] == 8 ? 4 : g_override[2];
      p.q = g_override[2] == 8 ? 8 : 16;
    }
  }
  if (p.mt == 0) {  // depth-paired: F(4,3), one row set, two planes (the instantiated tiles)
    p.f = 4;
    p.np = 1;
    p.td = 2;
  }
  p.d2 = false;
  // r02 sweep (tools/wino2_sweep.py, profiles/r02_wino2_sweep.txt): the W x D engine
  // with the per-chunk transform pass wins on every 32-cout block (stem0 -14 %,
  // conv1/2 -14 %), the per-lane form on the 16-cout L1 cells (-11 %)
  // (a 1-D tile override from the tuning tools keeps the planner on the 1-D engine)
  const int v = g_variant == 0 ? (g_override[0] > 0 ? 1 : 5) : g_variant;
  if (v >= 2) {
    p.p2 = plan2(v, p.mt, fits(64) ? 16 : 8);
    p.d2 = p.p2.q > 0;
    if (g_spw > 0) p.p2.spw = g_spw;
  }
  return p;
}

// The W x D transform-pass kernel stages its halo as 16-byte LDS-DMA pieces (PV = 2, 4
// pieces per channel instead of 13 dword pieces) when rows are whole 16-byte blocks:
// W % 4 == 0 and 16-byte aligned channel bases (r03 stamps: the DMA issue held 25-27 %
// of the kernel's wave cycles with dword pieces).  Plain volumes only (not the cost volume).
inline void plan_halo16(Plan& p, bool cv, int W, const ConvArgs* a, int cin = 0) {
  if (a) cin = a->cin;
  p.h16 = false;
  if (cv || !g_halo16 || W % 4 != 0) return;
  if (a) {
    const bool al = ((uintptr_t)a->x & 15) == 0 && a->xbs % 4 == 0 &&
                    (a->cin1 == a->cin || (((uintptr_t)a->x2 & 15) == 0 && a->x2bs % 4 == 0));
    if (!al) return;
  }
  if (p.d2) {
    // the one-barrier pipeline uses the buffer-addressed epilogue only
    // (layers of one or two chunks per depth pair stay on the two-barrier tile: L0 8->24
    // ran 286 us there, 296-301 us pipelined -- r03 sweeps)
    // (g_w44 == 2: the two-chunk layers -- L0 8 -> 24 -- on the F(4,3) x F(4,3) tile too)
    const bool pipe = g_pipe && g_epibuf && (a == nullptr || epi_buf_ok(*a)) &&
                      (cin == 0 || cin > 2 * CIN_B || (g_w44 >= 2 && cin > CIN_B));
    if (p.p2.pv == 1 && p.p2.nw == 4 && p.p2.mte == 1) p.p2.pv = pipe ? 3 : 2;
    // the per-lane 16-cout tile (the L1 cells): 16-byte pieces, interleaved row sets (r04)
    if (g_lane16 && p.p2.pv == 0 && p.p2.q == 8 && p.p2.wc == 1 && p.p2.mte == 1 && p.p2.nw == 4 &&
        p.p2.occ == 2)
      p.p2.pv = g_lane16 == 2 ? 5 : 4;
    // g_w44 == 3 (r06 experiment): the 16-cout layers on the F(4,3) x F(4,3) tile as half-empty
    // 32-cout blocks (the pipelined tile's plan: pv 3 with two cout tiles)
    if (g_w44 == 3 && pipe && p.mt == 1 && (p.p2.pv == 4 || p.p2.pv == 5)) {
      p.p2.pv = 3;
      p.p2.wc = 2;
    }
  } else if (p.mt == 0 && p.f == 4 && p.q == 16 && p.np == 1 && p.td == 2) {
    p.h16 = true;  // the depth-paired 64-wide tile (the L0 8-channel cell ops)
  }
}

#define LEA_WINO_CASE(F, Q, MT, NP, TD, CV)                                                   \
  if (p.f == F && p.q == Q && p.mt == MT && p.np == NP && p.td == TD) {                       \
    using C_ = Cfg<F, Q, MT, NP, TD>;                                                         \
    a.tiles_w = (a.W + C_::TW - 1) / C_::TW;                                                  \
    a.ntiles = a.tiles_w * ((a.H + C_::TH - 1) / C_::TH);                                     \
    a.ndz = (a.D + TD - 1) / TD;                                                              \
    a.spw = std::max(1, std::min(g_spw > 0 ? g_spw : auto_walk(a, B, 2), a.ndz));             \
    const long long n_ = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;    \
    LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino): grid too large");                      \
    a.nblk = (int)n_;                                                                         \
    conv3d_wino_kernel<F, Q, MT, NP, TD, CV><<<dim3((unsigned)n_), kConvThreads, 0, st>>>(a); \
    return launch_status("lea_conv3d(wino)");                                                \
  }
#define LEA_WINO_TILES(CV)                                                                                  \
  LEA_WINO_CASE(2, 16, 1, 1, 1, CV) LEA_WINO_CASE(2, 16, 1, 1, 2, CV) LEA_WINO_CASE(2, 16, 1, 2, 1, CV)     \
  LEA_WINO_CASE(2, 16, 1, 2, 2, CV) LEA_WINO_CASE(2, 16, 2, 1, 1, CV) LEA_WINO_CASE(2, 16, 2, 1, 2, CV)     \
  LEA_WINO_CASE(2, 16, 2, 2, 1, CV) LEA_WINO_CASE(2, 16, 2, 2, 2, CV) LEA_WINO_CASE(2, 16, 3, 1, 1, CV)     \
  LEA_WINO_CASE(2, 16, 3, 1, 2, CV) LEA_WINO_CASE(4, 16, 1, 1, 1, CV) LEA_WINO_CASE(4, 16, 1, 1, 2, CV)     \
  LEA_WINO_CASE(4, 16, 2, 1, 1, CV) LEA_WINO_CASE(4, 16, 2, 1, 2, CV) LEA_WINO_CASE(4, 8, 1, 1, 1, CV)      \
  LEA_WINO_CASE(4, 8, 1, 1, 2, CV) LEA_WINO_CASE(4, 8, 2, 1, 1, CV) LEA_WINO_CASE(4, 8, 2, 1, 2, CV)      \
  LEA_WINO_CASE(4, 8, 3, 1, 1, CV) LEA_WINO_CASE(4, 16, 0, 1, 2, CV) LEA_WINO_CASE(4, 8, 0, 1, 2, CV)

int run(const Plan& p, ConvArgs a, int B, hipStream_t st, bool cv) {
  if (p.d2) return run2(p.p2, a, B, st, cv);
  a.ncob = (a.cout + cop_of(p.mt) - 1) / cop_of(p.mt);
  if (p.h16) {
    using C_ = Cfg<4, 16, 0, 1, 2, true>;
    a.tiles_w = (a.W + C_::TW - 1) / C_::TW;
    a.ntiles = a.tiles_w * ((a.H + C_::TH - 1) / C_::TH);
    a.ndz = (a.D + 1) / 2;
    a.spw = std::max(1, std::min(g_spw > 0 ? g_spw : auto_walk(a, B, 2), a.ndz));
    const long long n_ = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;
    LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino): grid too large");
    a.nblk = (int)n_;
    if (g_fence)
      conv3d_wino_kernel<4, 16, 0, 1, 2, false, true, true><<<dim3((unsigned)n_), kConvThreads, 0, st>>>(a);
    else
      conv3d_wino_kernel<4, 16, 0, 1, 2, false, true><<<dim3((unsigned)n_), kConvThreads, 0, st>>>(a);
    return launch_status("lea_conv3d(wino)");
  }
  if (cv) {
    LEA_WINO_TILES(true)
  } else {
    LEA_WINO_TILES(false)
  }
  set_error("lea_conv3d(wino): no tile f=%d q=%d mt=%d np=%d td=%d", p.f, p.q, p.mt, p.np, p.td);
  return LEA_E_UNSUPPORTED;
}

thread_local char g_name[96];

const char* name(const Plan& p, bool cv) {
  if (p.d2) return name2(p.p2, cv);
  snprintf(g_name, sizeof(g_name), "conv3d_wino_kernel<%d, %d, %d, %d, %d, %s%s>", p.f, p.q, p.mt, p.np,
           p.td, cv ? "true" : "false", p.h16 ? (g_fence ? ", true, true" : ", true") : "");
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
                    (long long)(a.cout + 47) * a.D * a.H * a.W < (1LL << 31),
                "lea_conv3d(wino): volume too large");
  LEA_CHECK_ARG(a.x != a.y && a.x2 != a.y, "lea_conv3d(wino): input aliases output");
  if (dtype != LEA_F32) {
    set_error("lea_conv3d(wino): dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  Plan p = make_plan(B, a.cout, a.D, a.H, a.W);
  const bool pair = a.flags & LEA_PAIR_SUM;
  if (pair) {
    LEA_CHECK_ARG(!(a.flags & LEA_RESIDUAL) && a.cin1 > 0 && a.cin1 < a.cin && !cv,
                  "lea_conv3d(wino): LEA_PAIR_SUM needs two sources and no residual");
    if (!wino22_ok(a)) {
      set_error("lea_conv3d(wino): LEA_PAIR_SUM unsupported for cout=%d W=%d (or unaligned operands)", a.cout, a.W);
      return LEA_E_UNSUPPORTED;
    }
  }
  if (pair || (g_w22 && !cv && (p.mt == 1 || g_w22 == 2) && g_variant == 0 && g_override[0] == 0 &&
               wino22_ok(a))) {
    a.uoff = u22_offset(a.cout, a.cin);
    return run22(a, B, g_spw, as_stream(stream));
  }
  plan_halo16(p, cv, a.W, &a);
  if (g_epibuf && epi_buf_ok(a)) a.flags |= kEpiBuf;
  if (has_l44(a.cout)) a.uoff = l44_offset(a.cout, a.cin);  // (the F(4,3) x F(4,3) tile's section)
  return run(p, a, B, as_stream(stream), cv);
}

}  // namespace wino
}  // namespace lea

using namespace lea;

extern "C" size_t lea_conv3d_wino_packed_floats(int cout, int cin) {
  if (cout <= 0 || cin <= 0 || cin % wino::CIN_B != 0) return 0;
  // 32-cout blocks append the per-lane copy (16-byte slices) the one-barrier W x D tile loads
  // (PV = 3), couts <= 32 the F(2,3) x F(2,3) tile's U (conv3d_wino22.hip)
  return (size_t)wino::u22_offset(cout, cin) + (wino::has_u22(cout) ? (size_t)wino::u22_section(cout, cin) : 0);
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
  const long long staged = wino::staged_floats(cout, cin), uoff = wino::u22_offset(cout, cin),
                  l44 = wino::l44_offset(cout, cin);
  switch (wino::host_mt(cout)) {
    case 0: wino::pack_wino_dp_kernel<<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, staged); break;
    case 1: wino::pack_wino_kernel<1><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, staged); break;
    case 3: wino::pack_wino_kernel<3><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, staged); break;
    default: {
      const long long lane = wino::lane_raw_floats(cout, cin), lanew = l44 - staged - lane;
      wino::pack_wino_kernel<2><<<grid, 256, 0, st>>>(w, packed, cout, cin, cin / wino::CIN_B, staged);
      const int g2 = (int)std::min<long long>((lane + 255) / 256, 4096);
      wino::pack_wino_lane_kernel<<<g2, 256, 0, st>>>(w, packed + staged, cout, cin, cin / wino::CIN_B, lane);
      const int g3 = (int)std::min<long long>((lanew + 255) / 256, 4096);
      wino::pack_wino_lane_wpre_kernel<<<g3, 256, 0, st>>>(w, packed + staged + lane, cout, cin,
                                                           cin / wino::CIN_B, lanew);
    }
  }
  if (wino::has_l44(cout)) {  // the F(4,3) x F(4,3) tile's per-lane copies (G_W' g, then U)
    const long long n44 = wino::lane44_g_floats(cout, cin), n44u = wino::lane44_floats(cout, cin) - n44;
    const int g4 = (int)std::min<long long>((n44 + 255) / 256, 4096);
    wino::pack_wino44_lane_kernel<<<g4, 256, 0, st>>>(w, packed + l44, cout, cin, cin / wino::CIN_B, n44);
    const int g5 = (int)std::min<long long>((n44u + 255) / 256, 4096);
    wino::pack_wino44_lane_u_kernel<<<g5, 256, 0, st>>>(w, packed + l44 + n44, cout, cin, cin / wino::CIN_B, n44u);
  }
  if (wino::has_u22(cout)) {  // the F(2,3) x F(2,3) tile's U
    const long long u = total - uoff;
    const int g2 = (int)std::min<long long>((u + 255) / 256, 4096);
    wino::pack_wino22_kernel<<<g2, 256, 0, st>>>(w, packed + uoff, cout, cin, u);
  }
  return launch_status("lea_conv3d_wino_pack_weights");
}

extern "C" const char* lea_conv3d_wino_kernel_name(int B, int cin, int cout, int D, int H, int W,
                                                   int costvolume) {
  if (B <= 0 || cout <= 0 || D <= 0 || H <= 0 || W <= 0) return nullptr;
  wino::Plan p = wino::make_plan(B, cout, D, H, W);
  if (wino::g_w22 && !costvolume && (p.mt == 1 || (wino::g_w22 == 2 && cout <= 32)) && wino::g_variant == 0 &&
      wino::g_override[0] == 0 && W % 4 == 0)
    return "conv3d_wino22_kernel";  // (assumes 16-byte aligned sources)
  wino::plan_halo16(p, costvolume != 0, W, nullptr, cin);  // (assumes 16-byte aligned sources)
  return wino::name(p, costvolume != 0);
}

extern "C" int lea_conv3d_wino_set_tile_override(int np, int td, int f) {
  clear_error();
  if (np <= 0) {
    wino::g_override[0] = 0;
    return 0;
  }
  LEA_CHECK_ARG((np == 1 || np == 2) && (td == 1 || td == 2) && (f == 0 || f == 2 || f == 4 || f == 8),
                "lea_conv3d_wino_set_tile_override: bad tile np=%d td=%d f=%d", np, td, f);
  wino::g_override[0] = np;
  wino::g_override[1] = td;
  wino::g_override[2] = f;
  return 0;
}

extern "C" int lea_conv3d_wino_set_block48(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino_set_block48: on=%d", on);
  wino::g_block48 = on;
  return 0;
}

extern "C" int lea_conv3d_wino_set_epi_buf(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino_set_epi_buf: on=%d", on);
  wino::g_epibuf = on;
  return 0;
}

extern "C" int lea_conv3d_wino_set_small_cout(int mode) {
  clear_error();
  LEA_CHECK_ARG(mode == 0 || mode == 1, "lea_conv3d_wino_set_small_cout: mode=%d", mode);
  wino::g_small16 = mode;
  return 0;
}

extern "C" int lea_conv3d_wino2_set_pipeline(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino2_set_pipeline: on=%d", on);
  wino::g_pipe = on;
  return 0;
}

extern "C" int lea_conv3d_wino44_set(int on) {
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 3, "lea_conv3d_wino44_set: on=%d", on);
  wino::g_w44 = on;
  return 0;
}

extern "C" int lea_conv3d_wino44_set_group(int g) {
  clear_error();
  LEA_CHECK_ARG(g >= -1 && g <= 16, "lea_conv3d_wino44_set_group: %d", g);
  wino::g_w44g = g;
  return 0;
}

extern "C" int lea_conv3d_wino44_set_sched(int s) {
  clear_error();
  LEA_CHECK_ARG(s >= 0 && s <= 3, "lea_conv3d_wino44_set_sched: %d", s);
  wino::g_w44s = s;
  return 0;
}

extern "C" int lea_conv3d_wino44_set_upre(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino44_set_upre: on=%d", on);
  wino::g_w44u = on;
  return 0;
}

extern "C" int lea_conv3d_wino2p_set_wpre(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino2p_set_wpre: on=%d", on);
  wino::g_wpre = on;
  return 0;
}

extern "C" int lea_conv3d_wino_set_fence(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino_set_fence: on=%d", on);
  wino::g_fence = on;
  return 0;
}

extern "C" int lea_conv3d_wino2_set_lane_halo16(int on) {
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 2, "lea_conv3d_wino2_set_lane_halo16: on=%d", on);
  wino::g_lane16 = on;
  return 0;
}

extern "C" int lea_conv3d_wino2_set_halo16(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_wino2_set_halo16: on=%d", on);
  wino::g_halo16 = on;
  return 0;
}

extern "C" int lea_conv3d_wino2_set_walk(int spw) {
  clear_error();
  LEA_CHECK_ARG(spw >= 0 && spw <= 64, "lea_conv3d_wino2_set_walk: spw=%d", spw);
  wino::g_spw = spw;
  return 0;
}

extern "C" int lea_conv3d_wino_set_w22(int on) {
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 2, "lea_conv3d_wino_set_w22: on=%d", on);
  wino::g_w22 = on;
  return 0;
}

extern "C" int lea_conv3d_wino_set_variant(int variant) {
  clear_error();
  LEA_CHECK_ARG(variant >= 0 && variant <= 7, "lea_conv3d_wino_set_variant: bad variant %d", variant);
  wino::g_variant = variant;
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
  LEA_CHECK_FLAGS(flags, LEA_RELU | LEA_RESIDUAL | LEA_PAIR_SUM, "lea_conv3d_bnrelu_wino");
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
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_conv3d_bnrelu_costvolume_wino");
  LEA_CHECK_ARG(left && right && y != left && y != right,
                "lea_conv3d_bnrelu_costvolume_wino: null or aliased pointer");
  return wino::common(a, B, true, dtype, stream);
}
