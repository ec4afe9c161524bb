// ConvBR3d k=3 (fp32) with two-dimensional Winograd: F(4,3) along W x F(2,3) along D
// on the fp32 matrix cores.  Replaces models/operations_3d.py:31-47 for the matching
// net's 3x3x3 layers, as conv3d_wino.hip (F(4,3) along W only) does, with 2/3 of its
// MFMA work: per output group of 4 (W) x 2 (D) voxels and kernel row kh,
//     y[d0 + t][w + j] = sum_{kd, kw} g[kd][kh][kw] x[d0 - 1 + t + kd][w - 1 + j + kw]
//                      = A_D^T [ A_W^T ( (G_W g G_D^T) . (B_W^T x B_D) ) ]
// takes 6 x 4 = 24 products per input channel, against 2 planes x 3 kd x 6 = 36 for
// F(4,3) along W alone and 8 x 9 = 72 for the direct convolution.
//   W: points 0, +-1, +-2, inf (conv3d_wino.hip's transforms, G's row factors 1/4,
//      -1/6, -1/6, 1/24, 1/24, 1 applied to the accumulators in the epilogue)
//   D: F(2,3): B^T x = (x0 - x2, x1 + x2, x2 - x1, x1 - x3),
//      G g = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2), A^T m = (m0+m1+m2, m1-m2-m3)
// The two output planes of a group are exactly the TD = 2 planes the 1-D engine
// stages (4 input planes), so the halo, its LDS-DMA and the weight stage (the raw g
// rows of a 4-channel chunk) are the 1-D engine's; what changes is the step loop
// (3 kh steps of 24 points instead of 9 (kd, kh) steps of 6 points x 2 planes) and
// the accumulators (24 per 16 x 16 tile: 3 per output instead of 1.5).
//
// GEMM per point (xi, eta) and kh:
//     M[xi][eta][co][group] += sum_ci U[xi][eta][kh][co][ci] * V[xi][eta][kh][ci][group]
// on v_mfma_f32_16x16x4_f32 with the 1-D engine's lane map: A (lane l) = U[co = 16 m +
// (l & 15)][ci = l >> 4], B (lane l) = V[ci = l >> 4][group = l & 15].  Each lane forms
// its V from 4 planes x 6 staged inputs (12 ds_read_b64) and U from its cout's 9 g
// values of the step (B_W per plane row then B_D per point; G_W per kd row then G_D).
//
// Workgroup = NW waves = WR row sets x WC cout tiles; a wave owns MTE 16-row cout
// tiles (MTE = 2 only at one wave per SIMD: 192 accumulator registers).
#include "wino_common.h"

namespace lea {
namespace wino {

template <int Q, int WC, int MTE, int NW, int OCC, int PV>
struct Cfg2 {
  static constexpr int F = 4, NX = 6, NE = 4, TD = 2;
  static constexpr int WR = NW / WC;             // row sets (waves along H)
  static_assert(WR * WC == NW, "waves = row sets x cout tiles");
  static constexpr int COP = 16 * WC * MTE;      // couts per workgroup (packed block)
  static constexpr bool SWZ = (COP % 32) == 0;   // the packer's odd-ci half swap
  static constexpr int RPG = 16 / Q;             // tile rows per lane group
  static constexpr int TW = F * Q;               // outputs per tile row
  static constexpr int TH = WR * RPG;
  static constexpr int RH = TH + 2, RW = TW + 2;
  static constexpr int PLANE = RH * RW;
  static constexpr int PLANES = TD + 2;
  static constexpr int IMG = PLANES * PLANE;
  static constexpr int XSLOTS = (IMG + 63) / 64;
  // channel stride: for the per-lane V path, the 1-D engine's (the two channels of a
  // 32-lane ds_read_b64 group on disjoint banks); for PV = 1, = 32 mod 64 dwords, which
  // with RW = 34 puts the transform pass's 32-lane reads (8 groups x 2 rows x 2
  // channels, see below) on 64 distinct banks
  // (per-lane V: room for whole pieces of every wave -- NW * ceil(XSLOTS / NW) -- so the
  // staging issues the same count from each wave without a branch; the surplus pieces
  // read out of range: zeros into the padding)
  static constexpr int CIS = PV ? (64 * XSLOTS + 32)
                                : conflict_free_cis<F, Q>(64 * NW * ((XSLOTS + NW - 1) / NW), RW);
  // PV = 2: rows staged as 16-byte blocks from w0 - 4 (RWA = TW + 8 floats: 10 blocks
  // cover the w0 - 1 .. w0 + TW halo columns), one channel's 4 planes x RH rows
  // contiguous (BLK16 blocks = PIECES16 LDS-DMA pieces of 64 lanes, the last one
  // partial); channel c starts at CB2(c) == {1, 3, 33, 35}[c] mod 64 dwords, so column
  // w0 - 1 sits at an even dword (the pass's ds_read_b64s stay 8-byte aligned) and the
  // pass's 32 lanes (8 groups x 4 channels of one row) read 64 distinct banks
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
  // PV = 4 (r04, per-lane V, the 16-cout tiles): 16-byte halo pieces (PIECES16 = 7 per
  // channel, 28 per item) into channel regions CS4 = 7 x 256 floats apart (whole pieces: the
  // partial last piece's surplus lanes land in the region's pad), bases 1 mod 4 so column
  // w0 - 1 sits 16-byte aligned: a lane reads its 6 inputs per (plane, row) as two
  // ds_read_b128 (the compiler pairs float2 reads into ds_read2_b64, banked mod 32 over
  // 16-lane groups: 2-way on this tile, 42 % of the LDS cycles in the r04 counters).  With the
  // lane group's two rows 4 tile rows apart (rows wr, wr + 4) every b128 lane group
  // ({0-3,12-15,20-27}, ...) reads 64 distinct banks (exhaustive check over the row sets,
  // kh, planes and both reads)
  static constexpr bool H4 = PV == 4 || PV == 5;  // PV = 5: PV = 4 with the fenced step schedule
  static constexpr int CS4 = PIECES16 * 256;
  static constexpr int cb4(int c) { return 1 + c * CS4; }
  static constexpr int XS = PV == 2 ? (cb2(CIN_B - 1) + IMGA + 3) / 4 * 4
                          : H4 ? (cb4(CIN_B) + 3) / 4 * 4 : CIN_B * CIS;
  static constexpr int WS = 27 * CIN_B * COP;    // g[kd*3+kh][kw][ci][co] of one chunk
  static constexpr int WSLOTS = (WS + 255) / 256;
  static constexpr int STAGE = XS + 256 * WSLOTS;
  // PV: the chunk's V = B_W^T x B_D for every (channel, halo row, group), formed once
  // per chunk by the whole workgroup into T[ci][row][group][eta][xi] (24 floats per
  // group: six ds_read_b128 per lane and step) instead of per lane and step.
  // PV = 1: ds_read_b128 of 16 lanes (4 groups x 2 rows x 2 channels per LDS cycle):
  // groups 24 floats apart take 8 of the 16 16-B slots of a bank row, a row stride of
  // 4 mod 8 floats the other 8, a channel stride of 0 mod 64 keeps the channel pairs apart.
  // PV = 2 (r03, after the counters showed 60 M conflict cycles per launch): banked as the
  // hardware groups the lanes (MI355X_MICROARCH.md, LDS): the loop's ds_read_b128 serves
  // lanes {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32) per cycle, 64 banks; the pass's
  // ds_write_b128 serves 8 contiguous lanes (8 groups of one channel and row), 32 banks.
  // A group stride of GS = 28 floats (7 16-B slots: 8 groups on 8 distinct slots mod 32
  // banks), a row stride of 224 (56 slots = 8 mod 16) and a channel stride of 0 mod 64
  // put every read group on 16 distinct slots (exhaustive check over the 16 x 16 strides)
  static constexpr int GS = PV == 2 ? 28 : 24;   // floats per group's V (24 used)
  static constexpr int TRS = PV == 2 ? Q * GS : Q * 24 + 4;  // floats per halo row
  // floats per channel: 0 mod 64 (PV = 1: the pass's 16-lane b128 writes pair rows,
  // TRS = 4 mod 8 apart; PV = 2: see above)
  static constexpr int TCS = (RH * TRS + 63) / 64 * 64;
  static constexpr int TS = (PV == 1 || PV == 2) ? CIN_B * TCS : 0;
  static constexpr bool VPASS = PV == 1 || PV == 2;  // V formed by a per-chunk pass into LDS
  static constexpr int NUNIT = CIN_B * RH * Q;   // (channel, row, group) transforms per chunk
  static constexpr int WG_PER_CU = 4 * OCC / NW;
  static_assert(WG_PER_CU >= 1, "occupancy");
  static_assert(XS % 4 == 0 && WS % 4 == 0 && RW % 2 == 0 && PLANE % 2 == 0, "aligned LDS regions");
  static_assert(PV != 2 || (TW == 32 && NW % PIECES16 == 0 && cb2(1) % 64 == 3 && cb2(2) % 64 == 33 &&
                            cb2(3) % 64 == 35), "16-byte halo map");
  static_assert(!H4 || (Q == 8 && WC == 1 && MTE == 1 && NW == 4 && CS4 % 64 == 0 && (4 * RWA) % 64 == 32 &&
                            PLANEA % 4 == 0 && RWA % 4 == 0 && RH == 2 * NW + 2), "PV = 4 halo map");
  static_assert((2 * STAGE + TS) * 4 * WG_PER_CU <= 160 * 1024, "double-buffered stages fit the LDS");
};

// F(4,3) along W: B^T x of 6 staged inputs, G' g of one kernel row (G without its
// row factors), A^T (with the factors) of 6 accumulators -> 4 outputs.
__device__ __forceinline__ void bw4(const float x0, const float x1, const float x2, const float x3,
                                    const float x4, const float x5, float* v) {
  const float pa = fmaf(-4.f, x2, x4), pb = fmaf(-4.f, x1, x3);
  const float pc = x4 - x2, pd = 2.f * (x3 - x1);
  v[0] = fmaf(4.f, x0, fmaf(-5.f, x2, x4));
  v[1] = pa + pb;
  v[2] = pa - pb;
  v[3] = pc + pd;
  v[4] = pc - pd;
  v[5] = fmaf(4.f, x1, fmaf(-5.f, x3, x5));
}
__device__ __forceinline__ void gw4(const float g0, const float g1, const float g2, float* u) {
  const float s = g0 + g2, s4 = fmaf(4.f, g2, g0);
  u[0] = g0;
  u[1] = s + g1;
  u[2] = s - g1;
  u[3] = fmaf(2.f, g1, s4);
  u[4] = fmaf(-2.f, g1, s4);
  u[5] = g2;
}
__device__ __forceinline__ void aw4(const float a0, const float a1, const float a2, const float a3,
                                    const float a4, const float a5, float* y) {
  const float m0 = 0.25f * a0;
  const float m1 = (-1.f / 6.f) * a1, m2 = (-1.f / 6.f) * a2;
  const float m3 = (1.f / 24.f) * a3, m4 = (1.f / 24.f) * a4;
  const float sp = m1 + m2, sm = m1 - m2, tp = m3 + m4, tm = m3 - m4;
  y[0] = (m0 + sp) + tp;
  y[1] = fmaf(2.f, tm, sm);
  y[2] = fmaf(4.f, tp, sp);
  y[3] = fmaf(8.f, tm, sm) + a5;
}

// Diagnostic build (-DLEA_EXP_STAMPS, tools/build_variants.sh): s_memtime stamps around
// the loop's phases, per-wave cycle sums stored to ConvArgs::dbg (never in the real kernel)
#define LEA_STAMP(k) \
  do {               \
  } while (0)

template <int Q, int WC, int MTE, int NW, int OCC, int PV, bool CV>
__global__ __launch_bounds__(NW * 64, OCC) void conv3d_wino2_kernel(const ConvArgs a) {
  using C = Cfg2<Q, WC, MTE, NW, OCC, PV>;
  constexpr int F = C::F, NX = C::NX, NE = C::NE;
  constexpr int XSLOTS = C::XSLOTS;
  constexpr int XSLOTS_W = (XSLOTS + NW - 1) / NW;
  constexpr int WSLOTS = C::WSLOTS;
  constexpr int WSLOTS_W = (WSLOTS + NW - 1) / NW;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE + C::TS];
  float* const tv = smem + 2 * C::STAGE;  // PV: the chunk's transformed inputs
  const unsigned lds0 = lds_addr(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wr = wave / WC;
  // XCD-aware 1-D order (as the 1-D engine): each XCD walks a contiguous range of
  // (batch/cout-block, tile, depth-pair group), depth fastest.  A workgroup walks spw
  // consecutive depth pairs (items = pairs x chunks through one DMA pipeline): the
  // small-cin layers (2-4 chunks per pair) otherwise pay a cold first DMA and an
  // exposed epilogue per two planes
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int spw = a.spw > 0 ? a.spw : 1;
  const int ngz = (a.ndz + spw - 1) / spw;
  // cout block fastest (r03): the blocks of one (tile, depth group) run side by side on
  // one XCD and share its input through the L2 instead of each fetching it from HBM
  const int cob = lin % a.ncob;
  const int rest = lin / a.ncob;
  const int gz = rest % ngz;
  const int tile = (rest / ngz) % a.ntiles;
  const int b = rest / (ngz * a.ntiles);
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * C::TW;
  const int pz0 = gz * spw, npairs = min(spw, a.ndz - pz0);
  const int co0 = cob * C::COP;
  const int nchunks = a.cin / CIN_B;
  const int nitems = npairs * nchunks;
  const float* wp = a.wp + (long long)cob * nchunks * C::WS;
  const int HW = a.H * a.W;  // host checks D*H*W*4 < 2^32
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;

  // per-lane DMA pieces of this wave inside one channel volume: (plane, h, w) of each,
  // the (h, w) part once (hwo: byte offset in a plane, or OOB), the plane per pair
  unsigned hwo[XSLOTS_W];
  int pln[XSLOTS_W], wco[CV ? XSLOTS_W : 1];
#pragma unroll
  for (int t = 0; t < XSLOTS_W; ++t) {
    const int e = (wave + NW * t) * 64 + lane;
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
  // PV = 2: this wave's 16-byte pieces are block slot j16 of every channel it stages
  constexpr int PIECES16 = C::PIECES16;
  const int j16 = wave % PIECES16, e16 = 64 * j16 + lane;
  const bool ok16 = e16 < C::BLK16;  // the last piece is partial (exec-masked)
  unsigned hwo16 = 0xFFFFFFF0u, voff16 = 0xFFFFFFF0u;
  int pln16 = -1000;
  if constexpr (PV == 2) {
    const int p = e16 / (C::RH * (C::RWA / 4)), r = e16 - p * (C::RH * (C::RWA / 4));
    const int rr = r / (C::RWA / 4), blk = r - rr * (C::RWA / 4);
    const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;  // W % 4 == 0: a block is all in or all out
    if (ok16 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
      hwo16 = (unsigned)(h * a.W + w) * 4u;
      pln16 = p - 1;
    }
  }
  // PV = 4: this wave's 7 pieces of the item are P = wave + 4 k (k < 7) of the 28 (channel
  // P / 7, slot P % 7): their (plane, h, w) once, the plane per pair
  constexpr int K4 = C::H4 ? CIN_B * PIECES16 / NW : 1;
  unsigned hwo4[K4], voff4[K4];
  int pln4[K4];
  if constexpr (C::H4) {
    static_assert(CIN_B * PIECES16 % NW == 0, "whole pieces per wave");
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int e = 64 * ((wave + NW * k) % PIECES16) + lane;
      const int pl = e / (C::RH * (C::RWA / 4)), r = e - pl * (C::RH * (C::RWA / 4));
      const int rr = r / (C::RWA / 4), blk = r - rr * (C::RWA / 4);
      const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;  // W % 4 == 0: a block is all in or all out
      const bool ok = e < C::BLK16 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      hwo4[k] = ok ? (unsigned)(h * a.W + w) * 4u : 0xFFFFFFF0u;  // surplus lanes: zeros into the pad
      pln4[k] = ok ? pl - 1 : -1000;
      voff4[k] = 0xFFFFFFF0u;
    }
  }
  auto set_pair = [&](int d0) {  // DMA offsets of the pair at output planes d0, d0 + 1
    if constexpr (C::H4) {
#pragma unroll
      for (int k = 0; k < K4; ++k) {
        const int d = d0 + pln4[k];
        voff4[k] = (unsigned)d < (unsigned)a.D ? hwo4[k] + (unsigned)d * (unsigned)HW * 4u : 0xFFFFFFF0u;
      }
      return;
    }
    if constexpr (PV == 2) {
      const int d = d0 + pln16;
      voff16 = (hwo16 != 0xFFFFFFF0u && (unsigned)d < (unsigned)a.D) ? hwo16 + (unsigned)d * (unsigned)HW * 4u
                                                                      : 0xFFFFFFF0u;
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

  // H4 halo bases: channel c's = (c < cin1 ? xa : x2s) + c * cvol floats (x2s = x2's base cin1
  // channels down), byte addresses: a compare, select and add per piece, no 64-bit products
  const unsigned long long cvolb = (unsigned long long)HW * a.D * 4u;
  const unsigned long long xa = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned long long x2s =
      a.x2 ? (unsigned long long)(a.x2 + (long long)b * a.x2bs) - (unsigned long long)a.cin1 * cvolb : xa;
  unsigned long long coff4[K4];  // piece k's channel offset within the chunk
#pragma unroll
  for (int k = 0; k < K4; ++k) coff4[k] = (unsigned long long)((wave + NW * k) / PIECES16) * cvolb;
  // item = (chunk ch, depth pair pr) of this workgroup's walk (the caller's counters)
  auto issue = [&](int ch, int pr, float* st) {
    if (ch == 0) set_pair((pz0 + pr) * C::TD);
    const float* wsrc = wp + (long long)ch * C::WS;
    float* wdst = st + C::XS;
#pragma unroll
    for (int t = 0; t < WSLOTS_W; ++t) {
      const int j = wave + NW * t;
      if (j < WSLOTS)  // the last piece reads into the next chunk / the buffer's tail pad
        dma_dwordx4(wsrc + j * 256 + lane * 4, lds0 + 4 * (unsigned)(wdst - smem + j * 256));
    }
    const long long cvol = CV ? (long long)HW : (long long)HW * a.D;  // channel stride
    const unsigned crec = CV ? (unsigned)HW * 4u : nrec;
    if constexpr (C::H4) {
      static_assert(!CV, "16-byte halo: plain volumes only");
      const unsigned long long cbase = (unsigned long long)(ch * CIN_B) * cvolb;
#pragma unroll
      for (int k = 0; k < K4; ++k) {
        const int P = wave + NW * k, ci = P / PIECES16, j = P - ci * PIECES16;
        const int c = ch * CIN_B + ci;
        const unsigned long long base = (c < a.cin1 ? xa : x2s) + cbase + coff4[k];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, crec, 0x00020000);
        dma_dwordx4_buf(rs, voff4[k], lds0 + 4 * (unsigned)(st - smem + C::cb4(0) + ci * C::CS4 + j * 256));
      }
      return;
    }
    if constexpr (PV == 2) {
      static_assert(!CV || PV != 2, "16-byte halo: plain volumes only");
#pragma unroll
      for (int t = 0; t < CIN_B * PIECES16 / NW; ++t) {
        const int ci = (wave + NW * t) / PIECES16;  // (this wave's slot j16 of channel ci)
        const int c = ch * CIN_B + ci;
        const float* base = c < a.cin1 ? a.x + (long long)b * a.xbs + (long long)c * cvol
                                       : a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * cvol;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, crec, 0x00020000);
        const int cb = ci == 0 ? C::cb2(0) : ci == 1 ? C::cb2(1) : ci == 2 ? C::cb2(2) : C::cb2(3);
        if (ok16) dma_dwordx4_buf(rs, voff16, lds0 + 4 * (unsigned)(st - smem + cb + j16 * 256));
      }
      return;
    }
#pragma unroll
    for (int ci = 0; ci < CIN_B; ++ci) {
      const int c = ch * CIN_B + ci;
      // selects, not branches: the chunk's staging stays one basic block
      const float* base = c < a.cin1 ? a.x + (long long)b * a.xbs + (long long)c * cvol
                                     : a.x2 + (long long)b * a.x2bs + (long long)(c - a.cin1) * cvol;
      const unsigned n = c < a.cin ? crec : 0u;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
      const unsigned rmask = (CV && c >= a.cin1) ? 0xFFFFFFFFu : 0u;  // chunks never straddle cin1
#pragma unroll
      for (int t = 0; t < XSLOTS_W; ++t) {
        const int j = wave + NW * t;
        unsigned vo = voff[t];
        if constexpr (CV) vo = voff[t] ^ ((voff[t] ^ voffr[t]) & rmask);
        if (PV == 0 || j < XSLOTS) dma_dword(rs, vo, lds0 + 4 * (unsigned)(st - smem + ci * C::CIS + j * 64));
      }
    }
  };

  const int ci = lane >> 4, p = lane & 15;
  const int pq = p % Q, pr = p / Q;  // output group within the row, row within the lane group
  // tile row of the lane: PV = 4 interleaves the row sets (rows wr, wr + WR: bank map above)
  const int trow = C::H4 ? wr + C::WR * pr : wr * C::RPG + pr;
  const int xoff = C::H4 ? C::cb4(ci) + trow * C::RWA + 3 + F * pq : ci * C::CIS + trow * C::RW + F * pq;
  const int toff = ci * C::TCS + (wr * C::RPG + pr) * C::TRS + C::GS * pq;
  int woff[MTE];
#pragma unroll
  for (int m = 0; m < MTE; ++m) woff[m] = ci * C::COP + a_col(wc * MTE + m, ci, p, C::SWZ);

  // folded BN of this lane's couts, fetched now so the epilogue does not wait
  float sc[MTE][4], sh[MTE][4];
#pragma unroll
  for (int m = 0; m < MTE; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * (wc * MTE + m) + 4 * ci + r;
      const bool cv = co < a.cout;
      sc[m][r] = (cv && a.scale) ? a.scale[co] : 1.f;
      sh[m][r] = (cv && a.shift) ? a.shift[co] : 0.f;
    }

  f32x4 acc[NX][NE][MTE];
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int e = 0; e < NE; ++e)
#pragma unroll
      for (int m = 0; m < MTE; ++m) acc[x][e][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue of one depth pair (output planes d0, d0 + 1): A_W^T per D point, A_D^T
  // (with G_D's 1/2 factors), folded BN, ReLU, residual; the lane stores 4 outputs
  // along W for each of the two planes
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int w = w0 + F * pq;
  const int h = h0 + trow;
  const int nv = min(F, a.W - w);  // valid outputs of this group
  const bool ebuf = a.flags & kEpiBuf;
  constexpr int NST = MTE * 4 * C::TD;  // buffer stores per epilogue
  // the buffer-addressed form (wino_common.h): residual loads all issued first, every
  // lane the same NST float4 stores (invalid ones out of range: dropped)
  const int nco = min(C::COP, a.cout - co0);
  const __amdgpu_buffer_rsrc_t yrs = block_rsrc(a.y + (long long)b * a.ybs + (long long)co0 * DHW, nco * DHW * 4);
  const __amdgpu_buffer_rsrc_t rrs =
      block_rsrc((resid ? a.res : a.y) + (long long)b * (resid ? a.rbs : a.ybs) + (long long)co0 * DHW, nco * DHW * 4);
  auto epilogue_buf = [&](int d0) {
    const bool lv = h < a.H && w < a.W;
    unsigned off[MTE][4][C::TD];
#pragma unroll
    for (int m = 0; m < MTE; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < C::TD; ++t) {
          const int cr = 16 * (wc * MTE + m) + 4 * ci + r, d = d0 + t;
          off[m][r][t] = (lv && cr < nco && d < a.D)
                             ? (unsigned)(cr * DHW + (long long)d * HW + h * a.W + w) * 4u
                             : kEpiOob;
        }
    f32x4 rv[MTE][4][C::TD];
    if (resid) {
#pragma unroll
      for (int m = 0; m < MTE; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t = 0; t < C::TD; ++t) rv[m][r][t] = buf_load4(rrs, off[m][r][t]);
    }
#pragma unroll
    for (int m = 0; m < MTE; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float n[NE][F];
#pragma unroll
        for (int e = 0; e < NE; ++e)
          aw4(acc[0][e][m][r], acc[1][e][m][r], acc[2][e][m][r], acc[3][e][m][r], acc[4][e][m][r],
              acc[5][e][m][r], n[e]);
#pragma unroll
        for (int t = 0; t < C::TD; ++t) {
          f32x4 y;
#pragma unroll
          for (int j = 0; j < F; ++j) {
            const float s = t == 0 ? 0.5f * (n[1][j] + n[2][j]) : 0.5f * (n[1][j] - n[2][j]);
            float v = t == 0 ? n[0][j] + s : s - n[3][j];
            v = v * sc[m][r] + sh[m][r];
            if (relu) v = fmaxf(v, 0.f);
            y[j] = resid ? v + rv[m][r][t][j] : v;
          }
          buf_store4(yrs, off[m][r][t], y);
        }
      }
  };
  auto epilogue = [&](int d0) {
    if (h >= a.H || w >= a.W) return;
#pragma unroll
    for (int m = 0; m < MTE; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + 16 * (wc * MTE + m) + 4 * ci + r;
        if (co >= a.cout) continue;
        float n[NE][F];
#pragma unroll
        for (int e = 0; e < NE; ++e)
          aw4(acc[0][e][m][r], acc[1][e][m][r], acc[2][e][m][r], acc[3][e][m][r], acc[4][e][m][r],
              acc[5][e][m][r], n[e]);
#pragma unroll
        for (int t = 0; t < C::TD; ++t) {
          const int d = d0 + t;
          if (d >= a.D) break;
          float y[F];
#pragma unroll
          for (int j = 0; j < F; ++j) {
            const float s = t == 0 ? 0.5f * (n[1][j] + n[2][j]) : 0.5f * (n[1][j] - n[2][j]);
            y[j] = t == 0 ? n[0][j] + s : s - n[3][j];
            y[j] = y[j] * sc[m][r] + sh[m][r];
            if (relu) y[j] = fmaxf(y[j], 0.f);
          }
          const long long o = (long long)co * DHW + (long long)d * HW + (long long)h * a.W + w;
          float* yp = a.y + (long long)b * a.ybs + o;
          const float* rp = a.res + (long long)b * a.rbs + o;
          const bool vec = nv == F &&
              ((reinterpret_cast<uintptr_t>(yp) | (resid ? reinterpret_cast<uintptr_t>(rp) : 0)) & 15) == 0;
          if (vec) {
            if (resid) {
              const float4 rv = *reinterpret_cast<const float4*>(rp);
              y[0] += rv.x;
              y[1] += rv.y;
              y[2] += rv.z;
              y[3] += rv.w;
            }
            *reinterpret_cast<float4*>(yp) = make_float4(y[0], y[1], y[2], y[3]);
          } else {
#pragma unroll
            for (int j = 0; j < F; ++j)
              if (j < nv) {
                if (resid) y[j] += rp[j];
                yp[j] = y[j];
              }
          }
        }
      }
  };

  issue(0, 0, smem);
  LEA_STAMP(2);
  int ich = 0, ipr = 0;  // item it = (chunk, depth pair)
  for (int it = 0; it < nitems; ++it) {
    const int ch = ich;
    const bool wrap = ich + 1 == nchunks;  // item it + 1 starts the next pair
    wait_item<NST>(ebuf && ch == 0 && it > 0);  // this wave's pieces of item it landed
    LEA_STAMP(0);
    __syncthreads();  // ... and everyone's; item it-1's stage is free
    LEA_STAMP(1);
    if (it + 1 < nitems) issue(wrap ? 0 : ich + 1, wrap ? ipr + 1 : ipr, smem + ((it + 1) & 1) * C::STAGE);
    LEA_STAMP(2);
    const float* xs = smem + (it & 1) * C::STAGE;
    const float* ws = xs + C::XS;
    if constexpr (C::VPASS) {
      // the workgroup transforms the chunk's halo once: unit (ci, row, group) reads
      // 4 planes x 6 inputs and writes its 24 V values
      static_assert(PV == 2 || (C::RW % 64 == 34 && C::CIS % 64 == 32 && C::RH % 2 == 0 && Q == 8),
                    "transform pass bank map");
      static_assert(PV != 2 || (Q == 8 && CIN_B == 4), "transform pass bank map (16-byte halo)");
      for (int u = tid; u < C::NUNIT; u += NW * 64) {
        // PV = 1: 32 consecutive units = 8 groups x 2 rows x 2 channels: the b64 reads'
        // dword offsets 4 g + {0, RW, CIS, RW + CIS} cover the 64 banks once.
        // PV = 2: 8 groups x 4 channels of one row: 4 g + CB2(c) + 3 covers them (Cfg2)
        int g, r, c, xo;
        if constexpr (PV == 2) {
          g = u % Q;
          c = (u / Q) % CIN_B;
          r = u / (Q * CIN_B);
          const int cb = c == 0 ? C::cb2(0) : c == 1 ? C::cb2(1) : c == 2 ? C::cb2(2) : C::cb2(3);
          xo = cb + r * C::RWA + 3 + F * g;
        } else {
          g = u % Q;
          const int t = u / Q;
          const int rl = t & 1, cl = (t >> 1) & 1, t2 = t >> 2;
          r = 2 * (t2 % (C::RH / 2)) + rl;
          c = 2 * (t2 / (C::RH / 2)) + cl;
          xo = c * C::CIS + r * C::RW + F * g;
        }
        float bw[C::PLANES][NX];
#pragma unroll
        for (int pl = 0; pl < C::PLANES; ++pl) {
          const float* sp = xs + xo + pl * (PV == 2 ? C::PLANEA : C::PLANE);
          const float2 a0 = *reinterpret_cast<const float2*>(sp);
          const float2 a1 = *reinterpret_cast<const float2*>(sp + 2);
          const float2 a2 = *reinterpret_cast<const float2*>(sp + 4);
          bw4(a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, bw[pl]);
        }
        float v[NE][NX];
#pragma unroll
        for (int x = 0; x < NX; ++x) {
          v[0][x] = bw[0][x] - bw[2][x];
          v[1][x] = bw[1][x] + bw[2][x];
          v[2][x] = bw[2][x] - bw[1][x];
          v[3][x] = bw[1][x] - bw[3][x];
        }
        float4* tp = reinterpret_cast<float4*>(tv + c * C::TCS + r * C::TRS + C::GS * g);
        const float* vf = &v[0][0];
#pragma unroll
        for (int k = 0; k < 6; ++k) tp[k] = make_float4(vf[4 * k], vf[4 * k + 1], vf[4 * k + 2], vf[4 * k + 3]);
      }
      LEA_STAMP(3);
      __syncthreads();
      LEA_STAMP(4);
    }
    // one kh step: the inputs (4 planes x 6 staged values as float2s, or the 24
    // pre-transformed V as float4s) and the 9 g values (kd, kw) per cout tile
    struct Raw {
      float2 x2[(C::VPASS || C::H4) ? 1 : C::PLANES][3];
      float4 v4[C::VPASS ? 6 : 1];
      float4 h4[C::H4 ? C::PLANES : 1][2];  // PV = 4: inputs 0..7 of each plane (6, 7 unused)
      float g[9][MTE];
    };
    constexpr int XPL = C::H4 ? C::PLANEA : C::PLANE, XRW = C::H4 ? C::RWA : C::RW;
    auto load_step = [&](int kh, Raw& o) {
      if constexpr (C::VPASS) {
        const float4* tp = reinterpret_cast<const float4*>(tv + toff + kh * C::TRS);
#pragma unroll
        for (int k = 0; k < 6; ++k) o.v4[k] = tp[k];
      } else {
#pragma unroll
        for (int pl = 0; pl < C::PLANES; ++pl) {
          const float* sp = xs + xoff + pl * XPL + kh * XRW;
          if constexpr (C::H4) {
            o.h4[pl][0] = *reinterpret_cast<const float4*>(sp);
            // volatile keeps the whole 16-byte read (inputs 6, 7 are unused: as a plain load
            // the compiler narrows it to 8 bytes and pairs those into ds_read2_b64)
            typedef const volatile __attribute__((address_space(3))) f32x4 lds_f32x4;
            const f32x4 hi = *(lds_f32x4*)(sp + 4);
            o.h4[pl][1] = make_float4(hi[0], hi[1], hi[2], hi[3]);
            continue;
          }
#pragma unroll
          for (int q = 0; q < 3; ++q)
            o.x2[pl][q] = *reinterpret_cast<const float2*>(sp + 2 * q);
        }
      }
#pragma unroll
      for (int kd = 0; kd < 3; ++kd)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int m = 0; m < MTE; ++m)
            o.g[kd * 3 + kw][m] = ws[((kd * 3 + kh) * 3 + kw) * CIN_B * C::COP + woff[m]];
    };
    struct Xf {
      float v[NX][NE];
      float u[NX][NE][MTE];
    };
    auto xform = [&](const Raw& o, Xf& T) {
      if constexpr (C::VPASS) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const float e4[4] = {o.v4[k].x, o.v4[k].y, o.v4[k].z, o.v4[k].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) T.v[(4 * k + i) % NX][(4 * k + i) / NX] = e4[i];
        }
      } else {
        float bw[C::PLANES][NX];
#pragma unroll
        for (int pl = 0; pl < C::PLANES; ++pl)
        {
          if constexpr (C::H4)
            bw4(o.h4[pl][0].x, o.h4[pl][0].y, o.h4[pl][0].z, o.h4[pl][0].w, o.h4[pl][1].x, o.h4[pl][1].y, bw[pl]);
          else
            bw4(o.x2[pl][0].x, o.x2[pl][0].y, o.x2[pl][1].x, o.x2[pl][1].y, o.x2[pl][2].x, o.x2[pl][2].y, bw[pl]);
        }
#pragma unroll
        for (int x = 0; x < NX; ++x) {
          T.v[x][0] = bw[0][x] - bw[2][x];
          T.v[x][1] = bw[1][x] + bw[2][x];
          T.v[x][2] = bw[2][x] - bw[1][x];
          T.v[x][3] = bw[1][x] - bw[3][x];
        }
      }
#pragma unroll
      for (int m = 0; m < MTE; ++m) {
        float uw[3][NX];
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) gw4(o.g[kd * 3][m], o.g[kd * 3 + 1][m], o.g[kd * 3 + 2][m], uw[kd]);
#pragma unroll
        for (int x = 0; x < NX; ++x) {
          const float s = uw[0][x] + uw[2][x];
          T.u[x][0][m] = uw[0][x];
          T.u[x][1][m] = s + uw[1][x];
          T.u[x][2][m] = s - uw[1][x];
          T.u[x][3][m] = uw[2][x];
        }
      }
    };
    auto mfmas = [&](const Xf& T) {
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int e = 0; e < NE; ++e)
#pragma unroll
          for (int m = 0; m < MTE; ++m)
            acc[x][e][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(T.u[x][e][m], T.v[x][e], acc[x][e][m], 0, 0, 0);
    };
    // 3 kh steps: LDS reads two steps ahead, transforms one step ahead
    Raw raw[2];
    Xf xf[2];
    // scheduler hint: interleave the step's LDS reads / VALU transforms with the MFMAs
    // (same-box sweep r02: -1 to -4 % per layer; iglp_opt(1) and s_setprio gained less)
    if constexpr (PV == 5) {
      // fenced schedule (r04; L1 16 -> 16 cells 46.1 -> 44.2 us same box): at most one step's inputs in flight beside one
      // step's operands -- load(k + 1) | mfmas(k) | xform(k + 1) -- so the live set
      // (96 accumulators + 48 operands + 41 inputs) leaves the scheduler room; sched_barrier
      // keeps each step's LDS reads above the previous step's MFMAs
      load_step(0, raw[0]);
      xform(raw[0], xf[0]);
      load_step(1, raw[1]);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(xf[0]);
      __builtin_amdgcn_sched_barrier(0);
      xform(raw[1], xf[1]);
      load_step(2, raw[0]);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(xf[1]);
      __builtin_amdgcn_sched_barrier(0);
      xform(raw[0], xf[0]);
      mfmas(xf[0]);
    } else {
    __builtin_amdgcn_iglp_opt(0);
    load_step(0, raw[0]);
    load_step(1, raw[1]);
    xform(raw[0], xf[0]);
    load_step(2, raw[0]);
    xform(raw[1], xf[1]);
    mfmas(xf[0]);
    xform(raw[0], xf[0]);
    mfmas(xf[1]);
    mfmas(xf[0]);
    }
    LEA_STAMP(5);
    if (ch == nchunks - 1) {  // the pair's last chunk: its epilogue, fresh accumulators
      if (ebuf)
        epilogue_buf((pz0 + ipr) * C::TD);
      else
        epilogue((pz0 + ipr) * C::TD);
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int e = 0; e < NE; ++e)
#pragma unroll
          for (int m = 0; m < MTE; ++m) acc[x][e][m] = f32x4{0.f, 0.f, 0.f, 0.f};
      LEA_STAMP(6);
    }
    ich = wrap ? 0 : ich + 1;
    ipr += wrap;
  }
}


// ------------------------------------------------------------------------------------
// PV = 3 (r03): the transform-pass tile (Q = 8, two 16-row cout tiles x two row sets,
// 16-byte halo) as a one-barrier pipeline.  Item i = (depth pair, 4-channel chunk):
//   top      this wave's halo(i + 1) pieces and weight loads g(i) have landed (vmcnt),
//            barrier: V(i) in tv[i & 1] is complete, halo(i + 1) has landed for all
//   steps(i) V from tv[i & 1], U from g(i) in registers, 72 MFMAs per wave; interleaved
//            with V-pass(i + 1): halo[(i + 1) & 1] -> tv[(i + 1) & 1] (last read by
//            steps(i - 1), before the barrier)
//   halo(i + 2) -> halo[i & 1] (read by V-pass(i), before the barrier), issued after
//            step 0's transforms so the compiler's wait for g(i) never covers it
//   g(i + 1) -> registers after the last U of item i (7 dwordx4 per lane)
// The weights never touch LDS: each lane loads its (cout, channel)'s 27 taps of a chunk
// from the per-lane copy (16-byte slices) lea_conv3d_wino_pack_weights appends for 32-cout blocks.
// Ablations of the two-barrier tile (tools/wino2_ablate.sh, conv1/2: 858 us) put its
// V-pass at 118 us and the weight DMA at 49 us, serialised with the MFMAs.
constexpr int kGL = 28;   // floats per lane and chunk in the per-lane weights (27 taps + pad)
constexpr int kGLW = 56;  // the same with G_W applied by the packer (r06): [kh][kd][6 W points] + pad

// WPRE (r06, lea_conv3d_wino2p_set_wpre): the per-lane weights arrive with the W transform
// already applied (G_W g per kernel row, the packer's gw4 -- the same fp32 operations, so the
// same bits), 54 floats per (cout, channel) instead of 27 raw taps: the step transform is the
// D part alone (18 VALU instead of 36), for 7 more 16-byte loads per lane and item
template <bool WPRE>
__global__ __launch_bounds__(256, 2) void conv3d_wino2p_kernel(const ConvArgs a) {
  using C = Cfg2<8, 2, 1, 4, 2, 2>;  // the PV = 2 tile's geometry and maps (tv, V-pass banks)
  constexpr int Q = 8, WC = 2, F = 4, NX = 6, NE = 4, TD = 2;
  // halo channels 1024 floats apart (the PV = 2 map's bases mod 64): every lane of the 4
  // pieces per channel, the partial last one too, writes inside its channel's region, so
  // the pieces need no exec mask and the loop body stays one basic block
  constexpr int CB0 = 1, CB1 = CB0 + 1024 + 2, CB2 = CB1 + 1024 + 30, CB3 = CB2 + 1024 + 2;
  static_assert(CB1 % 64 == 3 && CB2 % 64 == 33 && CB3 % 64 == 35, "V-pass bank map");
  constexpr int XS = (CB3 + 1024 + 3) / 4 * 4, TS = C::TS;
  static_assert(C::NUNIT == 3 * 64 && C::BLK16 <= 4 * 64, "tile geometry");
  static_assert((2 * XS + 2 * TS) * 4 * 2 <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) float smem[2 * XS + 2 * TS];
  const unsigned lds0 = lds_addr(smem);
  float* const halo = smem;            // halo[k] = smem + k * XS
  float* const tvb = smem + 2 * XS;    // tv[k] = tvb + k * TS

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wr = wave / WC;
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int spw = a.spw > 0 ? a.spw : 1;
  const int ngz = (a.ndz + spw - 1) / spw;
  const int cob = lin % a.ncob;
  const int rest = lin / a.ncob;
  const int gz = rest % ngz;
  const int tile = (rest / ngz) % a.ntiles;
  const int b = rest / (ngz * a.ntiles);
  const int h0 = (tile / a.tiles_w) * C::TH;
  const int w0 = (tile % a.tiles_w) * C::TW;
  const int pz0 = gz * spw, npairs = min(spw, a.ndz - pz0);
  const int co0 = cob * C::COP;
  const int nchunks = a.cin / CIN_B;
  const int nitems = npairs * nchunks;
  const int HW = a.H * a.W;
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;
  const long long cvol = (long long)HW * a.D;
  // per-lane weights (slice-major, see pack_wino_lane_kernel): after the staged copy (ncob * nchunks * WS floats + 256 pad);
  // the W-transformed copy (WPRE) after the raw one
  constexpr int GL = WPRE ? kGLW : kGL;
  const float* wl = a.wp + (long long)a.ncob * nchunks * C::WS + 256 +
                    (WPRE ? (long long)a.ncob * nchunks * WC * 64 * kGL : 0LL) +
                    ((long long)cob * nchunks * WC + wc) * 64 * GL + lane * 4;

  // 16-byte halo pieces: block slot j16 = wave of every channel (4 per wave per item);
  // lanes past the halo (e16 >= BLK16) read out of range: zeros into the channel's pad
  const int e16 = 64 * wave + lane;
  const bool ok16 = e16 < C::BLK16;
  unsigned hwo16 = 0xFFFFFFF0u;
  int pln16 = -1000;
  {
    const int p = e16 / (C::RH * (C::RWA / 4)), r = e16 - p * (C::RH * (C::RWA / 4));
    const int rr = r / (C::RWA / 4), blk = r - rr * (C::RWA / 4);
    const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;
    if (ok16 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
      hwo16 = (unsigned)(h * a.W + w) * 4u;
      pln16 = p - 1;
    }
  }
  // channel c's base = (c < cin1 ? xa : x2s) + c * cvol floats, x2s = x2's base cin1 channels down
  // (byte addresses: one compare, select and add per channel instead of two 64-bit products)
  const unsigned long long cvolb = (unsigned long long)cvol * 4u;
  const unsigned long long xa = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned long long x2s =
      a.x2 ? (unsigned long long)(a.x2 + (long long)b * a.x2bs) - (unsigned long long)a.cin1 * cvolb : xa;
  // item = (chunk ch, depth pair pr) of this workgroup's walk (counters, no divisions in the loop)
  auto issue_halo = [&](int ch, int pr, int buf) {  // branch-free: every lane, every channel
    const int d = (pz0 + pr) * TD + pln16;
    const unsigned vo = (hwo16 != 0xFFFFFFF0u && (unsigned)d < (unsigned)a.D)
                            ? hwo16 + (unsigned)d * (unsigned)HW * 4u : 0xFFFFFFF0u;
    const unsigned long long cb = (unsigned long long)(ch * CIN_B) * cvolb;
#pragma unroll
    for (int ci = 0; ci < CIN_B; ++ci) {
      const int c = ch * CIN_B + ci;
      const unsigned long long base = (c < a.cin1 ? xa : x2s) + cb + (unsigned long long)ci * cvolb;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nrec, 0x00020000);
      constexpr int cbs[4] = {CB0, CB1, CB2, CB3};
      dma_dwordx4_buf(rs, vo, lds0 + 4 * (unsigned)(buf * XS + cbs[ci] + wave * 256));
    }
  };
  float4 gw[GL / 4];  // this lane's taps of the current chunk: [kh][kd][kw] (WPRE: [kh][kd][W point])
  auto load_g = [&](int ch) {
    const float4* src = reinterpret_cast<const float4*>(wl + (long long)ch * WC * 64 * GL);
#pragma unroll
    for (int k = 0; k < GL / 4; ++k) gw[k] = src[64 * k];
  };
  // V-pass of one item: unit u = (group g, channel c, halo row r), as PV = 2; branch-free:
  // the fourth wave repeats the first wave's units and stores the same values
  const int vu = tid % C::NUNIT;
  const int vg = vu % Q, vc = (vu / Q) % CIN_B, vr = vu / (Q * CIN_B);
  const int vxo = (vc == 0 ? CB0 : vc == 1 ? CB1 : vc == 2 ? CB2 : CB3) + vr * C::RWA + 3 + F * vg;
  const int vto = vc * C::TCS + vr * C::TRS + C::GS * vg;
  auto vpass = [&](int buf) {
    const float* xs = halo + buf * XS;
    float* tv = tvb + buf * TS;
    {
      const int g = vg;
      (void)g;
      const float* sp0 = xs + vxo;
      float bw[C::PLANES][NX];
#pragma unroll
      for (int pl = 0; pl < C::PLANES; ++pl) {
        const float* sp = sp0 + pl * C::PLANEA;
        const float2 a0 = *reinterpret_cast<const float2*>(sp);
        const float2 a1 = *reinterpret_cast<const float2*>(sp + 2);
        const float2 a2 = *reinterpret_cast<const float2*>(sp + 4);
        bw4(a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, bw[pl]);
      }
      float v[NE][NX];
#pragma unroll
      for (int x = 0; x < NX; ++x) {
        v[0][x] = bw[0][x] - bw[2][x];
        v[1][x] = bw[1][x] + bw[2][x];
        v[2][x] = bw[2][x] - bw[1][x];
        v[3][x] = bw[1][x] - bw[3][x];
      }
      float4* tp = reinterpret_cast<float4*>(tv + vto);
      const float* vf = &v[0][0];
#pragma unroll
      for (int k = 0; k < 6; ++k) tp[k] = make_float4(vf[4 * k], vf[4 * k + 1], vf[4 * k + 2], vf[4 * k + 3]);
    }
  };

  const int ci = lane >> 4, p = lane & 15;
  const int pq = p % Q, pr = p / Q;
  const int toff = ci * C::TCS + (wr * C::RPG + pr) * C::TRS + C::GS * pq;
  float sc[4], sh[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + 16 * wc + 4 * ci + r;
    const bool cv = co < a.cout;
    sc[r] = (cv && a.scale) ? a.scale[co] : 1.f;
    sh[r] = (cv && a.shift) ? a.shift[co] : 0.f;
  }
  f32x4 acc[NX][NE];
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[x][e] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int w = w0 + F * pq;
  const int h = h0 + wr * C::RPG + pr;
  constexpr int NST = 4 * TD;
  const int nco = min(C::COP, a.cout - co0);
  const __amdgpu_buffer_rsrc_t yrs = block_rsrc(a.y + (long long)b * a.ybs + (long long)co0 * DHW, nco * DHW * 4);
  const __amdgpu_buffer_rsrc_t rrs =
      block_rsrc((resid ? a.res : a.y) + (long long)b * (resid ? a.rbs : a.ybs) + (long long)co0 * DHW, nco * DHW * 4);
  auto epilogue = [&](int d0) {  // the buffer-addressed epilogue of conv3d_wino2_kernel
    const bool lv = h < a.H && w < a.W;
    unsigned off[4][TD];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < TD; ++t) {
        const int cr = 16 * wc + 4 * ci + r, d = d0 + t;
        off[r][t] = (lv && cr < nco && d < a.D) ? (unsigned)(cr * DHW + (long long)d * HW + h * a.W + w) * 4u
                                                : kEpiOob;
      }
    f32x4 rv[4][TD];
    if (resid) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < TD; ++t) rv[r][t] = buf_load4(rrs, off[r][t]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float n[NE][F];
#pragma unroll
      for (int e = 0; e < NE; ++e)
        aw4(acc[0][e][r], acc[1][e][r], acc[2][e][r], acc[3][e][r], acc[4][e][r], acc[5][e][r], n[e]);
#pragma unroll
      for (int t = 0; t < TD; ++t) {
        f32x4 y;
#pragma unroll
        for (int j = 0; j < F; ++j) {
          const float s = t == 0 ? 0.5f * (n[1][j] + n[2][j]) : 0.5f * (n[1][j] - n[2][j]);
          float v = t == 0 ? n[0][j] + s : s - n[3][j];
          v = v * sc[r] + sh[r];
          if (relu) v = fmaxf(v, 0.f);
          y[j] = resid ? v + rv[r][t][j] : v;
        }
        buf_store4(yrs, off[r][t], y);
      }
    }
  };

  // prologue: halo(0), g(0), halo(1); V(0)
  issue_halo(0, 0, 0);
  load_g(0);
  if (nitems > 1) {
    issue_halo(1 % nchunks, 1 / nchunks, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // all but halo(1)'s four pieces
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  vpass(0);
  bool after_epi = false;
  int ich = 0, ipr = 0;  // item it = (chunk, depth pair)
  // item min(it + 2, nitems - 1), the halo the loop issues
  int hch = min(2, nitems - 1) % nchunks, hpr = min(2, nitems - 1) / nchunks;
  for (int it = 0; it < nitems; ++it) {
    // halo(it + 1) and g(it) landed (only an epilogue's stores may stay in flight)
    if (after_epi)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* tv = tvb + (it & 1) * TS;
    struct Raw {
      float4 v4[6];
    };
    auto load_step = [&](int kh, Raw& o) {
      const float4* tp = reinterpret_cast<const float4*>(tv + toff + kh * C::TRS);
#pragma unroll
      for (int k = 0; k < 6; ++k) o.v4[k] = tp[k];
    };
    struct Xf {
      float v[NX][NE];
      float u[NX][NE];
    };
    auto xform = [&](int kh, const Raw& o, Xf& T) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float e4[4] = {o.v4[k].x, o.v4[k].y, o.v4[k].z, o.v4[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) T.v[(4 * k + i) % NX][(4 * k + i) / NX] = e4[i];
      }
      float uw[3][NX];
      if constexpr (WPRE) {
        const float* g = reinterpret_cast<const float*>(gw) + kh * 18;
#pragma unroll
        for (int kd = 0; kd < 3; ++kd)
#pragma unroll
          for (int x = 0; x < NX; ++x) uw[kd][x] = g[kd * 6 + x];
      } else {
        const float* g = reinterpret_cast<const float*>(gw) + kh * 9;
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) gw4(g[kd * 3], g[kd * 3 + 1], g[kd * 3 + 2], uw[kd]);
      }
#pragma unroll
      for (int x = 0; x < NX; ++x) {
        const float s = uw[0][x] + uw[2][x];
        T.u[x][0] = uw[0][x];
        T.u[x][1] = s + uw[1][x];
        T.u[x][2] = s - uw[1][x];
        T.u[x][3] = uw[2][x];
      }
    };
    auto mfmas = [&](const Xf& T) {
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int e = 0; e < NE; ++e)
          acc[x][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(T.u[x][e], T.v[x][e], acc[x][e], 0, 0, 0);
    };
    Raw raw[2];
    Xf xf[2];
    __builtin_amdgcn_iglp_opt(0);
    load_step(0, raw[0]);
    load_step(1, raw[1]);
    xform(0, raw[0], xf[0]);
    // halo(it + 2) into the buffer V-pass(it) read (after g(it)'s first use: see above);
    // past the last item the DMA / V-pass / loads repeat the last one (nothing reads
    // them), so the body is one basic block the scheduler can interleave with the MFMAs
    issue_halo(hch, hpr, it & 1);
    load_step(2, raw[0]);
    xform(1, raw[1], xf[1]);
    mfmas(xf[0]);
    vpass((it + 1) & 1);
    xform(2, raw[0], xf[0]);
    // g(min(it + 1, nitems - 1)): the last item's chunk is nchunks - 1 = ich
    load_g(it + 1 < nitems ? (ich + 1 == nchunks ? 0 : ich + 1) : ich);
    mfmas(xf[1]);
    mfmas(xf[0]);
    after_epi = false;
    if (ich == nchunks - 1) {
      epilogue((pz0 + ipr) * TD);
      after_epi = true;
#pragma unroll
      for (int x = 0; x < NX; ++x)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[x][e] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (++ich == nchunks) {
      ich = 0;
      ++ipr;
    }
    if (it + 3 < nitems && ++hch == nchunks) {
      hch = 0;
      ++hpr;
    }
  }
  // the last iterations' repeated DMA still writes this workgroup's LDS: let it land
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// per-lane weights of the pipelined tile, appended after the staged copy: per (cout block
// of 32, chunk, cout tile wc) seven 256-float slices; slice s holds, per lane = 16 ci + n,
// taps 4 s .. 4 s + 3 of [kh][kd][kw] (27 taps, then one zero) of cout 32 cb + 16 wc + n
// and input channel 4 chunk + ci as one 16-byte word: a wave's float4 load of a slice is
// one contiguous KB (r04; the lane-major form, 112 B between lanes, made each of the seven
// loads touch 56 cache lines instead of 8)
__global__ void pack_wino_lane_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                      int nchunks, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int e = (int)(q % (64 * kGL)); q /= 64 * kGL;
    const int k = (e / 256) * 4 + (e & 3), ln = (e & 255) >> 2;
    const int wc = (int)(q % 2); q /= 2;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int co = cb * 32 + 16 * wc + (ln & 15), c = ch * CIN_B + (ln >> 4);
    const int kh = k / 9, kd = (k % 9) / 3, kw = k % 3;
    out[i] = (k < 27 && co < cout && c < cin) ? w[(((long long)co * cin + c) * 9 + kd * 3 + kh) * 3 + kw] : 0.f;
  }
}

// the W-transformed copy (WPRE), after the raw one: slice s holds entries 4 s .. 4 s + 3 of
// [kh][kd][W point] (G_W g of each kernel row, gw4's operations: the kernel's own bits), then two zeros
__global__ void pack_wino_lane_wpre_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                           int nchunks, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int e = (int)(q % (64 * kGLW)); q /= 64 * kGLW;
    const int k = (e / 256) * 4 + (e & 3), ln = (e & 255) >> 2;
    const int wc = (int)(q % 2); q /= 2;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int co = cb * 32 + 16 * wc + (ln & 15), c = ch * CIN_B + (ln >> 4);
    float v = 0.f;
    if (k < 54 && co < cout && c < cin) {
      const int kh = k / 18, kd = (k % 18) / 6, x = k % 6;
      const float* g = w + (((long long)co * cin + c) * 9 + kd * 3 + kh) * 3;
      float u[6];
      gw4(g[0], g[1], g[2], u);
      v = u[x];
    }
    out[i] = v;
  }
}

long long lane_raw_floats(int cout, int cin) { return (long long)((cout + 31) / 32) * (cin / CIN_B) * 2 * 64 * kGL; }

long long lane_weights_floats(int cout, int cin) {
  return lane_raw_floats(cout, cin) + (long long)((cout + 31) / 32) * (cin / CIN_B) * 2 * 64 * kGLW;
}


thread_local char g_name2[96];


#define LEA_WINO2_DBG
#define LEA_WINO2_CASE(Q, WC, MTE, NW, OCC, PV, CV)                                                \
  if (p.q == Q && p.wc == WC && p.mte == MTE && p.nw == NW && p.occ == OCC && p.pv == PV) {        \
    using C_ = Cfg2<Q, WC, MTE, NW, OCC, PV>;                                                      \
    a.ncob = (a.cout + C_::COP - 1) / C_::COP;                                                     \
    a.tiles_w = (a.W + C_::TW - 1) / C_::TW;                                                       \
    a.ntiles = a.tiles_w * ((a.H + C_::TH - 1) / C_::TH);                                          \
    a.ndz = (a.D + C_::TD - 1) / C_::TD;                                                           \
    a.spw = std::max(1, std::min(p.spw > 0 ? p.spw : auto_walk(a, B, C_::WG_PER_CU), a.ndz));    \
    const long long n_ = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;         \
    LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino2): grid too large");                          \
    a.nblk = (int)n_;                                                                              \
    LEA_WINO2_DBG                                                                                  \
    conv3d_wino2_kernel<Q, WC, MTE, NW, OCC, PV, CV><<<dim3((unsigned)n_), NW * 64, 0, st>>>(a);   \
    return launch_status("lea_conv3d(wino2)");                                                    \
  }
#define LEA_WINO2_TILES(CV)                                                                        \
  LEA_WINO2_CASE(8, 1, 1, 4, 2, 0, CV) LEA_WINO2_CASE(8, 2, 1, 4, 2, 0, CV)                        \
  LEA_WINO2_CASE(8, 2, 1, 8, 2, 0, CV) LEA_WINO2_CASE(8, 1, 2, 4, 1, 0, CV)                        \
  LEA_WINO2_CASE(16, 1, 1, 4, 2, 0, CV) LEA_WINO2_CASE(16, 2, 1, 8, 2, 0, CV)                      \
  LEA_WINO2_CASE(16, 1, 2, 4, 1, 0, CV) LEA_WINO2_CASE(8, 2, 1, 4, 2, 1, CV)                       \
  LEA_WINO2_CASE(8, 2, 1, 8, 2, 1, CV) LEA_WINO2_CASE(8, 1, 2, 4, 1, 1, CV)

int run2(const Plan2& p, ConvArgs a, int B, hipStream_t st, bool cv) {
  if (cv) {
    LEA_WINO2_TILES(true)
  } else {
    LEA_WINO2_TILES(false)
    LEA_WINO2_CASE(8, 2, 1, 4, 2, 2, false)
    LEA_WINO2_CASE(8, 1, 1, 4, 2, 4, false)
    LEA_WINO2_CASE(8, 1, 1, 4, 2, 5, false)
    if (p.q == 8 && p.wc == 2 && p.mte == 1 && p.nw == 4 && p.occ == 2 && p.pv == 3) {
      if (g_w44) return run44(a, B, p.spw, st);  // F(4,3) x F(4,3) on the same layers (r06)
      using C_ = Cfg2<8, 2, 1, 4, 2, 2>;
      a.ncob = (a.cout + C_::COP - 1) / C_::COP;
      a.tiles_w = (a.W + C_::TW - 1) / C_::TW;
      a.ntiles = a.tiles_w * ((a.H + C_::TH - 1) / C_::TH);
      a.ndz = (a.D + C_::TD - 1) / C_::TD;
      a.spw = std::max(1, std::min(p.spw > 0 ? p.spw : auto_walk(a, B, C_::WG_PER_CU), a.ndz));
      const long long n_ = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;
      LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino2): grid too large");
      a.nblk = (int)n_;
      if (g_wpre)
        conv3d_wino2p_kernel<true><<<dim3((unsigned)n_), 256, 0, st>>>(a);
      else
        conv3d_wino2p_kernel<false><<<dim3((unsigned)n_), 256, 0, st>>>(a);
      return launch_status("lea_conv3d(wino2p)");
    }
  }
  set_error("lea_conv3d(wino2): no tile q=%d wc=%d mte=%d nw=%d occ=%d pv=%d", p.q, p.wc, p.mte, p.nw,
            p.occ, p.pv);
  return LEA_E_UNSUPPORTED;
}

const char* name2(const Plan2& p, bool cv) {
  if (p.pv == 3 && !cv) return g_w44 ? "conv3d_wino44_kernel" : "conv3d_wino2p_kernel";
  snprintf(g_name2, sizeof(g_name2), "conv3d_wino2_kernel<%d, %d, %d, %d, %d, %d, %s>", p.q, p.wc, p.mte,
           p.nw, p.occ, p.pv, cv ? "true" : "false");
  return g_name2;
}

}  // namespace wino
}  // namespace lea
