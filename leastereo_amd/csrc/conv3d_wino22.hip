// ConvBR3d k=3 (fp32) for the 16-cout cell convs (the L1 cells' 16 -> 16 ops,
// skip_model_3d.py:41-75 with models/operations_3d.py:31-47) on the fp32 matrix cores with
// two-dimensional Winograd F(2,3) along W x F(2,3) along D, built for occupancy:
//     y[d0 + t][w + j] = sum_{kd, kw} g[kd][kh][kw] x[d0 - 1 + t + kd][w - 1 + j + kw]
//                      = A_D^T [ A_W^T ( U . V ) ]  per kernel row kh,
//     U = G_W g G_D^T (4 x 4 points, G's 1/2 factors included), V = B_W^T x B_D.
// 16 products per 2 (W) x 2 (D) outputs and kh: 1.33x the MFMA work of the F(4,3) x F(2,3)
// engine (conv3d_wino2.hip), but with 64 accumulators instead of 96 and U transformed once
// by the packer (lea_conv3d_wino_pack_weights appends it for 16-cout blocks), the loop holds
// no U transform and the tile fits 128 VGPRs: four waves per SIMD instead of two.  The r04
// counters put the 16-cout L1 ops at MFMA busy 0.30 with 1,920 waves per launch at two per
// SIMD (profiles/r04_small_layer_pmc_b128.txt): bound by latency, not by the MFMA count.
//
// GEMM per point xi = (a, b) and kh, v_mfma_f32_16x16x4_f32 with the engines' lane map:
//     A (lane l) = U[xi][kh][co = l & 15][ci = l >> 4],  B (lane l) = V[xi][kh][ci = l >> 4][group = l & 15],
//     C (lane l, register i) = M[xi][co = 4 (l >> 4) + i][group = l & 15].
// A group is 2 (W) x 2 (D) outputs of one row; a wave's 16 groups are 32 columns of one row,
// a workgroup's 8 waves 8 rows: tile 32 W x 8 H x 2 D per depth pair.  Items = (depth pair,
// 4-channel chunk), double-buffered stages filled by 16-byte LDS-DMA: the chunk's halo
// (4 channels x 4 planes x 10 rows x 40 columns from w0 - 4) and its U (3 kh x 4 ci x 16 co
// x 16 points, 12 KB), one barrier per item.  Each lane reads its 4 planes x 4 inputs per kh
// (two ds_read_b64 per plane) and its U as four ds_read_b128 (quad q of cout co stored at
// q ^ ((co >> 2) & 3): the b128 lane groups read 64 distinct banks).
#include "wino_common.h"

namespace lea {
namespace wino {

struct Cfg22 {
  static constexpr int NW = 8;             // waves = tile rows
  static constexpr int TW = 32, TH = NW, TD = 2;
  static constexpr int RH = TH + 2;        // halo rows
  static constexpr int RWA = 40;           // staged columns w0 - 4 .. w0 + 35 (10 16-byte blocks)
  static constexpr int PLANES = 4;
  static constexpr int PLANEA = RH * RWA;  // floats per staged plane
  static constexpr int BLK = PLANES * PLANEA / 4;  // 16-byte blocks per channel (400)
  static constexpr int PIECES = (BLK + 63) / 64;   // LDS-DMA pieces per channel (7, the last partial)
  // channel stride = 32 mod 64 floats: the two channels of a 32-lane ds_read_b64 group read
  // disjoint bank halves; channel base 1 (odd): column w0 - 1 (staged column 3 + 2 n) of every
  // row is 8-byte aligned for the lane's reads
  static constexpr int CHS = PLANES * PLANEA + 32;
  static constexpr int CB = 1;
  static constexpr int XS = 4 * CHS + 4;   // U region after the halo, 16-byte aligned
  static constexpr int US = 3 * CIN_B * 16 * 16;  // U of one (cout block, chunk): [kh][ci][co][16]
  static constexpr int UPIECES = US / 256;
  static constexpr int STAGE = XS + US;
  static constexpr int NPIECES = CIN_B * PIECES + UPIECES;  // 40: five per wave
  static_assert(CHS % 64 == 32 && PLANEA % 2 == 0 && RWA % 2 == 0 && XS % 4 == 0 && STAGE % 4 == 0, "LDS map");
  static_assert(NPIECES % NW == 0, "whole pieces per wave");
  static_assert(2 * STAGE * 4 * 2 <= 160 * 1024, "two workgroups per CU");
};

// U section of the packed weights (floats): per 16-cout block and 4-channel chunk, US floats
long long u22_section(int cout, int cin) { return (long long)((cout + 15) / 16) * (cin / CIN_B) * Cfg22::US; }

// packer: U[cob][chunk][kh][ci][co][pos] with pos = 4 (q ^ ((co >> 2) & 3)) + e holding point
// (a = q along W, b = e along D) of G_W g G_D^T, G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
__global__ void pack_wino22_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                   long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int pos = (int)(q % 16); q /= 16;
    const int col = (int)(q % 16); q /= 16;
    const int ci = (int)(q % CIN_B); q /= CIN_B;
    const int kh = (int)(q % 3); q /= 3;
    const int nch = cin / CIN_B;
    const int ch = (int)(q % nch), cob = (int)(q / nch);
    const int qa = (pos >> 2) ^ ((col >> 2) & 3), e = pos & 3;  // W point a = qa, D point b = e
    const int co = cob * 16 + col, c = ch * CIN_B + ci;
    float v = 0.f;
    if (co < cout) {
      const float* g = w + ((long long)co * cin + c) * 27;  // [kd][kh][kw]
      float gw[3];  // G_W along kw for each kd
#pragma unroll
      for (int kd = 0; kd < 3; ++kd) {
        const float g0 = g[(kd * 3 + kh) * 3], g1 = g[(kd * 3 + kh) * 3 + 1], g2 = g[(kd * 3 + kh) * 3 + 2];
        gw[kd] = qa == 0 ? g0 : qa == 1 ? 0.5f * (g0 + g1 + g2) : qa == 2 ? 0.5f * (g0 - g1 + g2) : g2;
      }
      v = e == 0 ? gw[0] : e == 1 ? 0.5f * (gw[0] + gw[1] + gw[2]) : e == 2 ? 0.5f * (gw[0] - gw[1] + gw[2]) : gw[2];
    }
    out[i] = v;
  }
}

__global__ __launch_bounds__(512, 4) void conv3d_wino22_kernel(const ConvArgs a) {
  using C = Cfg22;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE];
  const unsigned lds0 = lds_addr(smem);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order (as the other Winograd engines): each XCD walks a contiguous range of
  // (batch/cout-block, tile, depth-pair group); the cout blocks of one (tile, group) adjacent
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
  const int co0 = cob * 16;
  const int nchunks = a.cin / CIN_B;
  const int nitems = npairs * nchunks;
  const int HW = a.H * a.W;  // host checks D*H*W*4 < 2^32
  const unsigned crec = (unsigned)(HW * a.D) * 4u;
  const float* up = a.wp + a.uoff + (long long)cob * nchunks * C::US;

  // this wave's halo pieces of every item (issue below): piece P = channel P / 7, slot P % 7,
  // block e = 64 slot + lane = (plane, row, 16-byte column block)
  constexpr int KP = C::NPIECES / C::NW;
  // per piece: byte offset of its (h, w) in a plane, the plane (0..3) in the low 4 bits
  // (offsets are 16-byte multiples); 0xFFFFFFFF = outside the volume or a surplus lane
  unsigned hwo[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int P = k < 3 ? wave + C::NW * k : 24 + (wave & 3);  // (k >= 3: U pieces for some waves)
    const int j = P % C::PIECES, e = 64 * j + lane;
    const int pl = e / (C::PLANEA / 4), r = e - pl * (C::PLANEA / 4);
    const int rr = r / (C::RWA / 4), blk = r - rr * (C::RWA / 4);
    const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;  // W % 4 == 0: a block is all in or all out
    const bool in = e < C::BLK && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
    hwo[k] = in ? (unsigned)(h * a.W + w) * 4u + (unsigned)pl : 0xFFFFFFFFu;
  }
  const unsigned long long cvolb = (unsigned long long)HW * a.D * 4u;
  const unsigned long long xa = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned long long x2s =
      a.x2 ? (unsigned long long)(a.x2 + (long long)b * a.x2bs) - (unsigned long long)a.cin1 * cvolb : xa;
  // piece k of this wave: k < 3 halo piece wave + 8 k; k = 3: halo piece 24 + wave (waves
  // 0-3) or U piece wave - 4 (waves 4-7); k = 4: U piece 4 + wave -- one DMA per piece,
  // selects instead of branches (a wave-dependent branch per piece made the compiler keep
  // every variant's addresses live across the loop)
  auto issue = [&](int ch, int pr, float* st) {
    const int dm1 = (pz0 + pr) * C::TD - 1;  // the pair's first input plane
    const unsigned sbase = lds0 + 4 * (unsigned)(st - smem);
    const __amdgpu_buffer_rsrc_t urs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(up + (long long)ch * C::US), 0, C::US * 4, 0x00020000);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int P = wave + C::NW * k;
      const bool halo = k < 3 || (k == 3 && wave < 4);  // wave-uniform
      const int hp = halo ? P : 0;
      const int ci = hp / C::PIECES, j = hp % C::PIECES;
      const int c = ch * CIN_B + ci;
      const unsigned long long base = (c < a.cin1 ? xa : x2s) + (unsigned long long)c * cvolb;
      const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, crec, 0x00020000);
      const int d = dm1 + (int)(hwo[k] & 15u);
      const unsigned hvo = (hwo[k] != 0xFFFFFFFFu && (unsigned)d < (unsigned)a.D)
                               ? (hwo[k] & ~15u) + (unsigned)d * (unsigned)HW * 4u : 0xFFFFFFF0u;
      const int u = k == 3 ? wave - 4 : 4 + wave;
      const unsigned uvo = (unsigned)(lane * 16 + u * 1024);
      const unsigned dst = sbase + 4 * (unsigned)(halo ? C::CB + ci * C::CHS + j * 256 : C::XS + u * 256);
      if (k < 3) {
        if (j < C::PIECES - 1 || 64 * j + lane < C::BLK) dma_dwordx4_buf(hrs, hvo, dst);
      } else if (k == 4) {
        dma_dwordx4_buf(urs, uvo, dst);
      } else if (!halo || j < C::PIECES - 1 || 64 * j + lane < C::BLK) {  // the last piece is partial
        dma_dwordx4_buf(halo ? hrs : urs, halo ? hvo : uvo, dst);
      }
    }
  };

  const int ci = lane >> 4, n = lane & 15;
  const int xoff = C::CB + ci * C::CHS + wave * C::RWA + 3 + 2 * n;  // column w0 + 2 n - 1 of row wave
  const int uoff = ci * 256 + n * 16;                                 // [kh][ci][co = n][16]
  const int usw = (n >> 2) & 3;

  f32x4 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue of one depth pair: A_W^T then A_D^T per cout row, BN, ReLU, residual; 8-byte
  // buffer loads / stores (every lane the same count: invalid ones out of range)
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int h = h0 + wave, w = w0 + 2 * n;
  const int nco = min(16, a.cout - co0);
  const __amdgpu_buffer_rsrc_t yrs = block_rsrc(a.y + (long long)b * a.ybs + (long long)co0 * DHW, nco * DHW * 4);
  const __amdgpu_buffer_rsrc_t rrs =
      block_rsrc(resid ? a.res + (long long)b * a.rbs + (long long)co0 * DHW : a.y, nco * DHW * 4);
  // 32-bit byte offsets (the host checks 16 * D * H * W * 4 < kEpiOob); BN through a buffer
  // resource too: no 64-bit per-lane pointers for the compiler to hoist out of the item loop
  const unsigned dhw4 = (unsigned)DHW * 4u, hw4 = (unsigned)HW * 4u;
  const unsigned lane4 = (unsigned)(h * a.W + w) * 4u;
  const bool lv = h < a.H && w < a.W;
  // BN of this cout block (LEA_PAIR_SUM: a's at 0, b's at cout floats further)
  const bool pair = a.flags & kPairSum;
  const int nbn = pair ? a.cout + nco : nco;
  const __amdgpu_buffer_rsrc_t srs = block_rsrc(a.scale ? a.scale + co0 : a.y, a.scale ? nbn * 4 : 0);
  const __amdgpu_buffer_rsrc_t hrs2 = block_rsrc(a.shift ? a.shift + co0 : a.y, a.shift ? nbn * 4 : 0);
  const int nch_a = pair ? a.cin1 / CIN_B : -1;  // LEA_PAIR_SUM: conv a's last chunk + 1
  // part: LEA_PAIR_SUM's second conv (1) reads back the first's output and uses the second
  // half of scale / shift
  auto epilogue = [&](int d0, int part) {
    const bool rd = resid || part == 1;
    const unsigned bn4 = (unsigned)(part * a.cout) * 4u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // one cout row at a time (registers)
      const int cr = 4 * ci + r;
      const bool cv = lv && cr < nco;
      // BN: scale 1, shift 0 without a BN (out-of-range loads read 0)
      const float sc = a.scale ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, bn4 + (unsigned)cr * 4u, 0, 0))
                               : 1.f;
      const float sh = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(hrs2, bn4 + (unsigned)cr * 4u, 0, 0));
      unsigned off[2];
      f32x2 rv[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        off[t] = (cv && d0 + t < a.D) ? (unsigned)cr * dhw4 + (unsigned)(d0 + t) * hw4 + lane4 : kEpiOob;
        if (rd) rv[t] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(part ? yrs : rrs, off[t], 0, 0));
      }
      float tq[2][4];  // A_W^T per D point
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m0 = acc[0 + e][r], m1 = acc[4 + e][r], m2 = acc[8 + e][r], m3 = acc[12 + e][r];
        tq[0][e] = (m0 + m1) + m2;
        tq[1][e] = (m1 - m2) - m3;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x2 y;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v = t == 0 ? (tq[j][0] + tq[j][1]) + tq[j][2] : (tq[j][1] - tq[j][2]) - tq[j][3];
          v = v * sc + sh;
          if (relu) v = fmaxf(v, 0.f);
          y[j] = rd ? v + rv[t][j] : v;
        }
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, y), yrs, off[t], 0, 0);
      }
    }
  };

  issue(0, 0, smem);
  int ich = 0, ipr = 0;
  for (int it = 0; it < nitems; ++it) {
    const int ch = ich;
    const bool wrap = ich + 1 == nchunks;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of item it landed
    __syncthreads();                                   // ... and everyone's; item it-1's stage is free
    if (it + 1 < nitems) issue(wrap ? 0 : ich + 1, wrap ? ipr + 1 : ipr, smem + ((it + 1) & 1) * C::STAGE);
    const float* xs = smem + (it & 1) * C::STAGE;
    const float* us = xs + C::XS;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      float x[4][4];
#pragma unroll
      for (int pl = 0; pl < 4; ++pl) {
        const float* sp = xs + xoff + pl * C::PLANEA + kh * C::RWA;
        const float2 p0 = *reinterpret_cast<const float2*>(sp);
        const float2 p1 = *reinterpret_cast<const float2*>(sp + 2);
        x[pl][0] = p0.x;
        x[pl][1] = p0.y;
        x[pl][2] = p1.x;
        x[pl][3] = p1.y;
      }
      float t[4][4];  // B_D over the planes: t[b][col]
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t[0][c] = x[0][c] - x[2][c];
        t[1][c] = x[1][c] + x[2][c];
        t[2][c] = x[2][c] - x[1][c];
        t[3][c] = x[1][c] - x[3][c];
      }
      float v[4][4];  // B_W over the columns: v[a][b]
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[0][e] = t[e][0] - t[e][2];
        v[1][e] = t[e][1] + t[e][2];
        v[2][e] = t[e][2] - t[e][1];
        v[3][e] = t[e][1] - t[e][3];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 u4 = *reinterpret_cast<const f32x4*>(us + kh * (CIN_B * 256) + uoff + 4 * (q ^ usw));
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[4 * q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(u4[e], v[q][e], acc[4 * q + e], 0, 0, 0);
      }
      // one kh step's operands live at a time (the 64 accumulators + 16 V + 4 U fit 128
      // VGPRs only without the next steps' reads hoisted above these MFMAs)
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ch == nchunks - 1 || ch == nch_a - 1) {  // the pair's (or conv a's) last chunk: epilogue, fresh accumulators
      epilogue((pz0 + ipr) * C::TD, ch == nchunks - 1 && pair ? 1 : 0);
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    ich = wrap ? 0 : ich + 1;
    ipr += wrap;
  }
}

// host: the layers this tile takes -- couts <= 32 (16-cout blocks over the grid), 16-byte rows
// and sources, the buffer-addressed epilogue's ranges; packed weights with the U section
bool wino22_ok(const ConvArgs& a) {
  return a.cout <= 32 && a.W % 4 == 0 && ((uintptr_t)a.x & 15) == 0 && a.xbs % 4 == 0 &&
         (a.cin1 == a.cin || (((uintptr_t)a.x2 & 15) == 0 && a.x2bs % 4 == 0)) && a.W % 2 == 0 &&
         ((uintptr_t)a.y & 7) == 0 && a.ybs % 2 == 0 &&
         (!(a.flags & LEA_RESIDUAL) || (((uintptr_t)a.res & 7) == 0 && a.rbs % 2 == 0)) &&
         16LL * a.D * a.H * a.W * 4 < (long long)kEpiOob;
}

int run22(ConvArgs a, int B, int spw, hipStream_t st) {
  using C = Cfg22;
  a.ncob = (a.cout + 15) / 16;
  a.tiles_w = (a.W + C::TW - 1) / C::TW;
  a.ntiles = a.tiles_w * ((a.H + C::TH - 1) / C::TH);
  a.ndz = (a.D + C::TD - 1) / C::TD;
  // depth pairs per workgroup: two when that leaves one round of workgroups (2 per CU) instead
  // of two (r05 tools/w22_ab.py, C2 L1 16 -> 16: 960 workgroups 47 us, 480 walking 2 pairs 44 us;
  // C5's 3696 workgroups equal either way)
  if (spw <= 0) {
    const long long base = (long long)a.ntiles * a.ndz * B * a.ncob;
    spw = base > 512 && base <= 1024 ? 2 : 1;
  }
  a.spw = std::max(1, std::min(spw, a.ndz));
  const long long n = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;
  LEA_CHECK_ARG(n < (1LL << 31), "lea_conv3d(wino22): grid too large");
  a.nblk = (int)n;
  conv3d_wino22_kernel<<<dim3((unsigned)n), 512, 0, st>>>(a);
  return launch_status("lea_conv3d(wino22)");
}

}  // namespace wino
}  // namespace lea
