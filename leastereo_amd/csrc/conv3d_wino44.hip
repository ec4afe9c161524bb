// ConvBR3d k=3 (fp32) with two-dimensional Winograd F(4,3) along W x F(4,3) along D (r06)
// on the fp32 matrix cores: the 32-cout layers the pipelined W x D kernel runs
// (conv3d_wino2.hip, conv3d_wino2p_kernel: F(4,3) x F(2,3)), with 3/4 of its MFMA work.
// Replaces models/operations_3d.py:31-47 for those layers (retrain/skip_model_3d.py:142,
// 150, 155: stem1, conv1, conv2, the cells' 3x3x3 ops).
//
// Per output group of 4 (W) x 4 (D) voxels and kernel row kh:
//     y = A_D^T [ A_W^T ( (G_W g G_D^T) . (B_W^T x B_D) ) ]
// takes 6 x 6 = 36 products per input channel against F(4,3) x F(2,3)'s 2 x 24 = 48 for the
// same four output planes (and 144 for the direct convolution).  Both axes use the points
// 0, +-1, +-2, inf (bw4 / gw4 / aw4 of conv3d_wino2.hip); G's row factors are applied to the
// accumulators in the epilogue along both axes.
//
// 36 points x 4 accumulators per 16 x 16 tile (144 VGPRs) do not fit beside the operands at
// two waves per SIMD, so the W points are split between two waves: wave (xh, wc) owns the W
// points 3 xh .. 3 xh + 2 of cout tile wc (16 couts) -- 18 points, 72 accumulator VGPRs.  The
// workgroup = 2 x-halves x 2 cout tiles = 4 waves over one 32 (W) x 2 (H) x 4 (D) x 32 (cout)
// output tile; two workgroups per CU (74 KB of LDS each).
//
// Item i = (depth quad, 4-channel chunk), the one-barrier pipeline of conv3d_wino2p_kernel:
//   top      this wave's halo(i + 1) pieces and weights g(i) have landed (vmcnt), barrier
//   steps(i) V from tv[i & 1], U = G_D' (G_W' g) from the per-lane weights, 18 MFMAs per kh
//            step and wave; interleaved with the V-pass(i + 1): halo[(i + 1) & 1] -> tv[(i + 1) & 1]
//   halo(i + 2) -> halo[i & 1] (16-byte LDS-DMA pieces, 4 per wave), g(i + 1) -> registers
// V-pass: thread t forms V for one (channel, halo row, W group, x-half): the W transform of
// its three points on each of the 6 input planes, then the D transform (B^T of F(4,3) along
// the planes) -- 18 floats [x][e], exactly what the consuming wave reads.
// Epilogue (the quad's last chunk): the two x-halves of a cout tile swap accumulators through
// LDS (the just-consumed V and halo buffers, one exchange) so each holds all 36 points of two of the
// four couts its lanes carry, then A_W^T and A_D^T (with G's factors), BN, ReLU, residual,
// buffer-addressed float4 stores.
//
// LDS maps (exhaustive checks in the comments below, tools/w44_banks.py):
//   halo: channel c at CB(c) == {1, 3, 33, 35}[c] mod 64, rows of RWA = 40 floats from w0 - 4
//         (whole 16-byte blocks), planes PLANEA = 160 apart; the V-pass's b64 reads
//         (32 lanes = 8 groups x 4 channels) hit 64 distinct banks
//   V:    [ci: TCS = 1284][row: TRS = 320][group: GS = 40][x-half: 20][x 3][e 6]; the steps'
//         ds_read_b128 lane groups read 16 distinct 16-byte slots, the V-pass's ds_write_b128
//         groups of 8 lanes (4 groups x 2 channels) 8 distinct slots of 32 banks
#include <type_traits>

#include "wino_common.h"

namespace lea {
namespace wino {

namespace w44 {
constexpr int Q = 8, F = 4, TW = 32, TH = 2, TD = 4, PLANES = 6, RH = TH + 2, RWA = TW + 8;
constexpr int PLANEA = RH * RWA;               // 160 floats per staged plane
constexpr int BLK16 = PLANES * PLANEA / 4;     // 240 16-byte blocks per channel
constexpr int CB0 = 1, CB1 = CB0 + 1024 + 2, CB2 = CB1 + 1024 + 30, CB3 = CB2 + 1024 + 2;
constexpr int XS = (CB3 + 1024 + 3) / 4 * 4;   // floats per halo buffer
constexpr int GS = 40, XHS = 20, TRS = 320, TCS = 1284, TS = 4 * TCS;
constexpr int KGL = 28;                        // per-lane weights per (cout, channel): [kh][kd][x 3] + pad
constexpr int KGU = 56;                        // UPRE: U = G_D' G_W' g, [kh][x 3][e 6] + pad
constexpr int NST = 8;                         // buffer stores per epilogue and lane
static_assert(CB1 % 64 == 3 && CB2 % 64 == 33 && CB3 % 64 == 35, "V-pass bank map");
static_assert(BLK16 <= 4 * 64 && 4 * 256 <= CB1 - CB0, "whole pieces per channel region");
static_assert(TRS % 64 == 0 && TCS % 8 == 4 && GS % 8 == 0 && XHS % 4 == 0 && TRS >= Q * GS && TCS >= RH * TRS,
              "V bank map");
static_assert(4 * 64 * 20 <= TS && 4 * 64 * 16 <= XS, "epilogue exchange fits a V and a halo buffer");
static_assert((2 * XS + 2 * TS) * 4 * 2 <= 160 * 1024, "two workgroups per CU");
}  // namespace w44

// per-lane weights of one (cout block of 32, chunk, cout tile wc, x-half xh): 7 slices of 64
// lanes x 4 floats; lane = 16 ci + n, entry k = kh * 9 + kd * 3 + x3 of G_W' g (gw4's outputs
// 3 xh .. 3 xh + 2 for kernel row (kd, kh)) of cout 32 cb + 16 wc + n, channel 4 chunk + ci
__global__ void pack_wino44_lane_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                        int nchunks, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int e = (int)(q % (64 * w44::KGL)); q /= 64 * w44::KGL;
    const int k = (e / 256) * 4 + (e & 3), ln = (e & 255) >> 2;
    const int xh = (int)(q % 2); q /= 2;
    const int wc = (int)(q % 2); q /= 2;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int co = cb * 32 + 16 * wc + (ln & 15), c = ch * CIN_B + (ln >> 4);
    float v = 0.f;
    if (k < 27 && co < cout && c < cin) {
      const int kh = k / 9, kd = (k % 9) / 3, x = 3 * xh + k % 3;
      const float* g = w + (((long long)co * cin + c) * 9 + kd * 3 + kh) * 3;
      const float s = g[0] + g[2], s4 = fmaf(4.f, g[2], g[0]);  // gw4 (conv3d_wino2.hip)
      const float u[6] = {g[0], s + g[1], s - g[1], fmaf(2.f, g[1], s4), fmaf(-2.f, g[1], s4), g[2]};
      v = u[x];
    }
    out[i] = v;
  }
}

// the UPRE copy (r06): entry k = kh * 18 + x3 * 6 + e of U = G_D' (G_W' g) -- the kernel's own
// transform (gw4 along W, then along D), so the same bits -- after the G_W' g copy
__global__ void pack_wino44_lane_u_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                          int nchunks, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long q = i;
    const int e = (int)(q % (64 * w44::KGU)); q /= 64 * w44::KGU;
    const int k = (e / 256) * 4 + (e & 3), ln = (e & 255) >> 2;
    const int xh = (int)(q % 2); q /= 2;
    const int wc = (int)(q % 2); q /= 2;
    const int ch = (int)(q % nchunks);
    const int cb = (int)(q / nchunks);
    const int co = cb * 32 + 16 * wc + (ln & 15), c = ch * CIN_B + (ln >> 4);
    float v = 0.f;
    if (k < 54 && co < cout && c < cin) {
      const int kh = k / 18, x = 3 * xh + (k % 18) / 6, ed = k % 6;
      float gwx[3];
      for (int kd = 0; kd < 3; ++kd) {
        const float* g = w + (((long long)co * cin + c) * 9 + kd * 3 + kh) * 3;
        const float s = g[0] + g[2], s4 = fmaf(4.f, g[2], g[0]);
        const float u[6] = {g[0], s + g[1], s - g[1], fmaf(2.f, g[1], s4), fmaf(-2.f, g[1], s4), g[2]};
        gwx[kd] = u[x];
      }
      const float g0 = gwx[0], g1 = gwx[1], g2 = gwx[2];
      const float s = g0 + g2, s4 = fmaf(4.f, g2, g0);
      const float u[6] = {g0, s + g1, s - g1, fmaf(2.f, g1, s4), fmaf(-2.f, g1, s4), g2};
      v = u[ed];
    }
    out[i] = v;
  }
}

long long lane44_g_floats(int cout, int cin) { return (long long)((cout + 31) / 32) * (cin / CIN_B) * 4 * 64 * w44::KGL; }
long long lane44_floats(int cout, int cin) {
  return lane44_g_floats(cout, cin) + (long long)((cout + 31) / 32) * (cin / CIN_B) * 4 * 64 * w44::KGU;
}

namespace {
// F(4,3): B^T x (6 -> 6), G' g (3 -> 6, no row factors), A^T with the factors (6 -> 4)
__device__ __forceinline__ void bt6(const float x0, const float x1, const float x2, const float x3, const float x4,
                                    const float x5, float* v) {
  const float pa = fmaf(-4.f, x2, x4), pb = fmaf(-4.f, x1, x3);
  const float pc = x4 - x2, pd = 2.f * (x3 - x1);
  v[0] = fmaf(4.f, x0, fmaf(-5.f, x2, x4));
  v[1] = pa + pb;
  v[2] = pa - pb;
  v[3] = pc + pd;
  v[4] = pc - pd;
  v[5] = fmaf(4.f, x1, fmaf(-5.f, x3, x5));
}
__device__ __forceinline__ void at6(const float a0, const float a1, const float a2, const float a3, const float a4,
                                    const float a5, float* y) {
  const float m0 = 0.25f * a0;
  const float m1 = (-1.f / 6.f) * a1, m2 = (-1.f / 6.f) * a2;
  const float m3 = (1.f / 24.f) * a3, m4 = (1.f / 24.f) * a4;
  const float sp = m1 + m2, sm = m1 - m2, tp = m3 + m4, tm = m3 - m4;
  y[0] = (m0 + sp) + tp;
  y[1] = fmaf(2.f, tm, sm);
  y[2] = fmaf(4.f, tp, sp);
  y[3] = fmaf(8.f, tm, sm) + a5;
}
}  // namespace

// UPRE (lea_conv3d_wino44_set_upre): the per-lane weights are U itself (the packer's second
// copy), so the step forms no U: 54 fewer VALU per item, 7 more 16-byte loads, 28 more VGPRs
// SCHED (lea_conv3d_wino44_set_sched, r06 A/B, profiles/r06_w44_sched_ab*.txt): 0 = the body
// below under iglp_opt(0) (the V-pass after the first step's MFMAs); 1 = the V-pass after the
// second step's MFMAs; 2 = as 0 without iglp_opt; 3 = the V-pass after all MFMAs.  (Measured
// and dropped: the V-pass issued first, +4 %; an explicit one-MFMA / three-VALU
// sched_group_barrier interleave, +10 %.)
template <bool UPRE, int SCHED>
__global__ __launch_bounds__(256, 2) void conv3d_wino44_kernel(const ConvArgs a) {
  using namespace w44;
  constexpr int NX = 3, NE = 6;  // this wave's W points x the D points
  __shared__ __attribute__((aligned(16))) float smem[2 * XS + 2 * TS];
  const unsigned lds0 = lds_addr(smem);
  float* const halo = smem;          // halo[k] = smem + k * XS
  float* const tvb = smem + 2 * XS;  // tv[k] = tvb + k * TS

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 1, xh = wave >> 1;
  const int nblk = a.nblk;
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = nblk / 8, r8 = nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int spw = a.spw > 0 ? a.spw : 1;
  const int ngz = (a.ndz + spw - 1) / spw;
  int cob, gz, th, tw, b;
  if (a.grp == 0) {  // linear: cout block fastest, then depth group, then tile
    cob = lin % a.ncob;
    const int rest = lin / a.ncob;
    gz = rest % ngz;
    const int tile = (rest / ngz) % a.ntiles;
    b = rest / (ngz * a.ntiles);
    th = tile / a.tiles_w;
    tw = tile % a.tiles_w;
  } else {
    // grouped: the ~64 workgroups an XCD holds at once (consecutive `lin`) cover a box of
    // GZ depth groups x G tile rows x G tile columns x every cout block, so the halo rows,
    // planes and columns neighbouring tiles share are fetched once into that XCD's L2.
    // Edge groups are partial; all divisions are scalar.
    const int G = a.grp, nth = a.ntiles / a.tiles_w, ntw = a.tiles_w;
    const int GZ = max(1, 64 / (a.ncob * G * G));
    const int per_b = a.ncob * ngz * a.ntiles;
    b = lin / per_b;
    int r = lin - b * per_b;
    const int slab = a.ncob * GZ * a.ntiles;
    const int i = r / slab;
    r -= i * slab;
    const int cz = min(GZ, ngz - i * GZ);
    const int rowg = a.ncob * cz * G * ntw;
    const int j = r / rowg;
    r -= j * rowg;
    const int ch = min(G, nth - j * G);
    const int cellg = a.ncob * cz * ch * G;
    const int k = r / cellg;
    r -= k * cellg;
    const int cw = min(G, ntw - k * G);
    cob = r % a.ncob;
    r /= a.ncob;
    tw = k * G + r % cw;
    r /= cw;
    th = j * G + r % ch;
    gz = i * GZ + r / ch;
  }
  const int h0 = th * TH;
  const int w0 = tw * TW;
  const int pz0 = gz * spw, nquads = min(spw, a.ndz - pz0);
  const int co0 = cob * 32;
  const int nchunks = a.cin / CIN_B;
  const int nitems = nquads * nchunks;
  const int HW = a.H * a.W;
  const unsigned nrec = (unsigned)(HW * a.D) * 4u;
  const long long cvol = (long long)HW * a.D;
  // per-lane weights: this kernel's section of the packed weights at a.uoff (the host's l44_offset)
  constexpr int GL = UPRE ? KGU : KGL;
  const float* wl = a.wp + a.uoff + (UPRE ? (long long)a.ncob * nchunks * 4 * 64 * KGL : 0LL) +
                    ((long long)(cob * nchunks) * 4 + wc * 2 + xh) * 64 * GL + lane * 4;

  // 16-byte halo pieces: piece = wave of every channel; block e16 = (plane, row, 16-byte column)
  const int e16 = 64 * wave + lane;
  unsigned hwo16 = 0xFFFFFFF0u;
  int pln16 = -1000;
  {
    const int p = e16 / (RH * (RWA / 4)), r = e16 - p * (RH * (RWA / 4));
    const int rr = r / (RWA / 4), blk = r - rr * (RWA / 4);
    const int h = h0 + rr - 1, w = w0 - 4 + 4 * blk;
    if (e16 < BLK16 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
      hwo16 = (unsigned)(h * a.W + w) * 4u;
      pln16 = p - 1;
    }
  }
  const unsigned long long cvolb = (unsigned long long)cvol * 4u;
  const unsigned long long xa = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned long long x2s =
      a.x2 ? (unsigned long long)(a.x2 + (long long)b * a.x2bs) - (unsigned long long)a.cin1 * cvolb : xa;
  auto issue_halo = [&](int ch, int qd, int buf) {  // branch-free: every lane, every channel
    const int d = (pz0 + qd) * TD + pln16;
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
  float4 gw[GL / 4];  // this lane's G_W' g of the current chunk: [kh][kd][x 3] (UPRE: U, [kh][x 3][e 6])
  auto load_g = [&](int ch) {
    const float4* src = reinterpret_cast<const float4*>(wl + (long long)ch * 4 * 64 * GL);
#pragma unroll
    for (int k = 0; k < GL / 4; ++k) gw[k] = src[64 * k];
  };
  // V-pass unit of thread t: W group vg, channel vc, halo row vr, x-half vxh (wave-uniform)
  const int vg = (tid & 3) | (((tid >> 3) & 1) << 2);
  const int vc = ((tid >> 2) & 1) | (((tid >> 4) & 1) << 1);
  const int vr = (tid >> 5) & 3;
  const int vxh = __builtin_amdgcn_readfirstlane(tid >> 7);
  const int vxo = (vc == 0 ? CB0 : vc == 1 ? CB1 : vc == 2 ? CB2 : CB3) + vr * RWA + 3 + F * vg;
  const int vto = vc * TCS + vr * TRS + GS * vg + XHS * vxh;
  auto vpass = [&](auto XHC, int buf) {
    constexpr int VXH = decltype(XHC)::value;  // == vxh (wave-uniform): a compile-time branch
    const float* sp0 = halo + buf * XS + vxo;
    float bw[PLANES][3];
#pragma unroll
    for (int pl = 0; pl < PLANES; ++pl) {
      const float* sp = sp0 + pl * PLANEA;
      // native 8-byte vectors, kept whole: HIP's float2 struct loaded as two dwords (and the
      // unused half of a2 dropped) became ds_read2_b32 / ds_read_b32, banked on 32 banks, where
      // the channel bases (1, 3, 33, 35 mod 64) collide two-way; as ds_read_b64 they are
      // conflict-free (tools/w44_banks.py)
      f32x2 a0 = *reinterpret_cast<const f32x2*>(sp);
      f32x2 a1 = *reinterpret_cast<const f32x2*>(sp + 2);
      f32x2 a2 = *reinterpret_cast<const f32x2*>(sp + 4);
      asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2));
      if constexpr (VXH == 0) {  // W points 0, 1, 2 (bt6's first three rows)
        const float pa = fmaf(-4.f, a1.x, a2.x), pb = fmaf(-4.f, a0.y, a1.y);
        bw[pl][0] = fmaf(4.f, a0.x, fmaf(-5.f, a1.x, a2.x));
        bw[pl][1] = pa + pb;
        bw[pl][2] = pa - pb;
      } else {  // W points 3, 4, 5
        const float pc = a2.x - a1.x, pd = 2.f * (a1.y - a0.y);
        bw[pl][0] = pc + pd;
        bw[pl][1] = pc - pd;
        bw[pl][2] = fmaf(4.f, a0.y, fmaf(-5.f, a1.y, a2.y));
      }
    }
    float v[3][NE];
#pragma unroll
    for (int x = 0; x < 3; ++x) bt6(bw[0][x], bw[1][x], bw[2][x], bw[3][x], bw[4][x], bw[5][x], v[x]);
    float* tp = tvb + buf * TS + vto;
    const float* vf = &v[0][0];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      *reinterpret_cast<float4*>(tp + 4 * k) = make_float4(vf[4 * k], vf[4 * k + 1], vf[4 * k + 2], vf[4 * k + 3]);
    // floats 16, 17 as a 16-byte store into the unit's 20-float slot (the last two are padding): as
    // ds_write_b64 they met two-way on 32 banks (tools/w44_banks.py)
    *reinterpret_cast<f32x4*>(tp + 16) = f32x4{vf[16], vf[17], vf[16], vf[17]};
  };

  const int ci = lane >> 4, p = lane & 15;
  const int pq = p % Q, pr = p / Q;
  const int toff = ci * TCS + pr * TRS + GS * pq + XHS * xh;
  f32x4 acc[NX][NE];
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[x][e] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue: this wave finalizes couts 4 ci + 2 xh + {0, 1} of its tile
  float sc[2], sh[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int co = co0 + 16 * wc + 4 * ci + 2 * xh + r;
    const bool cv = co < a.cout;
    sc[r] = (cv && a.scale) ? a.scale[co] : 1.f;
    sh[r] = (cv && a.shift) ? a.shift[co] : 0.f;
  }
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  const long long DHW = (long long)HW * a.D;
  const int w = w0 + F * pq;
  const int h = h0 + pr;
  const int nco = min(32, a.cout - co0);
  const __amdgpu_buffer_rsrc_t yrs = block_rsrc(a.y + (long long)b * a.ybs + (long long)co0 * DHW, nco * DHW * 4);
  const __amdgpu_buffer_rsrc_t rrs =
      block_rsrc((resid ? a.res : a.y) + (long long)b * (resid ? a.rbs : a.ybs) + (long long)co0 * DHW, nco * DHW * 4);
  // the epilogue body for x-half XH (a compile-time constant: every register index static)
  auto epilogue_xh = [&](auto XHC, int d0, float* xch0, float* xch1) {
    constexpr int XH = decltype(XHC)::value;
    constexpr int RS = 2 * (1 - XH);  // the element pair of the f32x4 the partner finalizes
    // swap accumulators with the other x-half of this cout tile (wave ^ 2) in one exchange through
    // xch0 (the V buffer just consumed) and xch1 (the halo buffer V-pass(it + 1) consumed)
    float mine[2][6][NE];  // [r][x 0..5][e]: all 36 points of this wave's two couts
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        mine[0][3 * XH + x][e] = acc[x][e][2 * XH];
        mine[1][3 * XH + x][e] = acc[x][e][2 * XH + 1];
      }
    // the 36 values this wave sends, [x][e][r]: 20 through xch0, 16 through xch1 (float4s, lanes contiguous)
    float snd[36];
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        snd[(x * 6 + e) * 2] = acc[x][e][RS];
        snd[(x * 6 + e) * 2 + 1] = acc[x][e][RS + 1];
      }
    __syncthreads();  // every wave done reading both buffers (the steps' V, the V-pass's halo)
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float* wr = k < 5 ? xch0 + wave * (20 * 64) + k * 256 : xch1 + wave * (16 * 64) + (k - 5) * 256;
      reinterpret_cast<float4*>(wr)[lane] = make_float4(snd[4 * k], snd[4 * k + 1], snd[4 * k + 2], snd[4 * k + 3]);
    }
    __syncthreads();
    float rcv[36];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float* rd = k < 5 ? xch0 + (wave ^ 2) * (20 * 64) + k * 256 : xch1 + (wave ^ 2) * (16 * 64) + (k - 5) * 256;
      const float4 t = reinterpret_cast<const float4*>(rd)[lane];
      rcv[4 * k] = t.x;
      rcv[4 * k + 1] = t.y;
      rcv[4 * k + 2] = t.z;
      rcv[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int x = 0; x < NX; ++x)
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        mine[0][3 * (1 - XH) + x][e] = rcv[(x * 6 + e) * 2];
        mine[1][3 * (1 - XH) + x][e] = rcv[(x * 6 + e) * 2 + 1];
      }
    const bool lv = h < a.H && w < a.W;
    unsigned off[2][TD];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < TD; ++t) {
        const int cr = 16 * wc + 4 * ci + 2 * XH + r, d = d0 + t;
        off[r][t] = (lv && cr < nco && d < a.D) ? (unsigned)(cr * DHW + (long long)d * HW + h * a.W + w) * 4u
                                                : kEpiOob;
      }
    f32x4 rv[2][TD];
    if (resid) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int t = 0; t < TD; ++t) rv[r][t] = buf_load4(rrs, off[r][t]);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float n[NE][F];  // A_W^T per D point
#pragma unroll
      for (int e = 0; e < NE; ++e)
        at6(mine[r][0][e], mine[r][1][e], mine[r][2][e], mine[r][3][e], mine[r][4][e], mine[r][5][e], n[e]);
      float yd[F][TD];  // A_D^T per W output
#pragma unroll
      for (int j = 0; j < F; ++j) at6(n[0][j], n[1][j], n[2][j], n[3][j], n[4][j], n[5][j], yd[j]);
#pragma unroll
      for (int t = 0; t < TD; ++t) {
        f32x4 y;
#pragma unroll
        for (int j = 0; j < F; ++j) {
          float v = yd[j][t] * sc[r] + sh[r];
          if (relu) v = fmaxf(v, 0.f);
          y[j] = resid ? v + rv[r][t][j] : v;
        }
        buf_store4(yrs, off[r][t], y);
      }
    }
  };
  // the prologue and the item loop, specialised per x-half (wave-uniform): no branch in the body
  auto run = [&](auto XHC) {
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
    vpass(XHC, 0);
    bool after_epi = false;
    int ich = 0, iqd = 0;  // item it = (chunk, depth quad)
    int hch = min(2, nitems - 1) % nchunks, hqd = min(2, nitems - 1) / nchunks;
    for (int it = 0; it < nitems; ++it) {
      if (after_epi)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const float* tv = tvb + (it & 1) * TS;
      struct Raw {
        float4 v4[4];
        f32x4 v2;  // floats 16, 17 (and the slot's two padding floats)
      };
      auto load_step = [&](int kh, Raw& o) {
        const float* tp = tv + toff + kh * TRS;
  #pragma unroll
        for (int k = 0; k < 4; ++k) o.v4[k] = reinterpret_cast<const float4*>(tp)[k];
        // read whole (ds_read_b128: conflict-free): as a b64 the compiler paired two kh rows into
        // a ds_read2_b64, four-way on 32 banks
        o.v2 = *reinterpret_cast<const f32x4*>(tp + 16);
        asm volatile("" : "+v"(o.v2));
      };
      struct Xf {
        float v[NX][NE];
        float u[NX][NE];
      };
      auto xform = [&](int kh, const Raw& o, Xf& T) {
        const float e18[18] = {o.v4[0].x, o.v4[0].y, o.v4[0].z, o.v4[0].w, o.v4[1].x, o.v4[1].y,
                               o.v4[1].z, o.v4[1].w, o.v4[2].x, o.v4[2].y, o.v4[2].z, o.v4[2].w,
                               o.v4[3].x, o.v4[3].y, o.v4[3].z, o.v4[3].w, o.v2[0], o.v2[1]};
  #pragma unroll
        for (int x = 0; x < NX; ++x)
  #pragma unroll
          for (int e = 0; e < NE; ++e) T.v[x][e] = e18[x * 6 + e];
        if constexpr (UPRE) {
          const float* u = reinterpret_cast<const float*>(gw) + kh * 18;
  #pragma unroll
          for (int x = 0; x < NX; ++x)
  #pragma unroll
            for (int e = 0; e < NE; ++e) T.u[x][e] = u[x * 6 + e];
        } else {
          const float* g = reinterpret_cast<const float*>(gw) + kh * 9;
  #pragma unroll
          for (int x = 0; x < NX; ++x) {  // G_D' along the kernel depth (gw4)
            const float g0 = g[x], g1 = g[3 + x], g2 = g[6 + x];
            const float s = g0 + g2, s4 = fmaf(4.f, g2, g0);
            T.u[x][0] = g0;
            T.u[x][1] = s + g1;
            T.u[x][2] = s - g1;
            T.u[x][3] = fmaf(2.f, g1, s4);
            T.u[x][4] = fmaf(-2.f, g1, s4);
            T.u[x][5] = g2;
          }
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
      if constexpr (SCHED != 2) __builtin_amdgcn_iglp_opt(0);
      load_step(0, raw[0]);
      load_step(1, raw[1]);
      xform(0, raw[0], xf[0]);
      // halo(it + 2) into the buffer V-pass(it) read; past the last item the DMA / V-pass /
      // loads repeat the last one (nothing reads them): one basic block
      issue_halo(hch, hqd, it & 1);
      load_step(2, raw[0]);
      xform(1, raw[1], xf[1]);
      mfmas(xf[0]);
      if constexpr (SCHED == 0 || SCHED == 2) vpass(XHC, (it + 1) & 1);
      xform(2, raw[0], xf[0]);
      load_g(it + 1 < nitems ? (ich + 1 == nchunks ? 0 : ich + 1) : ich);
      mfmas(xf[1]);
      if constexpr (SCHED == 1) vpass(XHC, (it + 1) & 1);
      mfmas(xf[0]);
      if constexpr (SCHED == 3) vpass(XHC, (it + 1) & 1);
      after_epi = false;
      if (ich == nchunks - 1) {
        epilogue_xh(XHC, (pz0 + iqd) * TD, tvb + (it & 1) * TS, halo + ((it + 1) & 1) * XS);
        after_epi = true;
  #pragma unroll
        for (int x = 0; x < NX; ++x)
  #pragma unroll
          for (int e = 0; e < NE; ++e) acc[x][e] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (++ich == nchunks) {
        ich = 0;
        ++iqd;
      }
      if (it + 3 < nitems && ++hch == nchunks) {
        hch = 0;
        ++hqd;
      }
    }
  };
  if (xh == 0)
    run(std::integral_constant<int, 0>{});
  else
    run(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// lea_conv3d_wino44_set (r06 default 1: -9.5 % on its layers, profiles/r06_w44_ab.txt; 2 since v45,
// after the LDS-conflict fixes: the L0 8 -> 24 group 275.6 -> 259.7 us, profiles/r06_w44_modes_ab.txt)
int g_w44 = 2;
int g_w44u = 0;  // lea_conv3d_wino44_set_upre
int g_w44s = 0;  // lea_conv3d_wino44_set_sched
int g_w44g = -1;  // lea_conv3d_wino44_set_group (-1: auto)

int run44(ConvArgs a, int B, int spw, hipStream_t st) {
  a.ncob = (a.cout + 31) / 32;
  a.tiles_w = (a.W + w44::TW - 1) / w44::TW;
  a.ntiles = a.tiles_w * ((a.H + w44::TH - 1) / w44::TH);
  a.ndz = (a.D + w44::TD - 1) / w44::TD;
  a.spw = std::max(1, std::min(spw > 0 ? spw : auto_walk(a, B, 2), a.ndz));
  const long long n_ = (long long)a.ntiles * ((a.ndz + a.spw - 1) / a.spw) * B * a.ncob;
  LEA_CHECK_ARG(n_ < (1LL << 31), "lea_conv3d(wino44): grid too large");
  a.nblk = (int)n_;
  // auto: 16 x 16-tile groups on the large grids (C2: conv1/2 and stem1, 3840 workgroups; HBM
  // traffic -42 / -44 %, time unchanged, profiles/r06_w44_group_traffic2.txt), linear on the
  // small ones (<= 864 workgroups, whose whole grid fits the L2s; grouped +1-2 %,
  // r06_w44_group_ab.txt)
  a.grp = g_w44g >= 0 ? g_w44g : (n_ >= 2048 ? 16 : 0);
  const dim3 grid((unsigned)n_);
  if (g_w44u)
    conv3d_wino44_kernel<true, 0><<<grid, 256, 0, st>>>(a);
  else if (g_w44s == 1)
    conv3d_wino44_kernel<false, 1><<<grid, 256, 0, st>>>(a);
  else if (g_w44s == 2)
    conv3d_wino44_kernel<false, 2><<<grid, 256, 0, st>>>(a);
  else if (g_w44s == 3)
    conv3d_wino44_kernel<false, 3><<<grid, 256, 0, st>>>(a);
  else
    conv3d_wino44_kernel<false, 0><<<grid, 256, 0, st>>>(a);
  return launch_status("lea_conv3d(wino44)");
}

}  // namespace wino
}  // namespace lea
