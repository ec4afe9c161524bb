// bf16 path (BASELINE configs 3 and 4): ConvBR3d on bf16 activations with the
// gfx950 bf16 matrix cores, v_mfma_f32_16x16x32_bf16 (f32 accumulate).
// Replaces models/operations_3d.py:31-47 like conv3d.hip, at dtype LEA_BF16.
//
// Layout "c8": bf16 NCDHW with channels blocked by 8 innermost,
//     x[b][c / 8][d][h][w][c % 8]
// so one voxel's 8 channels are one 16-byte word.  The MFMA wants, per lane, 8
// consecutive K values (lane l holds A[row l&15][k = 8(l>>4) + j] and
// B[k = 8(l>>4) + j][col l&15]); with K ordered (tap, channel block) a B fragment
// is one such word: ds_read_b128 from the staged halo.  K slot 4s + g of k-step s
// (lane group g = l >> 4) is tap (4s+g) / NB, channel block (4s+g) % NB of the
// chunk, NB in {1, 2} blocks per K chunk (4 for 1x1).
//
// Workgroup = 4 waves over a TH x 16 voxel x TD plane tile and COB = WC*MT*16
// output channels: WC waves split the couts (MT 16-row tiles each), WV = 4/WC
// split the voxel rows (NV 16-voxel rows each), so every wave reuses each B
// fragment for MT MFMAs and each A fragment for NV.  A fragments (weights) come
// straight from global memory (L2-resident, packed in fragment order) into
// registers at the start of each chunk; the input halo is staged by LDS-DMA
// (buffer_load_dwordx4 ... lds: one voxel-block per lane, out-of-range offsets
// return zeros = the conv's padding), double-buffered.
#include "common.h"

namespace lea {
namespace bf {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
using f32x4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;
using lds_void = __attribute__((address_space(3))) void;
constexpr int kThreads = 256;

struct Args {
  const __bf16* x;   // blocks [0, cb1)
  long long xbs;
  const __bf16* x2;  // blocks [cb1, cin/8): the virtual concat
  long long x2bs;
  int cb1;
  const __bf16* wp;
  const float* scale;
  const float* shift;
  const __bf16* res;
  long long rbs;
  __bf16* y;
  long long ybs;
  int cin, cout, D, H, W;
  int tiles_w, ntiles, ndz, nblk, ncob, nchunks;
  unsigned flags;
};

// packing geometry shared by host and device
__host__ __device__ constexpr int cob_of(int cout) { return cout <= 16 ? 16 : (cout <= 32 ? 32 : 64); }
__host__ __device__ constexpr int nb_of(int cin, int ks) { return ks == 1 ? 4 : (cin <= 8 ? 1 : 2); }
__host__ __device__ constexpr int ksteps(int ks, int nb) { return (ks * ks * ks * nb + 3) / 4; }

// KD = kernel depth: KS for the 3D convs, 1 for 2D 3x3 convs (feature net: the
// D = 1 case of a (1, 3, 3) kernel)
template <int KS, int MT, int WC, int TH, int TD, int NB, bool CV, int KD = KS>
struct Cfg {
  static constexpr int WV = 4 / WC;
  static constexpr int VT = TH * TD;        // 16-voxel rows in the tile
  static constexpr int NV = VT / WV;        // per wave
  static_assert(VT % WV == 0, "rows per wave");
  static constexpr int T = KD * KS * KS;
  static constexpr int S = (T * NB + 3) / 4;
  static constexpr int COB = WC * MT * 16;
  static constexpr int PLANES = KD + TD - 1;
  static constexpr int RH = TH + KS - 1, RW = 16 + KS - 1;
  static constexpr int PLANE = RH * RW;
  static constexpr int IMG = PLANES * PLANE;  // 16-B voxel-blocks per channel block
  // channel-block stride in LDS: a multiple of 16 slots, so the two blocks a ds_read_b128 lane
  // group reads (k-groups 2m, 2m + 1: NB = 2) sit on the same banks modulo their column and the
  // group's 16 columns stay on distinct ones (r06: IMG = 180 for the 2D tiles put them two-way,
  // half the LDS cycles of those launches were conflict cycles)
  static constexpr int IMGS = (IMG + 15) / 16 * 16;
  static constexpr int STAGE = NB * IMGS;     // 16-B slots per stage
  static constexpr int PIECES = (IMG + 63) / 64;
  static constexpr int PIECES_W = (PIECES + 3) / 4;
};

template <int KS, int MT, int WC, int TH, int TD, int NB, bool CV, int KD = KS>
__global__ __launch_bounds__(kThreads, 2) void conv_bf16_kernel(const Args a) {
  using C = Cfg<KS, MT, WC, TH, TD, NB, CV, KD>;
  // dynamic LDS: two stages, or one when the whole K is a single chunk (cin <= 16):
  // half the footprint doubles the workgroups per CU for the small cell layers
  extern __shared__ __attribute__((aligned(16))) bf16x8 smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wv = wave / WC;
  const int g = lane >> 4, n = lane & 15;

  // XCD-aware 1-D order as the f32 engine (conv3d_impl.h)
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = a.nblk / 8, r8 = a.nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int dz = lin % a.ndz;
  const int tile = (lin / a.ndz) % a.ntiles;
  const int bc = lin / (a.ndz * a.ntiles);
  const int b = bc / a.ncob, cob = bc - b * a.ncob;
  const int h0 = (tile / a.tiles_w) * TH, w0 = (tile % a.tiles_w) * 16, d0 = dz * TD;
  const int HW = a.H * a.W;
  const int DHW = HW * a.D;

  // per-lane byte offsets (within one channel block) of this wave's DMA pieces
  unsigned voff[C::PIECES_W], voffr[CV ? C::PIECES_W : 1];
#pragma unroll
  for (int t = 0; t < C::PIECES_W; ++t) {
    const int e = (wave + 4 * t) * 64 + lane;
    unsigned v = 0xFFFFFFF0u, vr = 0xFFFFFFF0u;
    if (e < C::IMG) {
      const int p = e / C::PLANE, r = e % C::PLANE;
      const int rr = r / C::RW, cc = r % C::RW;
      const int d = d0 + p - KD / 2, h = h0 + rr - KS / 2, w = w0 + cc - KS / 2;
      if ((unsigned)d < (unsigned)a.D && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
        if constexpr (CV) {
          if (w >= d) {
            v = (unsigned)(h * a.W + w) * 16u;
            vr = (unsigned)(h * a.W + w - d) * 16u;
          }
        } else {
          v = (unsigned)(d * HW + h * a.W + w) * 16u;
        }
      }
    }
    voff[t] = v;
    if constexpr (CV) voffr[t] = vr;
  }
  // plain locals: a lambda capturing the kernel-argument struct makes the
  // compiler copy it to scratch
  const int nblocks = a.cin / 8, cb1 = a.cb1;
  const __bf16* const xb1 = a.x + (long long)b * a.xbs;
  const __bf16* const xb2 = a.x2 + (long long)b * a.x2bs;
  const unsigned brec = (unsigned)(CV ? HW : DHW) * 16u;
  const long long bstride = (long long)(CV ? HW : DHW) * 8;
  auto issue = [&](int ch, bf16x8* st) {
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int blk = ch * NB + k;
      const __bf16* base = xb1;
      unsigned nrec = 0;
      if (blk < cb1) {
        base = xb1 + blk * bstride;
        nrec = brec;
      } else if (blk < nblocks) {
        base = xb2 + (blk - cb1) * bstride;
        nrec = brec;
      }
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nrec, 0x00020000);
      // right-image chunk: arithmetic select (a ?: between two register arrays
      // becomes a pointer select and sends both arrays to scratch)
      const unsigned rmask = (CV && blk >= cb1) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int t = 0; t < C::PIECES_W; ++t) {
        const int j = wave + 4 * t;
        unsigned vo = voff[t];
        if constexpr (CV) vo = voff[t] ^ ((voff[t] ^ voffr[t]) & rmask);
        if (j < C::PIECES && j * 64 + lane < C::IMG)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(st + k * C::IMGS + j * 64), 16, vo, 0, 0, 0);
      }
    }
  };

  // B fragment slot offset (in 16-B units) of k-step s for this lane
  auto boff = [&](int s) -> int {
    const int slot = 4 * s + g;
    const int tap = min(slot / NB, C::T - 1);  // slots past the last tap carry zero weights
    const int blk = slot % NB;
    const int kd = tap / (KS * KS), kh = (tap / KS) % KS, kw = tap % KS;
    return blk * C::IMGS + kd * C::PLANE + kh * C::RW + kw;
  };
  int vrow[C::NV];  // staged-halo slot of this wave's rows (output plane t, row r), column n
#pragma unroll
  for (int i = 0; i < C::NV; ++i) {
    const int q = wv * C::NV + i;
    const int t = q / TH, r = q % TH;
    vrow[i] = t * C::PLANE + r * C::RW + n;
  }

  const int mtile0 = wc * MT;
  const bf16x8* wpv = reinterpret_cast<const bf16x8*>(a.wp);
  f32x4 acc[MT][C::NV];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < C::NV; ++i) acc[m][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragments: a window of PF k-steps ahead in registers (the first PF issued
  // before the chunk's barrier so their L2 latency overlaps the halo DMA)
  constexpr int PF = C::S < 4 ? C::S : 4;
  issue(0, smem);
  for (int ch = 0; ch < a.nchunks; ++ch) {
    const long long wbase = ((long long)cob * a.nchunks + ch) * C::S * (WC * MT);
    auto wload = [&](int s, int m) {
      return wpv[((wbase + (long long)s * (WC * MT) + mtile0 + m) * 4 + g) * 16 + n];
    };
    bf16x8 av[C::S][MT];
#pragma unroll
    for (int s = 0; s < PF; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m) av[s][m] = wload(s, m);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ch + 1 < a.nchunks) issue(ch + 1, smem + ((ch + 1) & 1) * C::STAGE);
    const bf16x8* xs = smem + (ch & 1) * C::STAGE;
#pragma unroll
    for (int s = 0; s < C::S; ++s) {
      if (s + PF < C::S)
#pragma unroll
        for (int m = 0; m < MT; ++m) av[s + PF][m] = wload(s + PF, m);
      const int bo = boff(s);
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        const bf16x8 bv = xs[bo + vrow[i]];
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[s][m], bv, acc[m][i], 0, 0, 0);
      }
    }
  }

  // epilogue: lane holds couts 4g..4g+3 of each 16-row tile at voxel column n
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int co = cob * C::COB + (mtile0 + m) * 16 + 4 * g;  // first of 4
    if (co >= a.cout) continue;                                // cout % 4 == 0 (host)
    float sc[4], sh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = a.scale ? a.scale[co + r] : 1.f;
      sh[r] = a.shift ? a.shift[co + r] : 0.f;
    }
    const long long cofs = (long long)(co / 8) * DHW * 8 + (co % 8);
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      const int q = wv * C::NV + i;
      const int d = d0 + q / TH, h = h0 + q % TH, w = w0 + n;
      if (d >= a.D || h >= a.H || w >= a.W) continue;
      const long long o = cofs + ((long long)d * HW + h * a.W + w) * 8;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[m][i][r] * sc[r] + sh[r];
        if (relu) v[r] = fmaxf(v[r], 0.f);
      }
      if (resid) {
        const bf16x4 rv = *reinterpret_cast<const bf16x4*>(a.res + (long long)b * a.rbs + o);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
      }
      bf16x4 out;
#pragma unroll
      for (int r = 0; r < 4; ++r) out[r] = (__bf16)v[r];
      *reinterpret_cast<bf16x4*>(a.y + (long long)b * a.ybs + o) = out;
    }
  }
}

// weights [cout][cin][k^3] f32 -> [cob][chunk][s][mtile][g][16][8] bf16
__global__ void pack_bf16_kernel(const float* __restrict__ w, __bf16* __restrict__ packed, int cout,
                                 int cin, int T, int nb, int S, int mtiles, int nchunks,
                                 long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long r = i;
    const int j = (int)(r % 8); r /= 8;
    const int n = (int)(r % 16); r /= 16;
    const int g = (int)(r % 4); r /= 4;
    const int mt = (int)(r % mtiles); r /= mtiles;
    const int s = (int)(r % S); r /= S;
    const int ch = (int)(r % nchunks);
    const int cob = (int)(r / nchunks);
    const int slot = 4 * s + g;
    const int tap = slot / nb, blk = slot % nb;
    const int co = cob * mtiles * 16 + mt * 16 + n;
    const int ci = (ch * nb + blk) * 8 + j;
    float v = 0.f;
    if (tap < T && co < cout && ci < cin) v = w[((long long)co * cin + ci) * T + tap];
    packed[i] = (__bf16)v;
  }
}

// f32 NCDHW (batch stride xbs) <-> bf16 c8 layout converters
__global__ void to_c8_kernel(const float* __restrict__ x, long long xbs, __bf16* __restrict__ y,
                             long long ybs, int C, long long vol) {
  const int b = blockIdx.y;
  const long long nvox = vol * (C / 8);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvox;
       i += (long long)gridDim.x * blockDim.x) {
    const long long cb = i / vol, v = i % vol;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__bf16)x[(long long)b * xbs + (cb * 8 + j) * vol + v];
    reinterpret_cast<bf16x8*>(y + (long long)b * ybs)[i] = o;
  }
}

__global__ void from_c8_kernel(const __bf16* __restrict__ x, long long xbs, float* __restrict__ y,
                               long long ybs, int C, long long vol) {
  const int b = blockIdx.y;
  const long long nvox = vol * (C / 8);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvox;
       i += (long long)gridDim.x * blockDim.x) {
    const long long cb = i / vol, v = i % vol;
    const bf16x8 o = reinterpret_cast<const bf16x8*>(x + (long long)b * xbs)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[(long long)b * ybs + (cb * 8 + j) * vol + v] = (float)o[j];
  }
}

// Trilinear resample (aten source-index rule, common.h Axis) of a c8 volume with
// the optional per-channel relu(scale * . + shift) epilogue; 16-byte voxel blocks (8
// channels) per output word: 8 corner words, interpolated in f32.  K output words per
// thread (grid stride apart), all 8K corner loads issued before the first lerp: K = 1
// keeps the most loads in flight chip-wide for the read-heavy down-samplings, K = 4
// cuts the workgroup count of the write-heavy up-samplings (r02: one word per thread
// launched 123 K workgroups for an L1 -> L0 8-channel up-sampling and ran at 1.9 TB/s,
// dispatch-bound).
template <int K>
__global__ __launch_bounds__(256) void resample_c8_kernel(
    const __bf16* __restrict__ x, long long xbs, __bf16* __restrict__ y, long long ybs, int CB,
    int Di, int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh, float rw, int ac,
    const float* __restrict__ scale, const float* __restrict__ shift, unsigned flags) {
#pragma clang fp contract(off)
  const int plane = blockIdx.y;  // (b * CB + cb) * Do + od
  const int od = plane % Do;
  const int bcb = plane / Do;
  const int b = bcb / CB, cb = bcb % CB;
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const long long HWi = (long long)Hi * Wi;
  const bf16x8* xc = reinterpret_cast<const bf16x8*>(x + (long long)b * xbs) + (long long)cb * Di * HWi;
  bf16x8* yp = reinterpret_cast<bf16x8*>(y + (long long)b * ybs) + ((long long)cb * Do + od) * Ho * Wo;
  const bf16x8* p0 = xc + ad.i0 * HWi;
  const bf16x8* p1 = xc + ad.i1 * HWi;
  const bool relu = flags & LEA_RELU;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale ? scale[cb * 8 + j] : 1.f;
    sh[j] = scale ? shift[cb * 8 + j] : 0.f;
  }
  // XCD-aware order of the plane's workgroups (dispatch round-robins blockIdx over the
  // 8 XCDs): XCD x takes the contiguous x-th eighth of the rows, so its L2 holds only
  // that eighth of the source rows (r02: 3.4x fetch amplification on the up-samplings
  // with the plain order)
  const int nbx = gridDim.x;
  const int q8 = nbx / 8, r8 = nbx % 8, xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int bx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int cells = Ho * Wo;
  const int span = (cells + nbx - 1) / nbx;  // contiguous outputs per workgroup
  const int tend = min(cells, (bx + 1) * span);
  for (int t0 = bx * span + threadIdx.x; t0 < tend; t0 += K * (int)blockDim.x) {
    bf16x8 c[K][8];
    Axis ah[K], aw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = min(t0 + k * (int)blockDim.x, tend - 1);
      const int oh = t / Wo, ow = t % Wo;
      ah[k] = axis_index(rh, oh, Hi, Ho, ac);
      aw[k] = axis_index(rw, ow, Wi, Wo, ac);
      const long long r0 = (long long)ah[k].i0 * Wi, r1 = (long long)ah[k].i1 * Wi;
      c[k][0] = p0[r0 + aw[k].i0];
      c[k][1] = p0[r0 + aw[k].i1];
      c[k][2] = p0[r1 + aw[k].i0];
      c[k][3] = p0[r1 + aw[k].i1];
      c[k][4] = p1[r0 + aw[k].i0];
      c[k][5] = p1[r0 + aw[k].i1];
      c[k][6] = p1[r1 + aw[k].i0];
      c[k][7] = p1[r1 + aw[k].i1];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = t0 + k * (int)blockDim.x;
      if (t >= tend) break;
      const Axis &h = ah[k], &w = aw[k];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float r = ad.l0 * (h.l0 * (w.l0 * (float)c[k][0][j] + w.l1 * (float)c[k][1][j]) +
                           h.l1 * (w.l0 * (float)c[k][2][j] + w.l1 * (float)c[k][3][j])) +
                  ad.l1 * (h.l0 * (w.l0 * (float)c[k][4][j] + w.l1 * (float)c[k][5][j]) +
                           h.l1 * (w.l0 * (float)c[k][6][j] + w.l1 * (float)c[k][7][j]));
        if (scale) r = r * sc[j] + sh[j];
        if (relu) r = fmaxf(r, 0.f);
        o[j] = (__bf16)r;
      }
      yp[t] = o;
    }
  }
}

// Up-sampling form (r05; the default when the output volume is the larger): a wave owns 64
// consecutive output columns of R consecutive output rows of one output plane and walks
// down the rows.  Each source row it needs is loaded once per wave (the two corner words
// of each column in both source planes) and W-lerped into registers (aw.l0 * x[i0] +
// aw.l1 * x[i1], trilerp's innermost terms); consecutive output rows of an up-sampling share
// their source rows, so a row is lerped once for ~2 output rows.  Per output word: ~2
// 16-byte loads instead of the gather kernel's 8, ~5 lerp ops per channel instead of 7, the
// same expression tree (fp contraction off): bit-identical to resample_c8_kernel.
template <int R>
__global__ __launch_bounds__(256) void resample_c8_cols_kernel(
    const __bf16* __restrict__ x, long long xbs, __bf16* __restrict__ y, long long ybs, int CB,
    int Di, int Hi, int Wi, int Do, int Ho, int Wo, float rd, float rh, float rw, int ac,
    const float* __restrict__ scale, const float* __restrict__ shift, unsigned flags, int ctiles) {
#pragma clang fp contract(off)
  const int plane = blockIdx.y;  // (b * CB + cb) * Do + od
  const int od = plane % Do;
  const int bcb = plane / Do;
  const int b = bcb / CB, cb = bcb % CB;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ct = blockIdx.x % ctiles, rblk = blockIdx.x / ctiles;
  const int oh0 = (rblk * 4 + wave) * R;
  if (oh0 >= Ho) return;  // whole waves only
  const int oh1 = min(oh0 + R, Ho);
  const int ow = ct * 64 + lane;
  const bool active = ow < Wo;
  const Axis ad = axis_index(rd, od, Di, Do, ac);
  const Axis aw = axis_index(rw, active ? ow : Wo - 1, Wi, Wo, ac);
  const long long HWi = (long long)Hi * Wi;
  const bf16x8* xc = reinterpret_cast<const bf16x8*>(x + (long long)b * xbs) + (long long)cb * Di * HWi;
  bf16x8* yp = reinterpret_cast<bf16x8*>(y + (long long)b * ybs) + ((long long)cb * Do + od) * Ho * Wo;
  const bf16x8* p0 = xc + ad.i0 * HWi;
  const bf16x8* p1 = xc + ad.i1 * HWi;
  const bool relu = flags & LEA_RELU;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale ? scale[cb * 8 + j] : 1.f;
    sh[j] = scale ? shift[cb * 8 + j] : 0.f;
  }
  // walk the source rows r_lo .. r_hi the wave's output rows read, the next row's four corner
  // words loaded one row ahead; after row r is W-lerped, every output row whose upper source
  // row (ah.i1) is r is complete: its lower row is r - 1 (or r itself at the last row)
  const long long rs = (long long)Wi;
  auto load_row = [&](int r, bf16x8* q) {
    const long long o = (long long)r * rs;
    q[0] = p0[o + aw.i0];
    q[1] = p0[o + aw.i1];
    q[2] = p1[o + aw.i0];
    q[3] = p1[o + aw.i1];
  };
  Axis ah = axis_index(rh, oh0, Hi, Ho, ac);
  const int r_lo = ah.i0, r_hi = axis_index(rh, oh1 - 1, Hi, Ho, ac).i1;
  bf16x8 nxt[4];
  load_row(r_lo, nxt);
  float lo[2][8], hi[2][8];  // W-lerped rows r - 1 and r, both source planes
  int oh = oh0;
  for (int r = r_lo; r <= r_hi; ++r) {  // wave-uniform
    bf16x8 cur[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    if (r < r_hi) load_row(r + 1, nxt);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lo[0][j] = hi[0][j];
      lo[1][j] = hi[1][j];
      hi[0][j] = aw.l0 * (float)cur[0][j] + aw.l1 * (float)cur[1][j];
      hi[1][j] = aw.l0 * (float)cur[2][j] + aw.l1 * (float)cur[3][j];
    }
    for (; oh < oh1 && ah.i1 == r; ah = axis_index(rh, ++oh, Hi, Ho, ac)) {
      const bool same = ah.i0 == r;  // the last source row pairs with itself
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a0 = same ? hi[0][j] : lo[0][j], a1 = same ? hi[1][j] : lo[1][j];
        float v = ad.l0 * (ah.l0 * a0 + ah.l1 * hi[0][j]) + ad.l1 * (ah.l0 * a1 + ah.l1 * hi[1][j]);
        if (scale) v = v * sc[j] + sh[j];
        if (relu) v = fmaxf(v, 0.f);
        o[j] = (__bf16)v;
      }
      if (active) yp[(long long)oh * Wo + ow] = o;
    }
  }
}

// ---- 1x1 conv of a trilinearly resampled c8 input (align_corners=True): the cell
// preprocess after a level change (skip_model_3d.py:44-53) without materialising the
// resampled tensor.  A gather-GEMM: lane (g, n) of a wave forms its own B fragment of
// v_mfma_f32_16x16x32_bf16 -- channel block g of output voxel n, i.e. one 16-byte word
// of the resampled input -- from the 8 corner words (the resample_c8 expression,
// rounded to bf16 the same way), so no LDS; the A fragments (the k = 1 packing: one
// k-step per 32-channel chunk) sit in registers.  Bit-identical to resample_c8 + the
// 1x1 tile kernel; saves the resampled tensor's write and read.
// NCH = cin / 32 at compile time (1, 2; 4 covers 96 and 128 with a runtime count) so the
// corner words are sized to the layer, and a wave issues the corner loads of TU tiles before
// their MFMAs (r05: 196 VGPRs at two waves per SIMD with one tile in flight before).
template <int MT, int NCH, int TU>
__global__ __launch_bounds__(256) void conv1x1_rs_c8_kernel(
    const __bf16* __restrict__ x, long long xbs, int Di, int Hi, int Wi, const bf16x8* __restrict__ wp,
    const float* __restrict__ scale, const float* __restrict__ shift, __bf16* __restrict__ y,
    long long ybs, int cin, int cout, int Do, int Ho, int Wo, float rd, float rh, float rw,
    unsigned flags, int tiles_per_wave) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, n = lane & 15;
  const int b = blockIdx.y;
  const int nch = NCH < 4 ? NCH : cin / 32;
  const long long HWi = (long long)Hi * Wi, vin = HWi * Di;
  const int HWo = Ho * Wo;
  const long long vout = (long long)HWo * Do;
  const bf16x8* xb = reinterpret_cast<const bf16x8*>(x + (long long)b * xbs);
  // A fragments of every chunk and cout tile (cob block of 16 MT couts: [chunk][s][mtile][g][16])
  bf16x8 av[NCH][MT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int m = 0; m < MT; ++m) av[c][m] = c < nch ? wp[((c * MT + m) * 4 + g) * 16 + n] : bf16x8{};
  float sc[MT][4], sh[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * m + 4 * g + r;
      sc[m][r] = (scale && co < cout) ? scale[co] : 1.f;
      sh[m][r] = (scale && co < cout) ? shift[co] : 0.f;
    }
  const bool relu = flags & LEA_RELU;
  const long long tile0 = ((long long)blockIdx.x * 4 + wave) * tiles_per_wave;
  for (int tt = 0; tt < tiles_per_wave; tt += TU) {
    if ((tile0 + tt) * 16 >= vout) break;
    bf16x8 cw[TU][NCH][8];
    Axis ad[TU], ah[TU], aw[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      // tiles past the wave's share or the volume load the last voxel's corners (never stored)
      const long long v = min((tile0 + tt + u) * 16 + n, vout - 1);
      const int od = (int)(v / HWo), rem = (int)(v - (long long)od * HWo);
      const int oh = rem / Wo, ow = rem - oh * Wo;
      ad[u] = axis_index(rd, od, Di, Do, 1);
      ah[u] = axis_index(rh, oh, Hi, Ho, 1);
      aw[u] = axis_index(rw, ow, Wi, Wo, 1);
      const long long o00 = (long long)ad[u].i0 * HWi + (long long)ah[u].i0 * Wi;
      const long long o01 = (long long)ad[u].i0 * HWi + (long long)ah[u].i1 * Wi;
      const long long o10 = (long long)ad[u].i1 * HWi + (long long)ah[u].i0 * Wi;
      const long long o11 = (long long)ad[u].i1 * HWi + (long long)ah[u].i1 * Wi;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c >= nch) break;
        const bf16x8* xc = xb + (long long)(4 * c + g) * vin;
        cw[u][c][0] = xc[o00 + aw[u].i0];
        cw[u][c][1] = xc[o00 + aw[u].i1];
        cw[u][c][2] = xc[o01 + aw[u].i0];
        cw[u][c][3] = xc[o01 + aw[u].i1];
        cw[u][c][4] = xc[o10 + aw[u].i0];
        cw[u][c][5] = xc[o10 + aw[u].i1];
        cw[u][c][6] = xc[o11 + aw[u].i0];
        cw[u][c][7] = xc[o11 + aw[u].i1];
      }
    }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const long long v0 = (tile0 + tt + u) * 16;
      if (tt + u >= tiles_per_wave || v0 >= vout) break;
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c >= nch) break;
        bf16x8 bv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const Axis &pd = ad[u], &ph = ah[u], &pw = aw[u];
          const float r = pd.l0 * (ph.l0 * (pw.l0 * (float)cw[u][c][0][j] + pw.l1 * (float)cw[u][c][1][j]) +
                                   ph.l1 * (pw.l0 * (float)cw[u][c][2][j] + pw.l1 * (float)cw[u][c][3][j])) +
                          pd.l1 * (ph.l0 * (pw.l0 * (float)cw[u][c][4][j] + pw.l1 * (float)cw[u][c][5][j]) +
                                   ph.l1 * (pw.l0 * (float)cw[u][c][6][j] + pw.l1 * (float)cw[u][c][7][j]));
          bv[j] = (__bf16)r;
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][m], bv, acc[m], 0, 0, 0);
      }
      if (v0 + n >= vout) continue;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int co = 16 * m + 4 * g;  // first of the lane's 4 couts
        if (co >= cout) continue;
        bf16x4 out;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = acc[m][r] * sc[m][r] + sh[m][r];
          if (relu) t = fmaxf(t, 0.f);
          out[r] = (__bf16)t;
        }
        *reinterpret_cast<bf16x4*>(y + (long long)b * ybs + ((long long)(co / 8) * vout + v0 + n) * 8 + co % 8) = out;
      }
    }
  }
}

// ---- 1x1 ConvBR on c8 tensors, streamed (conv1x1_rs_c8_kernel without the resample): a
// 1x1 conv reads every input word once, so nothing is staged -- lane (g, n) loads its own
// B fragment (channel block 4 c + g of voxel v0 + n, one 16-byte word) straight into
// registers, the A fragments (the k = 1 packing) sit in registers, and a wave issues the
// words of TU tiles before their MFMAs so TU * nch loads per lane are in flight.  Same
// operands, order and epilogue as the tile kernel's k = 1 path: bit-identical.
// NCH = the 32-channel chunk count at compile time (1, 2; 4 covers 3 and 4 at run time): r05,
// 114 -> fewer VGPRs for the one- and two-chunk layers
template <int MT, int NCH>
__global__ __launch_bounds__(256) void conv1x1_c8_kernel(const Args a, int tpw) {
  constexpr int MAXCH = NCH, TU = 4;  // cin <= 128 (host); tiles per load group
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, n = lane & 15;
  const int b = blockIdx.y / a.ncob, cob = blockIdx.y - b * a.ncob;
  const int nch = NCH < 4 ? NCH : (a.cin / 8 + 3) / 4;
  const long long vox = (long long)a.D * a.H * a.W;
  const bf16x8* wp = reinterpret_cast<const bf16x8*>(a.wp);
  bf16x8 av[MAXCH][MT];
#pragma unroll
  for (int c = 0; c < MAXCH; ++c)
#pragma unroll
    for (int m = 0; m < MT; ++m)
      av[c][m] = c < nch ? wp[((((long long)cob * nch + c) * MT + m) * 4 + g) * 16 + n] : bf16x8{};
  const int co0 = cob * 16 * MT;
  float sc[MT][4], sh[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * m + 4 * g + r;
      sc[m][r] = (a.scale && co < a.cout) ? a.scale[co] : 1.f;
      sh[m][r] = (a.shift && co < a.cout) ? a.shift[co] : 0.f;
    }
  const bool relu = a.flags & LEA_RELU, resid = a.flags & LEA_RESIDUAL;
  // this lane's channel block of chunk c: source pointer (x or the cat's second tensor)
  const bf16x8* src[MAXCH];
  bool live[MAXCH];
#pragma unroll
  for (int c = 0; c < MAXCH; ++c) {
    const int blk = 4 * c + g;
    live[c] = c < nch && blk < a.cin / 8;
    src[c] = blk < a.cb1 ? reinterpret_cast<const bf16x8*>(a.x + (long long)b * a.xbs) + (long long)blk * vox
                         : reinterpret_cast<const bf16x8*>(a.x2 + (long long)b * a.x2bs) + (long long)(blk - a.cb1) * vox;
  }
  const long long t0 = ((long long)blockIdx.x * 4 + wave) * tpw;
  for (int tt = 0; tt < tpw; tt += TU) {
    bf16x8 bw[TU][MAXCH];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const long long v = min((t0 + tt + u) * 16 + n, vox - 1);
#pragma unroll
      for (int c = 0; c < MAXCH; ++c) bw[u][c] = (live[c] && tt + u < tpw) ? src[c][v] : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const long long v0 = (t0 + tt + u) * 16;
      if (tt + u >= tpw || v0 >= vox) break;
      f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < MAXCH; ++c) {
        if (c >= nch) break;
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][m], bw[u][c], acc[m], 0, 0, 0);
      }
      if (v0 + n >= vox) continue;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int co = co0 + 16 * m + 4 * g;  // first of the lane's 4 couts
        if (co >= a.cout) continue;
        const long long o = ((long long)(co / 8) * vox + v0 + n) * 8 + co % 8;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[m][r] * sc[m][r] + sh[m][r];
          if (relu) v[r] = fmaxf(v[r], 0.f);
        }
        if (resid) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(a.res + (long long)b * a.rbs + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
        }
        bf16x4 out;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = (__bf16)v[r];
        *reinterpret_cast<bf16x4*>(a.y + (long long)b * a.ybs + o) = out;
      }
    }
  }
}

// ---- D-streaming form for the single-chunk 3x3x3 layers (cin <= 16: the whole K is
// one chunk).  The tile kernel above stages a (TH+2) x 18 x (TD+2) halo per TH x 16 x TD
// tile and waits for it: r01 counters put these layers' waves 60-78 % parked on that
// DMA, with 2.1-2.8x halo re-reads.  Here a workgroup owns one (16 W x TH H) column
// and walks D two output planes per step through an LDS ring of 8 input planes:
// step s uses planes 2s-1 .. 2s+2 and issues planes 2s+5, 2s+6 (two steps ahead) as
// inline-asm LDS-DMA (invisible to the compiler's vmcnt bookkeeping; the kernel
// waits with counted vmcnt), so each input plane is fetched once per column (halo
// re-reads (TH+2)/TH along H only) and the fetch of step s+2 overlaps steps s, s+1.
// The weights (one chunk) sit in registers for the whole walk; the residual /
// accumulate operand of each step is LDS-DMA'd by the wave that consumes it (no
// barrier), and BN scale/shift are read once, so no compiler-visible load inside the
// walk drains the prefetch.
template <int MT, int WC, int TH, int NB, int NCH>
struct SCfg {
  static constexpr int TD = 2, WV = 4 / WC, VT = TH * TD, NV = VT / WV;
  static_assert(VT % WV == 0, "rows per wave");
  static constexpr int T = 27, S = (T * NB + 3) / 4;             // k-steps per chunk
  static constexpr int NBK = NB * NCH;                           // channel blocks in the ring
  static constexpr int COB = WC * MT * 16;
  static constexpr int RH = TH + 2, RW = 18, PLANE = RH * RW;   // 16-B words per plane and block
  static constexpr int PIECES = (PLANE + 63) / 64;              // 64-word DMA pieces per plane and block
  static constexpr int PLANEP = 64 * PIECES;
  static constexpr int SLOTW = NBK * PLANEP;                     // words per ring slot
  static constexpr int PPW = (NBK * PIECES + 3) / 4;             // pieces per wave and plane (padded)
  static constexpr int RING = 8;
  static constexpr int RESW = MT * 2 * NV * 16;                  // residual words per wave and step
  static constexpr int RPW = RESW / 64;                          // residual pieces per wave
  static constexpr int RINGW = RING * SLOTW + 64 * (4 * PPW - NBK * PIECES);  // + padding pieces
  static constexpr int LDSW = RINGW + 4 * 2 * RESW;  // with two residual slots per wave (dynamic LDS)
  // B-fragment prefetch distance in k-steps (r05): as deep as keeps 4 waves per SIMD (<= 128
  // VGPRs) on the one-chunk 16-cout forms; 2 on the two-chunk forms (two waves per SIMD
  // already: 204 / 240 VGPRs; same box C4 +1.3-2 %, 3 was no better); 0 = the compiler's
  // schedule (one MFMA pair ahead)
#ifdef LEA_BF_PF
  static constexpr int PF = LEA_BF_PF;
#else
  static constexpr int PF = (WC == 1 && MT == 1 && NCH == 1) ? (NB == 2 ? 3 : 2) : (NCH == 2 ? 2 : 0);
#endif
  static_assert(RESW % 64 == 0, "whole residual pieces");
  static_assert(LDSW * 16 <= 96 * 1024, "ring + residual");
};

__device__ __forceinline__ void dma_x4(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MT, int WC, int TH, int NB, int NCH>
__global__ __launch_bounds__(kThreads, 2) void conv_bf16_stream_kernel(const Args a, int nsplit) {
  using C = SCfg<MT, WC, TH, NB, NCH>;
  extern __shared__ __attribute__((aligned(16))) bf16x8 smem[];  // RINGW (+ residual slots)
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wv = wave / WC;
  const int g = lane >> 4, n = lane & 15;

  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = a.nblk / 8, r8 = a.nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int sp = lin % nsplit;
  const int tile = (lin / nsplit) % a.ntiles;
  const int bc = lin / (nsplit * a.ntiles);
  const int b = bc / a.ncob, cob = bc - b * a.ncob;
  const int h0 = (tile / a.tiles_w) * TH, w0 = (tile % a.tiles_w) * 16;
  const int HW = a.H * a.W;
  const int DHW = HW * a.D;
  const int nst = (a.D + 1) / 2;
  const int s0 = sp * nst / nsplit, s1 = (sp + 1) * nst / nsplit;

  // DMA pieces of one plane: piece q = wave + 4t -> (block q / PIECES, words 64 (q % PIECES)
  // + lane); one buffer resource over the batch element's blocks (host: < 4 GiB)
  // (LEA_PAIR_SUM: blocks [cb1, cin / 8) come from the second source, offsets relative to it)
  unsigned hwo[C::PPW];
  unsigned ldo[C::PPW];
  bool src2[C::PPW];
#pragma unroll
  for (int t = 0; t < C::PPW; ++t) {
    const int q = wave + 4 * t;
    const int blk = q / C::PIECES, e = (q % C::PIECES) * 64 + lane;
    src2[t] = blk >= a.cb1;  // wave-uniform
    const int sblk = src2[t] ? blk - a.cb1 : blk;
    unsigned v = 0xFFFFFFF0u;
    if (q < C::NBK * C::PIECES && e < C::PLANE && blk * 8 < a.cin) {
      const int rr = e / C::RW, cc = e % C::RW;
      const int h = h0 + rr - 1, w = w0 + cc - 1;
      if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        v = (unsigned)sblk * (unsigned)DHW * 16u + (unsigned)(h * a.W + w) * 16u;
    }
    hwo[t] = v;
    // padding pieces (q >= NBK * PIECES) land past the ring
    ldo[t] = q < C::NBK * C::PIECES ? (unsigned)(blk * C::PLANEP + (q % C::PIECES) * 64)
                                    : (unsigned)(C::RING * C::SLOTW + (q - C::NBK * C::PIECES) * 64);
  }
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)b * a.xbs), 0, (unsigned)a.cb1 * (unsigned)DHW * 16u, 0x00020000);
  const __amdgpu_buffer_rsrc_t x2rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x2 ? a.x2 + (long long)b * a.x2bs : a.x), 0,
      a.x2 ? (unsigned)(a.cin / 8 - a.cb1) * (unsigned)DHW * 16u : 0u, 0x00020000);
  auto load_plane = [&](int d) {  // plane d (zeros outside 0..D-1) -> ring slot d & 7
    const bool dv = (unsigned)d < (unsigned)a.D;
    const unsigned slot = (unsigned)(d & 7) * C::SLOTW;
#pragma unroll
    for (int t = 0; t < C::PPW; ++t) {
      const unsigned vo = (dv && hwo[t] != 0xFFFFFFF0u) ? hwo[t] + (unsigned)d * (unsigned)HW * 16u : 0xFFFFFFF0u;
      const unsigned dst = ldo[t] < (unsigned)(C::RING * C::SLOTW) ? slot + ldo[t] : ldo[t];
      dma_x4(src2[t] ? x2rs : xrs, vo, lds0 + 16u * dst);
    }
  };

  // this wave's residual words per step: (m-tile, block of its 2, row i, column) -> its own
  // slot s & 1; one resource over the batch element's output blocks
  const bool resid = a.flags & LEA_RESIDUAL;
  const unsigned resbase = (unsigned)(C::RINGW + wave * 2 * C::RESW);
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.res + (long long)b * a.rbs), 0, (unsigned)((a.cout + 7) / 8) * (unsigned)DHW * 16u, 0x00020000);
  auto load_res = [&](int s) {
    const unsigned rslot = resbase + (unsigned)(s & 1) * C::RESW;
#pragma unroll
    for (int t = 0; t < C::RPW; ++t) {
      const int e = t * 64 + lane;  // word: ((m * 2 + blk2) * NV + i) * 16 + col
      const int col = e % 16, i = (e / 16) % C::NV, mb = e / (16 * C::NV);
      const int m = mb / 2, blk2 = mb % 2;
      const int qrow = wv * C::NV + i;
      const int d = 2 * s + qrow / TH, h = h0 + qrow % TH, w = w0 + col;
      const int cblk = (cob * C::COB + (wc * MT + m) * 16) / 8 + blk2;
      unsigned vo = 0xFFFFFFF0u;
      if (d < a.D && h < a.H && w < a.W && cblk * 8 < a.cout)
        vo = (unsigned)cblk * (unsigned)DHW * 16u + (unsigned)(d * HW + h * a.W + w) * 16u;
      dma_x4(rrs, vo, lds0 + 16u * (rslot + (unsigned)t * 64u));
    }
  };

  // per-lane K slot geometry: k-step ks of a chunk, lane group g -> tap (kd, kh, kw), block
  int kdv[C::S], koff[C::S];
#pragma unroll
  for (int ks = 0; ks < C::S; ++ks) {
    const int slot = 4 * ks + g;
    const int tap = min(slot / NB, C::T - 1);  // slots past the last tap carry zero weights
    const int blk = slot % NB;
    kdv[ks] = tap / 9;
    koff[ks] = blk * C::PLANEP + ((tap / 3) % 3) * C::RW + tap % 3;
  }
  // A fragments of every chunk, resident for the whole walk
  const int mtile0 = wc * MT;
  const bf16x8* wpv = reinterpret_cast<const bf16x8*>(a.wp);
  bf16x8 av[NCH][C::S][MT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int ks = 0; ks < C::S; ++ks)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        av[c][ks][m] = wpv[((((long long)cob * NCH + c) * C::S + ks) * (WC * MT) + mtile0 + m) * 64 + g * 16 + n];
  // LEA_PAIR_SUM: chunks [0, NCH / 2) are conv a's (BN at scale[co]), the rest conv b's
  // (BN at scale[cout + co]); a's activation is kept in registers until b's epilogue
  // (sc / sh: the final epilogue's BN -- conv b's under LEA_PAIR_SUM; sca / sha: conv a's; static
  // indices only: a runtime-indexed register array is placed in scratch memory)
  const bool pair = a.flags & LEA_PAIR_SUM;
  float sc[MT][4], sh[MT][4], sca[MT][4], sha[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cob * C::COB + (mtile0 + m) * 16 + 4 * g + r;
      const bool cv = co < a.cout;
      const int o = (pair ? a.cout : 0) + co;
      sc[m][r] = (a.scale && cv) ? a.scale[o] : 1.f;
      sh[m][r] = (a.shift && cv) ? a.shift[o] : 0.f;
      sca[m][r] = (a.scale && cv && NCH % 2 == 0) ? a.scale[co] : 1.f;
      sha[m][r] = (a.shift && cv && NCH % 2 == 0) ? a.shift[co] : 0.f;
    }
  const bool relu = a.flags & LEA_RELU;
  // the output through one buffer resource: every lane issues the same MT * NV 8-byte stores
  // per step (invalid ones at an out-of-range offset: dropped), so the waits can count them
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.y + (long long)b * a.ybs), 0, (unsigned)((a.cout + 7) / 8) * (unsigned)DHW * 16u, 0x00020000);

  // Pipeline (issue order = completion order for vmcnt): after step s's barrier the wave
  // issues step s+1's residual into its slot (s+1) & 1, then planes 2s+5, 2s+6 (into the
  // slots of planes 2s-3, 2s-2, which only step s-1 read), and step s's MT * NV stores at
  // its end (r05: the planes used to follow the stores, so the top of step s+1 waited for
  // step s's stores).  The top of step s+1 waits for all but planes 2s+5, 2s+6 and the
  // stores -- i.e. for step s+1's planes (issued after step s-1's barrier) and residual.
  if (resid) load_res(s0);
  for (int j = -1; j <= 4; ++j) load_plane(2 * s0 + j);
  for (int s = s0; s < s1; ++s) {
    if (s > s0)
      wait_vm<2 * C::PPW + MT * C::NV>();
    else
      wait_vm<2 * C::PPW>();
    __syncthreads();  // everyone's planes landed; everyone done with step s-1
    if (resid && s + 1 < s1) load_res(s + 1);
    load_plane(2 * s + 5);
    load_plane(2 * s + 6);
    f32x4 acc[MT][C::NV];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < C::NV; ++i) acc[m][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int base = 2 * s - 1;
    float va[MT][C::NV][4];  // LEA_PAIR_SUM: conv a's activation
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      auto ldb = [&](int ks, int i) {
        const int qrow = wv * C::NV + i;
        const int t = qrow / TH, r = qrow % TH;
        return smem[((base + t + kdv[ks]) & 7) * C::SLOTW + c * NB * C::PLANEP + koff[ks] + r * C::RW + n];
      };
      if constexpr (C::PF > 0) {
        // B fragments PF k-steps ahead of their MFMAs, in that issue order
        bf16x8 bq[C::S][C::NV];
#pragma unroll
        for (int ks = 0; ks < C::PF && ks < C::S; ++ks)
#pragma unroll
          for (int i = 0; i < C::NV; ++i) bq[ks][i] = ldb(ks, i);
#pragma unroll
        for (int ks = 0; ks < C::S; ++ks) {
          if (ks + C::PF < C::S)
#pragma unroll
            for (int i = 0; i < C::NV; ++i) bq[ks + C::PF][i] = ldb(ks + C::PF, i);
#pragma unroll
          for (int i = 0; i < C::NV; ++i)
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[m][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][ks][m], bq[ks][i], acc[m][i], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < C::S; ++ks)
#pragma unroll
          for (int i = 0; i < C::NV; ++i) {
            const bf16x8 bv = ldb(ks, i);
#pragma unroll
            for (int m = 0; m < MT; ++m)
              acc[m][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][ks][m], bv, acc[m][i], 0, 0, 0);
          }
      }
      if (NCH % 2 == 0 && c == NCH / 2 - 1 && pair) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int i = 0; i < C::NV; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[m][i][r] * sca[m][r] + sha[m][r];
              va[m][i][r] = relu ? fmaxf(v, 0.f) : v;
            }
            acc[m][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
    }
    const unsigned rslot = resbase + (unsigned)(s & 1) * C::RESW;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int co = cob * C::COB + (mtile0 + m) * 16 + 4 * g;
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        const int qrow = wv * C::NV + i;
        const int d = 2 * s + qrow / TH, h = h0 + qrow % TH, w = w0 + n;
        const bool ok = d < a.D && h < a.H && w < a.W && co < a.cout;
        const unsigned off = ok ? (unsigned)(co / 8) * (unsigned)DHW * 16u + (unsigned)(co % 8) * 2u +
                                      (unsigned)(d * HW + h * a.W + w) * 16u
                                : 0xFFFFFFF0u;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[m][i][r] * sc[m][r] + sh[m][r];
          if (relu) v[r] = fmaxf(v[r], 0.f);
          if (NCH % 2 == 0 && pair) v[r] = va[m][i][r] + v[r];  // conv a's term + conv b's
        }
        if (resid) {
          // word ((m * 2 + 4g / 8) * NV + i) * 16 + n of this wave's slot, bf16 (4g) % 8 on
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(
              reinterpret_cast<const __bf16*>(smem + rslot + ((m * 2 + (4 * g) / 8) * C::NV + i) * 16 + n) + (4 * g) % 8);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
        }
        bf16x4 out;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = (__bf16)v[r];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, out), yrs, off, 0, 0);
      }
    }
  }
  wait_vm<0>();  // no LDS-DMA may outlive the workgroup
}

// LEA_PAIR_SUM (a matching-cell step: relu(BN_a(conv_a(xa))) + relu(BN_b(conv_b(xb))), one K chunk
// per conv) on the D-streaming form with the two convs on separate wave halves (r05): 8 waves, waves
// 0-3 run conv a and 4-7 conv b over the same 16 x TH x 2 tile rows (wave w and w + 4 on one
// SIMD), so each wave holds ONE chunk's A fragments -- the single-wave-group form held both
// (184 VGPRs: two waves per SIMD, 2.5 TB/s on the L1 steps).  Conv a's activation goes to LDS as
// bf16 (the rounding the two-launch form applies to a's output), and the conv-b wave adds it in
// its epilogue of step s, deferred to after the next step's barrier; the ring holds both
// sources' planes (blocks a0..a(NB-1), b0..b(NB-1) per slot).
// PP (the 8 -> 8 steps, cout <= 8, NB = 1; r05): "plane-paired" M rows -- the MFMA's 16 rows are
// the 8 couts of output plane 2s (rows 0-7) and of plane 2s+1 (rows 8-15), so one 16 x 16 tile
// covers both planes of an H row and no row is the zero padding of an 8-cout block.  K runs over
// the 4 input planes 2s-1 .. 2s+2 (36 (plane, kh, kw) slots = 9 k-steps instead of 7 per plane
// pair's rows: 9 MFMAs and B reads per H row and step instead of 14); rows 0-7 take kd = plane - 0,
// rows 8-15 kd = plane - 1 (zero outside 0..2).  Those A fragments are gathered once from the
// ordinary packing (each is one of its 16-byte words, or zero), so the weights need no own layout.
template <int TH, int NB, bool PP = false>
struct PCfg {
  static constexpr int TD = 2, VT = TH * TD;
  static constexpr int NV = PP ? TH / 4 : VT / 4;             // MFMA rows per wave (H rows if PP)
  static constexpr int T = 27, S0 = (T * NB + 3) / 4;         // k-steps of one conv's packing
  static constexpr int S = PP ? 9 : S0;                       // k-steps of the tile
  static constexpr int NBK = 2 * NB;                          // blocks per ring slot
  static constexpr int RH = TH + 2, RW = 18, PLANE = RH * RW;
  static constexpr int PIECES = (PLANE + 63) / 64, PLANEP = 64 * PIECES;
  static constexpr int SLOTW = NBK * PLANEP;
  static constexpr int PPW = (NBK * PIECES + 7) / 8;           // pieces per wave and plane
  static constexpr int RING = 8;
  static constexpr int RINGW = RING * SLOTW + 64 * (8 * PPW - NBK * PIECES);  // + padding pieces
  static constexpr int XW = 4 * NV * 16 * 2;                   // a's activations per parity (16-B words)
  static constexpr int LDSW = RINGW + 2 * XW;
#ifdef LEA_BF_PF
  static constexpr int PF = LEA_BF_PF > 0 ? LEA_BF_PF : 1;
#else
  static constexpr int PF = NB == 2 ? 2 : (PP ? 2 : 1);  // B-fragment prefetch distance (k-steps)
#endif
  static_assert(VT % 4 == 0 && (!PP || (NB == 1 && TH % 4 == 0)), "rows per wave");
  static_assert(2 * LDSW * 16 <= 160 * 1024, "two workgroups per CU");
};

template <int TH, int NB, bool PP>
__global__ __launch_bounds__(512, 2) void conv_bf16_pair_kernel(const Args a, int nsplit) {
  using C = PCfg<TH, NB, PP>;
  extern __shared__ __attribute__((aligned(16))) bf16x8 smem[];  // ring + a's activations
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int part = wave >> 2, wv = wave & 3;  // conv a (0) / b (1); rows wv * NV ..
  const int g = lane >> 4, n = lane & 15;

  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int q8 = a.nblk / 8, r8 = a.nblk % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + idx;
  const int sp = lin % nsplit;
  const int tile = (lin / nsplit) % a.ntiles;
  const int b = lin / (nsplit * a.ntiles);  // (one 16-cout block)
  const int h0 = (tile / a.tiles_w) * TH, w0 = (tile % a.tiles_w) * 16;
  const int HW = a.H * a.W;
  const int DHW = HW * a.D;
  const int nst = (a.D + 1) / 2;
  const int s0 = sp * nst / nsplit, s1 = (sp + 1) * nst / nsplit;

  // DMA pieces of one plane: piece q = wave + 8t -> (block q / PIECES, words 64 (q % PIECES) + lane);
  // blocks [0, NB) from xa, [NB, 2NB) from xb
  unsigned hwo[C::PPW], ldo[C::PPW];
  bool src2[C::PPW];
#pragma unroll
  for (int t = 0; t < C::PPW; ++t) {
    const int q = wave + 8 * t;
    const int blk = q / C::PIECES, e = (q % C::PIECES) * 64 + lane;
    src2[t] = blk >= NB;
    const int sblk = src2[t] ? blk - NB : blk;
    unsigned v = 0xFFFFFFF0u;
    if (q < C::NBK * C::PIECES && e < C::PLANE) {
      const int rr = e / C::RW, cc = e % C::RW;
      const int h = h0 + rr - 1, w = w0 + cc - 1;
      if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        v = (unsigned)sblk * (unsigned)DHW * 16u + (unsigned)(h * a.W + w) * 16u;
    }
    hwo[t] = v;
    ldo[t] = q < C::NBK * C::PIECES ? (unsigned)(blk * C::PLANEP + (q % C::PIECES) * 64)
                                    : (unsigned)(C::RING * C::SLOTW + (q - C::NBK * C::PIECES) * 64);
  }
  const unsigned srcb = (unsigned)NB * (unsigned)DHW * 16u;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)b * a.xbs), 0, srcb, 0x00020000);
  const __amdgpu_buffer_rsrc_t x2rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.x2 + (long long)b * a.x2bs), 0, srcb, 0x00020000);
  auto load_plane = [&](int d) {  // plane d (zeros outside 0..D-1) -> ring slot d & 7
    const bool dv = (unsigned)d < (unsigned)a.D;
    const unsigned slot = (unsigned)(d & 7) * C::SLOTW;
#pragma unroll
    for (int t = 0; t < C::PPW; ++t) {
      const unsigned vo = (dv && hwo[t] != 0xFFFFFFF0u) ? hwo[t] + (unsigned)d * (unsigned)HW * 16u : 0xFFFFFFF0u;
      const unsigned dst = ldo[t] < (unsigned)(C::RING * C::SLOTW) ? slot + ldo[t] : ldo[t];
      dma_x4(src2[t] ? x2rs : xrs, vo, lds0 + 16u * dst);
    }
  };

  // this wave's K slots: k-step ks, lane group g -> tap, block of its conv's chunk
  int kdv[C::S], koff[C::S];
#pragma unroll
  for (int ks = 0; ks < C::S; ++ks) {
    const int slot = 4 * ks + g;
    if (PP) {  // k-step ks = tap (kh, kw), lane group g = input plane 2s-1 + g (r06): the lane groups a
      // ds_read_b128 serves together (k-groups 0 / 1, 2 / 3) then read the same tap of planes whose ring
      // slots are 0 mod 16 apart -- conflict-free; the former order (slot = plane x 9 + tap) paired
      // neighbouring taps, two-way on 22 % of the LDS cycles
      const int j = g, t2 = ks;
      kdv[ks] = j;
      koff[ks] = part * C::PLANEP + (t2 / 3) * C::RW + t2 % 3;
    } else {
      const int tap = min(slot / NB, C::T - 1);  // slots past the last tap carry zero weights
      const int blk = slot % NB + part * NB;
      kdv[ks] = tap / 9;
      koff[ks] = blk * C::PLANEP + ((tap / 3) % 3) * C::RW + tap % 3;
    }
  }
  // this wave's conv: chunk `part` of the pair's packed weights (conv a's pack, then b's)
  const bf16x8* wpv = reinterpret_cast<const bf16x8*>(a.wp);
  bf16x8 av[C::S];
#pragma unroll
  for (int ks = 0; ks < C::S; ++ks) {
    if (PP) {
      // row n: cout n % 8 of output plane 2s + n / 8, whose kd for input plane 2s-1 + j is j - n / 8;
      // its 8 channels of tap (kd, kh, kw) are word (tap / 4, tap % 4, cout) of the packing
      const int j = g, t2 = ks;
      const int kd = j - n / 8, co = n % 8, tap = kd * 9 + t2;
      const bool ok = kd >= 0 && kd <= 2 && co < a.cout;
      av[ks] = ok ? wpv[((long long)part * C::S0 + tap / 4) * 64 + (tap % 4) * 16 + co] : bf16x8{};
    } else {
      av[ks] = wpv[((long long)part * C::S + ks) * 64 + g * 16 + n];
    }
  }
  float sc[4], sh[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = (PP ? 4 * (g % 2) : 4 * g) + r;  // PP: lane group g holds plane 2s + g / 2
    sc[r] = (a.scale && co < a.cout) ? a.scale[part * a.cout + co] : 1.f;
    sh[r] = (a.shift && co < a.cout) ? a.shift[part * a.cout + co] : 0.f;
  }
  const bool relu = a.flags & LEA_RELU;
  // a's activations: [parity][wv][row i][column n][16 couts] bf16, lane (g, n) owns couts 4g..4g+3
  __bf16* xa_lds = reinterpret_cast<__bf16*>(smem + C::RINGW);
  auto xoff = [&](int parity, int i) { return ((((parity * 4 + wv) * C::NV + i) * 16 + n) * 16 + 4 * g); };

  // conv b's output through one buffer resource: every lane issues the same NV 8-byte stores
  // per step (invalid ones at an out-of-range offset: dropped), so the waits below can count them
  f32x4 prev[C::NV];  // conv b: the previous step's accumulators (epilogue after the next barrier)
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.y + (long long)b * a.ybs), 0, (unsigned)((a.cout + 7) / 8) * (unsigned)DHW * 16u, 0x00020000);
  auto epilogue_b = [&](int s) {
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      const int qrow = wv * C::NV + i;
      const int d = 2 * s + (PP ? g / 2 : qrow / TH), h = h0 + (PP ? qrow : qrow % TH), w = w0 + n;
      const bf16x4 va = *reinterpret_cast<const bf16x4*>(xa_lds + xoff(s & 1, i));
      const int co = PP ? 4 * (g % 2) : 4 * g;
      const bool ok = d < a.D && h < a.H && w < a.W && co < a.cout;
      const unsigned off = ok ? (unsigned)(co / 8) * (unsigned)DHW * 16u + (unsigned)(co % 8) * 2u +
                                    (unsigned)(d * HW + h * a.W + w) * 16u
                              : 0xFFFFFFF0u;
      bf16x4 out;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = prev[i][r] * sc[r] + sh[r];
        if (relu) v = fmaxf(v, 0.f);
        out[r] = (__bf16)((float)va[r] + v);
      }
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, out), yrs, off, 0, 0);
    }
  };

  // Pipeline: after step s's barrier every wave issues planes 2s+5, 2s+6 (into the slots of
  // planes 2s-3, 2s-2, which only step s-1 read) -- two steps of planes in flight during the
  // MFMAs -- then conv b's waves store step s-1.  The top of step s+1 waits for all but the
  // younger operations than planes 2s+3, 2s+4: planes 2s+5, 2s+6 and, on conv b's waves, the
  // stores issued since (of steps s-2 and s-1: NV each; none for step s0 - 1)
  for (int j = -1; j <= 4; ++j) load_plane(2 * s0 + j);
  for (int s = s0; s < s1; ++s) {
    if (part == 1 && s - s0 >= 3)
      wait_vm<2 * C::PPW + 2 * C::NV>();
    else if (part == 1 && s - s0 == 2)
      wait_vm<2 * C::PPW + C::NV>();  // (step s0 stored nothing)
    else
      wait_vm<2 * C::PPW>();  // conv a; s0 (the prologue's planes 2s0+3, 2s0+4 may stay in flight)
    __syncthreads();  // everyone's planes landed; step s-1 done (its activations in LDS)
    load_plane(2 * s + 5);
    load_plane(2 * s + 6);
    if (part == 1 && s > s0) epilogue_b(s - 1);
    f32x4 acc[C::NV];
#pragma unroll
    for (int i = 0; i < C::NV; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int base = 2 * s - 1;
    auto ldb = [&](int ks, int i) {
      const int qrow = wv * C::NV + i;
      const int t = PP ? 0 : qrow / TH, r = PP ? qrow : qrow % TH;
      return smem[((base + t + kdv[ks]) & 7) * C::SLOTW + koff[ks] + r * C::RW + n];
    };
    // B fragments PF k-steps ahead of their MFMAs, in that issue order (as the stream kernel)
    bf16x8 bq[C::S][C::NV];
#pragma unroll
    for (int ks = 0; ks < C::PF && ks < C::S; ++ks)
#pragma unroll
      for (int i = 0; i < C::NV; ++i) bq[ks][i] = ldb(ks, i);
#pragma unroll
    for (int ks = 0; ks < C::S; ++ks) {
      if (ks + C::PF < C::S)
#pragma unroll
        for (int i = 0; i < C::NV; ++i) bq[ks + C::PF][i] = ldb(ks + C::PF, i);
#pragma unroll
      for (int i = 0; i < C::NV; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[ks], bq[ks][i], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (part == 0) {
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][r] * sc[r] + sh[r];
          o[r] = (__bf16)(relu ? fmaxf(v, 0.f) : v);
        }
        *reinterpret_cast<bf16x4*>(xa_lds + xoff(s & 1, i)) = o;
      }
    } else {
#pragma unroll
      for (int i = 0; i < C::NV; ++i) prev[i] = acc[i];
    }
  }
  wait_vm<0>();  // no LDS-DMA may outlive the workgroup
  __syncthreads();
  if (part == 1 && s1 > s0) epilogue_b(s1 - 1);
}

struct Plan {
  int ks, mt, wc, th, td, nb;
  int nsplit;  // > 0: the D-streaming kernel with nsplit column segments along D
  bool s1x1;   // the streamed 1x1 (conv1x1_c8_kernel)
};

int g_override[3] = {0, 0, 0};  // th, td, mt (lea_conv3d_bf16_set_tile_override)
int g_variant = 0;              // lea_conv3d_bf16_set_variant: 0 planner, 1 tile kernel only
int g_stream1x1 = 1;            // lea_conv3d_bf16_set_stream1x1
int g_pair_split = 3;           // lea_conv3d_bf16_set_pair_split: LEA_PAIR_SUM on the split-wave kernel
                                // (2: the plane-paired tile for the 8 -> 8 steps; 3: that, and the
                                // 16-channel steps on the two-source D-streaming kernel)
// conv1x1_rs_c8_kernel: tiles per wave (r05 probe at the C4 shapes, tools/rs_probe.py: two tiles'
// corner loads in flight together 4-5 % faster than one; more tiles per wave slower)
constexpr int g_rs_tpw = 2;

inline Plan plan(int B, int cout, int D, int H, int W, int ks, int cin) {
  // r01 sweep (tools/conv_sweep.py --bf16, profiles/r01_conv_sweep_bf16.txt): one
  // 16-row tile per wave with the waves splitting the couts beat 32-row tiles on
  // every layer; 4-row tiles win on the small (L2) volumes; the 8-channel-input
  // layers (one short K chunk) want deeper tiles to amortise staging.
  Plan p;
  p.ks = ks;
  const int cobv = cob_of(cout);
  p.mt = 1;
  p.wc = cobv / 16;
  p.nb = nb_of(cin, ks);
  p.td = (ks == 3) ? 2 : 1;
  const long long ncob = (cout + cobv - 1) / cobv;
  auto wgs = [&](int th, int td) {
    return (long long)((W + 15) / 16) * ((H + th - 1) / th) * ((D + td - 1) / td) * B * ncob;
  };
  p.th = wgs(8, p.td) < 8192 ? 4 : 8;
  if (ks == 3 && p.nb == 1 && wgs(8, 4) >= 2048) {
    p.th = 8;
    p.td = 4;
  }
  // r05: the deep-K 64-cout layers (conv1/2, cin 128) with two cout tiles per wave (each B
  // fragment read from LDS by two waves instead of four): same-box C4 +0.35 %, C3 +0.55 % over
  // four order-balanced rounds (profiles/r05_conv12_mt2_ab.txt; the first, fixed-order A/B
  // read +1.2 % -- part of that was the second-run bias)
  if (ks == 3 && cin >= 64 && cobv == 64) {
    p.th = 8;
    p.td = 2;
    p.mt = 2;
    p.wc = cobv / 16 / p.mt;
  }
  if (g_override[0] > 0) {
    p.th = g_override[0];
    p.td = g_override[1];
    p.mt = std::min(g_override[2], cobv / 16);
    p.wc = cobv / 16 / p.mt;
  }
  p.nsplit = 0;
  p.s1x1 = ks == 1 && cin <= 128 && g_stream1x1 && g_variant == 0 && g_override[0] == 0;
  // (r02 tools/bf16_stream_bench.py: two-chunk layers with 64-cout blocks -- the L2
  // 32->96 sibling groups -- hold 221 VGPRs of weights and accumulators and run slower
  // streamed; they stay on the tile kernel)
  const bool two_chunks_wide = cin > 8 * p.nb && cobv > 32;
  if (ks == 3 && cin <= 16 * p.nb && !two_chunks_wide && g_variant == 0 && g_override[0] == 0 && D >= 4) {
    // one or two K chunks (cin <= 32): stream along D; column segments so the grid
    // holds >= 6 workgroups per CU, each walking >= 4 steps
    p.mt = 1;
    p.wc = cobv / 16;
    p.th = cin <= 8 ? 8 : 4;
    p.td = 2;
    const long long cols = (long long)((W + 15) / 16) * ((H + p.th - 1) / p.th) * B * ncob;
    const int nst = (D + 1) / 2;
    long long ns = (1536 + cols - 1) / cols;
    ns = std::min<long long>(ns, std::max(1, nst / 4));
    p.nsplit = (int)std::max<long long>(ns, 1);
  }
  return p;
}

#define LEA_BF_CASE(KS, MT, WC, TH, TD, NB, CV)                                       \
  if (p.ks == KS && p.mt == MT && p.wc == WC && p.th == TH && p.td == TD && p.nb == NB) { \
    a.tiles_w = (a.W + 15) / 16;                                                      \
    a.ntiles = a.tiles_w * ((a.H + TH - 1) / TH);                                     \
    a.ndz = (a.D + TD - 1) / TD;                                                      \
    const long long nb_ = (long long)a.ntiles * a.ndz * B * a.ncob;                   \
    LEA_CHECK_ARG(nb_ < (1LL << 31), "lea_conv3d(bf16): grid too large");             \
    a.nblk = (int)nb_;                                                                \
    const size_t lds_ = (size_t)(a.nchunks > 1 ? 2 : 1) * Cfg<KS, MT, WC, TH, TD, NB, CV>::STAGE * 16; \
    conv_bf16_kernel<KS, MT, WC, TH, TD, NB, CV><<<dim3((unsigned)nb_), kThreads, lds_, st>>>(a); \
    return launch_status("lea_conv3d(bf16)");                                         \
  }
#define LEA_BF_TH(KS, MT, WC, TD, NB, CV) \
  LEA_BF_CASE(KS, MT, WC, 16, TD, NB, CV) LEA_BF_CASE(KS, MT, WC, 8, TD, NB, CV) LEA_BF_CASE(KS, MT, WC, 4, TD, NB, CV)
#define LEA_BF_MT(KS, TD, NB, CV)                                                         \
  LEA_BF_TH(KS, 1, 1, TD, NB, CV) LEA_BF_TH(KS, 2, 1, TD, NB, CV) LEA_BF_TH(KS, 1, 2, TD, NB, CV) \
  LEA_BF_TH(KS, 2, 2, TD, NB, CV) LEA_BF_TH(KS, 1, 4, TD, NB, CV)

#define LEA_BFS_CASE(WC, TH, NB, NCH)                                                         \
  if (p.wc == WC && p.th == TH && p.nb == NB && a.nchunks == NCH) {                           \
    a.tiles_w = (a.W + 15) / 16;                                                              \
    a.ntiles = a.tiles_w * ((a.H + TH - 1) / TH);                                             \
    const long long nb_ = (long long)a.ntiles * p.nsplit * B * a.ncob;                        \
    LEA_CHECK_ARG(nb_ < (1LL << 31), "lea_conv3d(bf16 stream): grid too large");              \
    a.nblk = (int)nb_;                                                                        \
    using S_ = SCfg<1, WC, TH, NB, NCH>;                                                      \
    const size_t lds_ = (size_t)((a.flags & LEA_RESIDUAL) ? S_::LDSW : S_::RINGW) * 16;       \
    conv_bf16_stream_kernel<1, WC, TH, NB, NCH><<<dim3((unsigned)nb_), kThreads, lds_, st>>>(a, p.nsplit); \
    return launch_status("lea_conv3d(bf16 stream)");                                         \
  }

int run(const Plan& p, Args a, int B, hipStream_t st, bool cv) {
  if (p.s1x1 && !cv) {
    const long long vox = (long long)a.D * a.H * a.W;
    const long long tiles = (vox + 15) / 16;
    // about 8192 waves over the batch and cout blocks, each walking tpw tiles
    const long long tpw = std::max(1LL, (tiles * B * a.ncob + 8191) / 8192);
    const long long gx = (tiles + 4 * tpw - 1) / (4 * tpw);
    LEA_CHECK_ARG(gx < (1LL << 31) && (long long)B * a.ncob <= 65535, "lea_conv3d(bf16 1x1): grid too large");
    const dim3 grid((unsigned)gx, B * a.ncob);
    // one-chunk layers and the two-chunk ones with >= 2 cout tiles on the specialised forms;
    // the two-chunk single-tile layers measured 2 % slower at 6 waves per SIMD than at 4
    // (r05 tools/rs_probe.py --one, profiles/r05_1x1_rs_probe.txt)
    const int nch0 = (a.cin / 8 + 3) / 4, nch = (nch0 == 1 || (nch0 == 2 && p.wc >= 2)) ? nch0 : 4;
#define LEA_1X1(MT_)                                                                            \
  if (p.wc == MT_) {                                                                            \
    if (nch == 1) conv1x1_c8_kernel<MT_, 1><<<grid, 256, 0, st>>>(a, (int)tpw);                 \
    else if (nch == 2) conv1x1_c8_kernel<MT_, 2><<<grid, 256, 0, st>>>(a, (int)tpw);            \
    else conv1x1_c8_kernel<MT_, 4><<<grid, 256, 0, st>>>(a, (int)tpw);                          \
  }
    LEA_1X1(1) LEA_1X1(2) LEA_1X1(4)
#undef LEA_1X1
    return launch_status("lea_conv3d(bf16 1x1)");
  }
  if ((a.flags & LEA_PAIR_SUM) && g_pair_split && p.nsplit > 0 && a.ncob == 1 && (a.nchunks == 2) &&
      ((p.nb == 2 && p.th == 4 && g_pair_split != 3) || (p.nb == 1 && p.th == 8))) {
    // the split-wave pair kernel (conv a / conv b on separate wave halves)
    a.tiles_w = (a.W + 15) / 16;
    a.ntiles = a.tiles_w * ((a.H + p.th - 1) / p.th);
    const long long nb_ = (long long)a.ntiles * p.nsplit * B;
    LEA_CHECK_ARG(nb_ < (1LL << 31), "lea_conv3d(bf16 pair): grid too large");
    LEA_CHECK_ARG((long long)(a.cin / 16 + 1) * a.D * a.H * a.W * 16 < 0xFFFFFFF0LL,
                  "lea_conv3d(bf16 pair): volume too large");
    a.nblk = (int)nb_;
    if (p.nb == 2)
      conv_bf16_pair_kernel<4, 2, false><<<dim3((unsigned)nb_), 512, PCfg<4, 2>::LDSW * 16, st>>>(a, p.nsplit);
    else if (g_pair_split >= 2 && a.cout <= 8)
      conv_bf16_pair_kernel<8, 1, true><<<dim3((unsigned)nb_), 512, PCfg<8, 1, true>::LDSW * 16, st>>>(a, p.nsplit);
    else
      conv_bf16_pair_kernel<8, 1, false><<<dim3((unsigned)nb_), 512, PCfg<8, 1>::LDSW * 16, st>>>(a, p.nsplit);
    return launch_status("lea_conv3d(bf16 pair)");
  }
  // (one source, or LEA_PAIR_SUM's two: the ring walks the blocks of both)
  if (p.nsplit > 0 && !cv && (a.cb1 * 8 == a.cin || (a.flags & LEA_PAIR_SUM))) {
    LEA_CHECK_ARG((long long)std::max(a.cin, a.cout + 7) / 8 * a.D * a.H * a.W * 16 < 0xFFFFFFF0LL,
                  "lea_conv3d(bf16 stream): volume too large");
    LEA_BFS_CASE(1, 8, 1, 1) LEA_BFS_CASE(2, 8, 1, 1) LEA_BFS_CASE(4, 8, 1, 1)
    LEA_BFS_CASE(1, 4, 2, 1) LEA_BFS_CASE(2, 4, 2, 1) LEA_BFS_CASE(4, 4, 2, 1)
    LEA_BFS_CASE(1, 4, 2, 2) LEA_BFS_CASE(2, 4, 2, 2) LEA_BFS_CASE(1, 8, 1, 2)
  }
  if (a.flags & LEA_PAIR_SUM) {
    set_error("lea_conv3d(bf16): LEA_PAIR_SUM runs on the D-streaming kernel only (cout <= 16, D >= 4)");
    return LEA_E_UNSUPPORTED;
  }
  if (cv) {
    LEA_BF_MT(3, 2, 2, true)
    LEA_BF_MT(3, 1, 2, true)
  } else {
    LEA_BF_MT(3, 2, 1, false)
    LEA_BF_MT(3, 2, 2, false)
    LEA_BF_MT(3, 1, 1, false)
    LEA_BF_MT(3, 1, 2, false)
    LEA_BF_MT(3, 4, 1, false)
    LEA_BF_MT(3, 4, 2, false)
    LEA_BF_MT(1, 1, 4, false)
  }
  set_error("lea_conv3d(bf16): no tile ks=%d mt=%d wc=%d th=%d td=%d nb=%d cv=%d", p.ks, p.mt, p.wc,
            p.th, p.td, p.nb, (int)cv);
  return LEA_E_UNSUPPORTED;
}

#define LEA_BF2D_CASE(WC, TH, NB)                                                           \
  if (p.wc == WC && p.th == TH && p.nb == NB) {                                             \
    a.tiles_w = (a.W + 15) / 16;                                                            \
    a.ntiles = a.tiles_w * ((a.H + TH - 1) / TH);                                           \
    a.ndz = 1;                                                                              \
    const long long nb_ = (long long)a.ntiles * B * a.ncob;                                 \
    LEA_CHECK_ARG(nb_ < (1LL << 31), "lea_conv2d(bf16): grid too large");                   \
    a.nblk = (int)nb_;                                                                      \
    const size_t lds_ = (size_t)(a.nchunks > 1 ? 2 : 1) * Cfg<3, 1, WC, TH, 1, NB, false, 1>::STAGE * 16; \
    conv_bf16_kernel<3, 1, WC, TH, 1, NB, false, 1><<<dim3((unsigned)nb_), kThreads, lds_, st>>>(a); \
    return launch_status("lea_conv2d(bf16)");                                               \
  }
#define LEA_BF2D_NB(WC, NB) LEA_BF2D_CASE(WC, 8, NB) LEA_BF2D_CASE(WC, 4, NB)

int run2d(const Plan& p, Args a, int B, hipStream_t st) {
  LEA_BF2D_NB(1, 1) LEA_BF2D_NB(1, 2) LEA_BF2D_NB(2, 1) LEA_BF2D_NB(2, 2) LEA_BF2D_NB(4, 1)
  LEA_BF2D_NB(4, 2)
  set_error("lea_conv2d(bf16): no tile wc=%d th=%d nb=%d", p.wc, p.th, p.nb);
  return LEA_E_UNSUPPORTED;
}

thread_local char g_bf_name[96];

}  // namespace bf
}  // namespace lea

using namespace lea;
using bf16x8_t = bf::bf16x8;

extern "C" int lea_conv3d_bf16_set_tile_override(int th, int td, int mt) {
  clear_error();
  if (th <= 0) {
    bf::g_override[0] = 0;
    return 0;
  }
  LEA_CHECK_ARG((th == 4 || th == 8 || th == 16) && (td == 1 || td == 2 || td == 4) && (mt == 1 || mt == 2),
                "lea_conv3d_bf16_set_tile_override: bad tile th=%d td=%d mt=%d", th, td, mt);
  bf::g_override[0] = th;
  bf::g_override[1] = td;
  bf::g_override[2] = mt;
  return 0;
}

extern "C" int lea_conv3d_bf16_set_stream1x1(int on) {
  clear_error();
  LEA_CHECK_ARG(on == 0 || on == 1, "lea_conv3d_bf16_set_stream1x1: on=%d", on);
  bf::g_stream1x1 = on;
  return 0;
}

extern "C" int lea_conv3d_bf16_set_pair_split(int on) {
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 3, "lea_conv3d_bf16_set_pair_split: %d", on);
  bf::g_pair_split = on;
  return 0;
}

extern "C" int lea_conv3d_bf16_set_variant(int variant) {
  clear_error();
  LEA_CHECK_ARG(variant == 0 || variant == 1, "lea_conv3d_bf16_set_variant: bad variant %d", variant);
  bf::g_variant = variant;
  return 0;
}

extern "C" size_t lea_conv3d_packed_elems_bf16(int cout, int cin, int k) {
  if (cout <= 0 || cin <= 0 || cin % 8 != 0 || (k != 1 && k != 3)) return 0;
  const int cobv = bf::cob_of(cout), nb = bf::nb_of(cin, k);
  const int nch = (cin / 8 + nb - 1) / nb;
  return (size_t)((cout + cobv - 1) / cobv) * nch * bf::ksteps(k, nb) * (cobv / 16) * 4 * 16 * 8;
}

extern "C" int lea_conv3d_pack_weights_bf16(const float* w, void* packed, int cout, int cin, int k,
                                            void* stream) {
  clear_error();
  LEA_CHECK_ARG(w && packed, "lea_conv3d_pack_weights_bf16: null pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0 && cin % 8 == 0 && cout % 4 == 0 && (k == 1 || k == 3),
                "lea_conv3d_pack_weights_bf16: unsupported shape cout=%d cin=%d k=%d", cout, cin, k);
  const int cobv = bf::cob_of(cout), nb = bf::nb_of(cin, k);
  const int nch = (cin / 8 + nb - 1) / nb;
  const long long total = (long long)lea_conv3d_packed_elems_bf16(cout, cin, k);
  const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
  bf::pack_bf16_kernel<<<grid, 256, 0, as_stream(stream)>>>(w, (__bf16*)packed, cout, cin, k * k * k,
                                                            nb, bf::ksteps(k, nb), cobv / 16, nch, total);
  return launch_status("lea_conv3d_pack_weights_bf16");
}

extern "C" int lea_conv3d_bf16_pair_supported(int B, int cin, int cout, int D, int H, int W) {
  // the same conditions bf16_conv_common applies to LEA_PAIR_SUM (the tuning
  // knobs can take a shape off the D-streaming plan)
  if (B <= 0 || cin <= 0 || cout <= 0 || D <= 0 || H <= 0 || W <= 0 || cin % 8 || cout % 8) return 0;
  const bf::Plan p = bf::plan(B, cout, D, H, W, 3, cin);
  return cout <= 16 && p.nsplit > 0 && cin <= 8 * p.nb ? 1 : 0;
}

extern "C" const char* lea_conv3d_kernel_name_bf16(int B, int cout, int cin, int D, int H, int W,
                                                   int k, int costvolume) {
  if (B <= 0 || cout <= 0 || cin <= 0 || (k != 1 && k != 3) || D <= 0 || H <= 0 || W <= 0) return nullptr;
  const bf::Plan p = bf::plan(B, cout, D, H, W, k, cin);
  if (p.s1x1 && !costvolume)
    snprintf(bf::g_bf_name, sizeof(bf::g_bf_name), "conv1x1_c8_kernel<%d>", p.wc);
  else if (p.nsplit > 0 && !costvolume)
    snprintf(bf::g_bf_name, sizeof(bf::g_bf_name), "conv_bf16_stream_kernel<1, %d, %d, %d, %d>", p.wc, p.th,
             p.nb, (cin / 8 + p.nb - 1) / p.nb);
  else
    snprintf(bf::g_bf_name, sizeof(bf::g_bf_name), "conv_bf16_kernel<%d, %d, %d, %d, %d, %d, %s>",
             p.ks, p.mt, p.wc, p.th, p.td, p.nb, costvolume ? "true" : "false");
  return bf::g_bf_name;
}

static int bf16_conv_common(bf::Args& a, int B, int k, bool cv, void* stream) {
  clear_error();
  LEA_CHECK_ARG(a.x && a.wp && a.y, "lea_conv3d(bf16): null pointer");
  LEA_CHECK_ARG((a.scale == nullptr) == (a.shift == nullptr),
                "lea_conv3d(bf16): scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(!(a.flags & LEA_RESIDUAL) || a.res, "lea_conv3d(bf16): LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && a.cin > 0 && a.cout > 0 && a.D > 0 && a.H > 0 && a.W > 0,
                "lea_conv3d(bf16): bad shape");
  LEA_CHECK_ARG(a.cin % 8 == 0 && a.cout % 8 == 0 && a.cb1 * 8 <= a.cin,
                "lea_conv3d(bf16): channels must be multiples of 8 (cin=%d cout=%d)", a.cin, a.cout);
  LEA_CHECK_ARG((long long)a.D * a.H * a.W * 16 < (1LL << 32), "lea_conv3d(bf16): volume too large");
  LEA_CHECK_ARG(a.x != (const __bf16*)a.y && a.x2 != (const __bf16*)a.y,
                "lea_conv3d(bf16): input aliases output");
  const bool pair = a.flags & LEA_PAIR_SUM;
  bf::Plan p = bf::plan(B, a.cout, a.D, a.H, a.W, k, pair ? a.cb1 * 8 : a.cin);
  if (pair) {
    // two equal sources of one K chunk each (the L0 / L1 cell steps), one 16-cout block: the
    // packed weight is conv a's chunk then conv b's
    LEA_CHECK_ARG(!(a.flags & LEA_RESIDUAL) && a.x2 && 2 * a.cb1 * 8 == a.cin && k == 3 && !cv,
                  "lea_conv3d(bf16): LEA_PAIR_SUM needs two equal sources and no residual");
    if (a.cout > 16 || p.nsplit <= 0 || a.cb1 * 8 > 8 * p.nb) {
      set_error("lea_conv3d(bf16): LEA_PAIR_SUM unsupported for cin=%d cout=%d D=%d", a.cin, a.cout, a.D);
      return LEA_E_UNSUPPORTED;
    }
  }
  // the D-streaming kernels address one batch element's input, residual and output blocks
  // through 32-bit buffer offsets
  LEA_CHECK_ARG(p.nsplit <= 0 || (long long)std::max(a.cin, a.cout) / 8 * a.D * a.H * a.W * 16 < (1LL << 32),
                "lea_conv3d(bf16): batch element too large for the D-streaming kernel");
  const int cobv = bf::cob_of(a.cout);
  a.ncob = (a.cout + cobv - 1) / cobv;
  a.nchunks = (a.cin / 8 + p.nb - 1) / p.nb;
  return bf::run(p, a, B, as_stream(stream), cv);
}

// dtype LEA_BF16 counterparts of lea_conv3d_bnrelu / lea_conv3d_bnrelu_costvolume
// (tensors in the c8 layout; batch strides in elements)
extern "C" int lea_conv3d_bnrelu_bf16(const void* x, int64_t x_bstride, const void* x2,
                                      int64_t x2_bstride, int cin2, const void* w_packed,
                                      const float* scale, const float* shift, const void* residual,
                                      int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                      int cout, int D, int H, int W, int k, unsigned flags,
                                      void* stream) {
  bf::Args a{};
  a.x = (const __bf16*)x;
  a.xbs = x_bstride;
  a.x2 = (const __bf16*)x2;
  a.x2bs = x2_bstride;
  a.cb1 = (cin - cin2) / 8;
  a.wp = (const __bf16*)w_packed;
  a.scale = scale;
  a.shift = shift;
  a.res = (const __bf16*)residual;
  a.rbs = r_bstride;
  a.y = (__bf16*)y;
  a.ybs = y_bstride;
  a.cin = cin;
  a.cout = cout;
  a.D = D;
  a.H = H;
  a.W = W;
  a.flags = flags;
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU | LEA_RESIDUAL | LEA_PAIR_SUM, "lea_conv3d_bnrelu_bf16");
  if (cin2 % 8 != 0 || (cin2 > 0 && !x2)) {
    set_error("lea_conv3d_bnrelu_bf16: bad second source");
    return LEA_E_INVALID;
  }
  return bf16_conv_common(a, B, k, false, stream);
}

extern "C" int lea_conv3d_bnrelu_costvolume_bf16(const void* left, const void* right,
                                                 int64_t f_bstride, const void* w_packed,
                                                 const float* scale, const float* shift, void* y,
                                                 int64_t y_bstride, int B, int C, int cout, int D3,
                                                 int H, int W, unsigned flags, void* stream) {
  bf::Args a{};
  a.x = (const __bf16*)left;
  a.xbs = f_bstride;
  a.x2 = (const __bf16*)right;
  a.x2bs = f_bstride;
  a.cb1 = C / 8;
  a.wp = (const __bf16*)w_packed;
  a.scale = scale;
  a.shift = shift;
  a.y = (__bf16*)y;
  a.ybs = y_bstride;
  a.cin = 2 * C;
  a.cout = cout;
  a.D = D3;
  a.H = H;
  a.W = W;
  a.flags = flags & LEA_RELU;
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_conv3d_bnrelu_costvolume_bf16");
  if (C % 16 != 0) {  // chunks of 2 blocks must not straddle left/right
    set_error("lea_conv3d_bnrelu_costvolume_bf16: C=%d must be a multiple of 16", C);
    return LEA_E_INVALID;
  }
  return bf16_conv_common(a, B, 3, true, stream);
}

extern "C" int lea_to_c8_bf16(const float* x, int64_t x_bstride, void* y, int64_t y_bstride, int B,
                              int C, int64_t vol, void* stream) {
  clear_error();
  LEA_CHECK_ARG(x && y && B > 0 && C > 0 && C % 8 == 0 && vol > 0 && B <= 65535,
                "lea_to_c8_bf16: bad arguments");
  const long long n = vol * (C / 8);
  dim3 grid((unsigned)std::min<long long>((n + 255) / 256, 65535), B);
  bf::to_c8_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, x_bstride, (__bf16*)y, y_bstride, C, vol);
  return launch_status("lea_to_c8_bf16");
}

extern "C" int lea_from_c8_bf16(const void* x, int64_t x_bstride, float* y, int64_t y_bstride, int B,
                                int C, int64_t vol, void* stream) {
  clear_error();
  LEA_CHECK_ARG(x && y && B > 0 && C > 0 && C % 8 == 0 && vol > 0 && B <= 65535,
                "lea_from_c8_bf16: bad arguments");
  const long long n = vol * (C / 8);
  dim3 grid((unsigned)std::min<long long>((n + 255) / 256, 65535), B);
  bf::from_c8_kernel<<<grid, 256, 0, as_stream(stream)>>>((const __bf16*)x, x_bstride, y, y_bstride, C, vol);
  return launch_status("lea_from_c8_bf16");
}

// resample words per thread (lea_resample_bf16_set_batch; 0 = up-sampling 4, else 1)
static int g_resample_k = 0;

// 1 (default) = up-samplings on the column-walking kernel (lea_resample_bf16_set_cols)
static int g_resample_cols = 1;

extern "C" int lea_resample_bf16_set_cols(int on) {
  clear_error();
  LEA_CHECK_ARG(on >= 0 && on <= 2, "lea_resample_bf16_set_cols: %d", on);
  g_resample_cols = on;
  return 0;
}

extern "C" int lea_resample_bf16_set_batch(int k) {
  clear_error();
  LEA_CHECK_ARG(k == 0 || k == 1 || k == 2 || k == 4, "lea_resample_bf16_set_batch: k=%d", k);
  g_resample_k = k;
  return 0;
}

extern "C" int lea_resample3d_trilinear_bf16(const void* x, int64_t x_bstride, void* y,
                                             int64_t y_bstride, int B, int C, int Di, int Hi,
                                             int Wi, int Do, int Ho, int Wo, int align_corners,
                                             const float* scale, const float* shift,
                                             unsigned flags, void* stream) {
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_resample3d_trilinear_bf16");
  LEA_CHECK_ARG(x && y && x != y, "lea_resample3d_trilinear_bf16: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_resample3d_trilinear_bf16: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && C > 0 && C % 8 == 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 &&
                    Wo > 0 && (long long)B * (C / 8) * Do <= 65535,
                "lea_resample3d_trilinear_bf16: bad shape");
  const int ac = align_corners ? 1 : 0;
  const long long cells = (long long)Ho * Wo;
  const bool up = (long long)Do * Ho * Wo > (long long)Di * Hi * Wi;
  if (up && g_resample_cols && g_resample_k == 0) {
    const int R = g_resample_cols == 2 ? 16 : 8;  // output rows per wave; 4 waves per workgroup
    const int ctiles = (Wo + 63) / 64, rblocks = (Ho + 4 * R - 1) / (4 * R);
    dim3 g((unsigned)(ctiles * rblocks), B * (C / 8) * Do);
#define LEA_RS_COLS(R_)                                                                                        \
  if (R == R_)                                                                                                \
    bf::resample_c8_cols_kernel<R_><<<g, 256, 0, as_stream(stream)>>>(                                         \
        (const __bf16*)x, x_bstride, (__bf16*)y, y_bstride, C / 8, Di, Hi, Wi, Do, Ho, Wo, axis_ratio(Di, Do, ac), \
        axis_ratio(Hi, Ho, ac), axis_ratio(Wi, Wo, ac), ac, scale, shift, flags, ctiles);
    LEA_RS_COLS(8) LEA_RS_COLS(16)
#undef LEA_RS_COLS
    return launch_status("lea_resample3d_trilinear_bf16");
  }
  const int k = g_resample_k > 0 ? g_resample_k : (up ? 4 : 1);
  dim3 grid((unsigned)((cells + 256LL * k - 1) / (256LL * k)), B * (C / 8) * Do);
#define LEA_RS_K(K_)                                                                                \
  if (k == K_)                                                                                     \
    bf::resample_c8_kernel<K_><<<grid, 256, 0, as_stream(stream)>>>(                               \
        (const __bf16*)x, x_bstride, (__bf16*)y, y_bstride, C / 8, Di, Hi, Wi, Do, Ho, Wo,          \
        axis_ratio(Di, Do, ac), axis_ratio(Hi, Ho, ac), axis_ratio(Wi, Wo, ac), ac, scale, shift, flags);
  LEA_RS_K(1) LEA_RS_K(2) LEA_RS_K(4)
#undef LEA_RS_K
  return launch_status("lea_resample3d_trilinear_bf16");
}

extern "C" int lea_conv1x1_resampled_bf16(const void* x, int64_t x_bstride, int Di, int Hi, int Wi,
                                          const void* w_packed, const float* scale, const float* shift,
                                          void* y, int64_t y_bstride, int B, int cin, int cout, int D,
                                          int H, int W, unsigned flags, void* stream) {
  clear_error();
  LEA_CHECK_FLAGS(flags, LEA_RELU, "lea_conv1x1_resampled_bf16");
  LEA_CHECK_ARG(x && w_packed && y && x != y, "lea_conv1x1_resampled_bf16: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_conv1x1_resampled_bf16: scale/shift must both be set or both NULL");
  LEA_CHECK_ARG(B > 0 && B <= 65535 && Di > 0 && Hi > 0 && Wi > 0 && D > 0 && H > 0 && W > 0,
                "lea_conv1x1_resampled_bf16: bad shape");
  LEA_CHECK_ARG(cin % 32 == 0 && cin <= 128 && cout % 16 == 0 && cout <= 64,
                "lea_conv1x1_resampled_bf16: cin %% 32 (<= 128), cout %% 16 (<= 64) required, got %d/%d",
                cin, cout);
  const long long vout = (long long)D * H * W;
  const int tpw = bf::g_rs_tpw;  // 16-voxel tiles per wave
  const long long nblk = (vout + 64LL * tpw - 1) / (64LL * tpw);
  LEA_CHECK_ARG(nblk < (1LL << 31), "lea_conv1x1_resampled_bf16: grid too large");
  const dim3 grid((unsigned)nblk, B);
  const float rd = axis_ratio(Di, D, 1), rh = axis_ratio(Hi, H, 1), rw = axis_ratio(Wi, W, 1);
  // the packed weights are the k = 1 layout of lea_conv3d_pack_weights_bf16 for this cout
  // (one block of cob_of(cout) couts: cout = 16 MT)
  LEA_CHECK_ARG(bf::cob_of(cout) == cout, "lea_conv1x1_resampled_bf16: cout %d is not one packing block", cout);
  const bf16x8_t* wp = reinterpret_cast<const bf16x8_t*>(w_packed);
  const int nchk = cin == 32 ? 1 : cin == 64 ? 2 : 4;
  // TU tiles' corner loads in flight (1 for the three- and four-chunk layers: 222-256 VGPRs at 2)
#define LEA_RS1(MT_, NCH_, TU_)                                                                      \
  if (cout == 16 * MT_ && nchk == NCH_)                                                              \
    bf::conv1x1_rs_c8_kernel<MT_, NCH_, TU_><<<grid, 256, 0, as_stream(stream)>>>(                   \
        (const __bf16*)x, x_bstride, Di, Hi, Wi, wp, scale, shift, (__bf16*)y, y_bstride, cin, cout, D, \
        H, W, rd, rh, rw, flags, tpw);
  LEA_RS1(1, 1, 2) LEA_RS1(1, 2, 2) LEA_RS1(1, 4, 1)
  LEA_RS1(2, 1, 2) LEA_RS1(2, 2, 2) LEA_RS1(2, 4, 1)
  LEA_RS1(4, 1, 2) LEA_RS1(4, 2, 2) LEA_RS1(4, 4, 1)
#undef LEA_RS1
  return launch_status("lea_conv1x1_resampled_bf16");
}

// ---- 2D 3x3 (feature net) on the bf16 engine: the D = 1 case of a (1, 3, 3) kernel
extern "C" size_t lea_conv2d_packed_elems_bf16(int cout, int cin) {
  if (cout <= 0 || cin <= 0 || cin % 8 != 0) return 0;
  const int cobv = bf::cob_of(cout), nb = bf::nb_of(cin, 3);
  const int nch = (cin / 8 + nb - 1) / nb;
  return (size_t)((cout + cobv - 1) / cobv) * nch * ((9 * nb + 3) / 4) * (cobv / 16) * 4 * 16 * 8;
}

extern "C" int lea_conv2d_pack_weights_bf16(const float* w, void* packed, int cout, int cin,
                                            void* stream) {
  clear_error();
  LEA_CHECK_ARG(w && packed, "lea_conv2d_pack_weights_bf16: null pointer");
  LEA_CHECK_ARG(cout > 0 && cin > 0 && cin % 8 == 0 && cout % 8 == 0,
                "lea_conv2d_pack_weights_bf16: unsupported shape cout=%d cin=%d", cout, cin);
  const int cobv = bf::cob_of(cout), nb = bf::nb_of(cin, 3);
  const int nch = (cin / 8 + nb - 1) / nb;
  const long long total = (long long)lea_conv2d_packed_elems_bf16(cout, cin);
  const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
  bf::pack_bf16_kernel<<<grid, 256, 0, as_stream(stream)>>>(w, (__bf16*)packed, cout, cin, 9, nb,
                                                            (9 * nb + 3) / 4, cobv / 16, nch, total);
  return launch_status("lea_conv2d_pack_weights_bf16");
}

extern "C" int lea_conv2d_bnrelu_bf16(const void* x, int64_t x_bstride, const void* w_packed,
                                      const float* scale, const float* shift, const void* residual,
                                      int64_t r_bstride, void* y, int64_t y_bstride, int B, int cin,
                                      int cout, int H, int W, unsigned flags, void* stream) {
  clear_error();
  bf::Args a{};
  a.x = (const __bf16*)x;
  a.xbs = x_bstride;
  a.x2 = (const __bf16*)x;
  a.cb1 = cin / 8;
  a.wp = (const __bf16*)w_packed;
  a.scale = scale;
  a.shift = shift;
  a.res = (const __bf16*)residual;
  a.rbs = r_bstride;
  a.y = (__bf16*)y;
  a.ybs = y_bstride;
  a.cin = cin;
  a.cout = cout;
  a.D = 1;
  a.H = H;
  a.W = W;
  a.flags = flags;
  LEA_CHECK_ARG(x && w_packed && y && x != y, "lea_conv2d_bnrelu_bf16: null or aliased pointer");
  LEA_CHECK_ARG((scale == nullptr) == (shift == nullptr),
                "lea_conv2d_bnrelu_bf16: scale/shift must both be set or both NULL");
  LEA_CHECK_FLAGS(flags, LEA_RELU | LEA_RESIDUAL, "lea_conv2d_bnrelu_bf16");
  LEA_CHECK_ARG(!(flags & LEA_RESIDUAL) || residual, "lea_conv2d_bnrelu_bf16: LEA_RESIDUAL without residual");
  LEA_CHECK_ARG(B > 0 && cin > 0 && cout > 0 && H > 0 && W > 0 && cin % 8 == 0 && cout % 8 == 0,
                "lea_conv2d_bnrelu_bf16: bad shape B=%d cin=%d cout=%d H=%d W=%d", B, cin, cout, H, W);
  const int cobv = bf::cob_of(cout);
  bf::Plan p;
  p.ks = 3;
  p.mt = 1;
  p.wc = cobv / 16;
  p.nb = bf::nb_of(cin, 3);
  p.td = 1;
  const long long wgs8 = (long long)((W + 15) / 16) * ((H + 7) / 8) * B * ((cout + cobv - 1) / cobv);
  p.th = wgs8 >= 1024 ? 8 : 4;
  a.ncob = (cout + cobv - 1) / cobv;
  a.nchunks = (cin / 8 + p.nb - 1) / p.nb;
  return bf::run2d(p, a, B, as_stream(stream));
}
