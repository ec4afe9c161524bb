// Shared pieces of the Winograd conv engines (conv3d_wino.hip: F(2,3) / F(4,3)
// along W; conv3d_wino2.hip: F(4,3) along W x F(2,3) along D): the lane -> output
// group map, the bank-conflict-free channel stride of the staged halo, and the
// LDS-DMA issue as inline asm.
#pragma once
#include "conv3d_impl.h"

namespace lea {
namespace wino {

constexpr int CIN_B = 4;

// 16-row MFMA tiles per cout block: 16, 32 or 48 couts (48 for 48k couts that are not
// multiples of 32: the L1 16->48 sibling groups would pad a 64-row block by a third)
// MT = 0: the depth-paired block for couts <= 8 -- one 16-row tile holding the couts
// of TWO output planes (as the direct engine's KD = 4 tile, conv3d_impl.h)
__host__ __device__ constexpr int mt_of(int cout) {
  return cout <= 8 ? 0 : cout <= 16 ? 1 : (cout % 32 != 0 && cout % 48 == 0) ? 3 : 2;
}
__host__ __device__ constexpr int cop_of(int mt) { return 16 * (mt > 0 ? mt : 1); }

// Lane group (16 lanes of one input channel) -> output groups: Q groups of F outputs
// per tile row and 16/Q rows (Q = 8 lets F(4,3) tile a 32-wide row pair).
template <int F, int Q>
__host__ __device__ constexpr int lane_dword(int lane, int cis, int rw) {
  return (lane >> 4) * cis + ((lane & 15) / Q) * rw + F * ((lane & 15) % Q);
}
// The two channels of a 32-lane ds_read_b64 group must hit disjoint banks: pick the
// smallest even channel stride >= img for which the first read's 64 dwords of lanes
// 0..31 fall on 64 distinct banks.
template <int F, int Q>
__host__ __device__ constexpr int conflict_free_cis(int img, int rw) {
  for (int cis = img + (img & 1);; cis += 2) {
    bool used[64] = {};
    bool ok = true;
    for (int l = 0; l < 32 && ok; ++l)
      for (int k = 0; k < 2 && ok; ++k) {
        const int bank = (lane_dword<F, Q>(l, cis, rw) + k) % 64;
        ok = !used[bank];
        used[bank] = true;
      }
    if (ok) return cis;
  }
}

// LDS-DMA pieces as inline asm: with the builtins hipcc treats every in-flight
// DMA as a possible write to any LDS word and waits vmcnt(0) before the first
// ds_read of each chunk -- i.e. for the NEXT chunk's halo, which de-pipelines the
// double buffer (r01 PMC: 17 % of wave cycles parked).  As asm they are invisible
// to its wait bookkeeping; the kernel's own vmcnt(0) + barrier at the chunk head is
// the one wait they need.  M0 (the LDS destination base) is saved and restored.
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)p);
}
__device__ __forceinline__ void dma_dword(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma_dwordx4_buf(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma_dwordx4(const float* src, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

__device__ __forceinline__ int a_col(int m, int ci, int n, bool swz) { return ((swz ? (m ^ (ci & 1)) : m) * 16) + n; }

// Buffer-addressed epilogue (host sets kEpiBuf, `epi_buf_ok`): every lane issues the
// same residual loads and output stores whatever its validity -- an invalid lane's
// offset is out of the block's range, so its load reads 0 and its store is dropped.
// The loads go out together (one latency instead of one round trip per store), and the
// count of stores per epilogue is a compile-time constant, so the next chunk head can
// wait for its DMA with vmcnt(stores) -- loads, stores and LDS-DMA retire in issue
// order (MI355X_MICROARCH.md, s_waitcnt) -- instead of for the stores as well.
constexpr unsigned kEpiBuf = 1u << 16;  // internal ConvArgs::flags bit
constexpr unsigned kPairSum = LEA_PAIR_SUM;
constexpr unsigned kEpiOob = 0xFFFFFF00u;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t block_rsrc(const float* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(unsigned)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
__device__ __forceinline__ void buf_store4(__amdgpu_buffer_rsrc_t rs, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, off, 0, 0);
}
// chunk head: this wave's DMA of the coming item landed; after an epilogue of nst
// buffer stores (issued after that DMA) those may stay in flight
template <int NST>
__device__ __forceinline__ void wait_item(bool after_epilogue) {
  static_assert(NST > 0 && NST < 64, "vmcnt immediate");
  if (after_epilogue)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// host: whole float4 output groups, 16-B aligned blocks, a cout block (<= 48 channels)
// addressable by 32-bit byte offsets below kEpiOob
inline bool epi_buf_ok(const ConvArgs& a) {
  const long long dhw = (long long)a.D * a.H * a.W;
  bool ok = a.W % 4 == 0 && dhw % 4 == 0 && ((uintptr_t)a.y & 15) == 0 && a.ybs % 4 == 0 &&
            48LL * dhw * 4 < (long long)kEpiOob;
  if (a.flags & LEA_RESIDUAL) ok = ok && ((uintptr_t)a.res & 15) == 0 && a.rbs % 4 == 0;
  return ok;
}

// Two-dimensional engine (conv3d_wino2.hip): Q output groups of 4 per tile row,
// WC cout tiles x (NW / WC) row sets of waves, MTE 16-row cout tiles per wave, OCC
// waves per SIMD (launch bound), PV = inputs transformed once per chunk into LDS; the packed weights are the 1-D engine's for the
// block of 16 WC MTE couts.
struct Plan2 {
  int q, wc, mte, nw, occ;
  int pv;   // V transformed once per chunk into LDS by the workgroup: 1 = halo staged by
            // dword LDS-DMA pieces, 2 = by 16-byte pieces (W % 4 == 0, aligned sources)
  int spw;  // depth pairs walked per workgroup
};
// Depth groups (pairs) per workgroup when the planner leaves it open (both engines) (r02 walk sweep,
// profiles/r02_wino2_walk_sweep.txt): walking 4 pairs gains 4-17 % on the L0 layers
// (cin 8-32: 2-8 chunks per pair) and 2 on the 16-channel L1 cells, as long as about a
// full round of workgroups remains (walks that leave the chip half empty lose up to 5x
// on the small L2 volumes); pairs of 32 chunks (conv1/2) gain nothing from it.
inline int auto_walk(const ConvArgs& a, int B, int wg_per_cu) {
  const long long base = (long long)a.ntiles * a.ndz * B * a.ncob;
  const long long round = 256LL * wg_per_cu;
  if (a.cin / CIN_B > 16) return 1;
  int s = 1;
  while (s < 4 && base / (2 * s) >= round * 15 / 16) s *= 2;
  return s;
}

int run2(const Plan2& p, ConvArgs a, int B, hipStream_t st, bool cv);
// the PV = 3 tile's per-lane weight copy (16-byte slices) (appended to the packed weights of 32-cout
// blocks by lea_conv3d_wino_pack_weights), in floats, and its packer
long long lane_weights_floats(int cout, int cin);
long long lane_raw_floats(int cout, int cin);  // the raw-tap part of it (the W-transformed copy follows)
__global__ void pack_wino_lane_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                      int nchunks, long long total);
__global__ void pack_wino_lane_wpre_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                           int nchunks, long long total);
extern int g_wpre;  // lea_conv3d_wino2p_set_wpre
// F(4,3) x F(4,3) tile (conv3d_wino44.hip, r06): the layers of the pipelined W x D kernel when
// g_w44 (lea_conv3d_wino44_set); its per-lane weight section (the last of lane_weights_floats)
extern int g_w44;
extern int g_w44u;  // lea_conv3d_wino44_set_upre
extern int g_w44s;  // lea_conv3d_wino44_set_sched
extern int g_w44g;  // lea_conv3d_wino44_set_group
long long lane44_floats(int cout, int cin);
long long lane44_g_floats(int cout, int cin);  // the G_W' g part (the U copy follows)
__global__ void pack_wino44_lane_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                        int nchunks, long long total);
__global__ void pack_wino44_lane_u_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                          int nchunks, long long total);
int run44(ConvArgs a, int B, int spw, hipStream_t st);
const char* name2(const Plan2& p, bool cv);

// F(2,3) x F(2,3) tile for the 16-cout layers (conv3d_wino22.hip): the U section the packer
// appends for 16-cout blocks (floats), the host's shape / alignment check and the launch
long long u22_section(int cout, int cin);
bool wino22_ok(const ConvArgs& a);
int run22(ConvArgs a, int B, int spw, hipStream_t st);
__global__ void pack_wino22_kernel(const float* __restrict__ w, float* __restrict__ out, int cout, int cin,
                                   long long total);

}  // namespace wino
}  // namespace lea
