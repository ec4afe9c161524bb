// Cost-volume build: the left/right feature concat over D3 disparity planes.
// Replaces retrain/LEAStereo.py:34-48 (zero fill + 2*D3 strided slice copies) by
// one write-once pass: every output element is stored exactly once, so the
// kernel is bound by the B*2C*D3*H*W*4-byte write (HBM roofline).
//
// Mapping: grid.y walks output planes p = (b*2C + c2)*D3 + i; inside a plane a
// thread owns 4 consecutive w of one row and stores them as one 16-byte vector
// (W % 4 == 0).  Left-half reads are aligned float4; right-half reads are shifted
// by i and served by L1/L2 (each feature row is re-read by all D3 planes).
#include "common.h"

namespace lea {

template <bool VEC>
__global__ __launch_bounds__(256) void cost_volume_f32(const float* __restrict__ left,
                                                       const float* __restrict__ right,
                                                       float* __restrict__ cost, int C, int H,
                                                       int W, int D3, int planes) {
  const int wq = VEC ? (W >> 2) : W;
  const int per_plane = H * wq;
  for (int p = blockIdx.y; p < planes; p += gridDim.y) {
    const int i = p % D3;
    const int bc = p / D3;  // b*2C + c2
    const int c2 = bc % (2 * C);
    const int b = bc / (2 * C);
    const bool is_left = c2 < C;
    const int c = is_left ? c2 : c2 - C;
    const float* src = (is_left ? left : right) + ((size_t)b * C + c) * H * W;
    float* dst = cost + (size_t)p * H * W;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < per_plane; t += gridDim.x * blockDim.x) {
      const int h = t / wq;
      const int q = t - h * wq;
      const float* s = src + h * W;
      if (VEC) {
        const int w0 = q * 4;
        float4 v;
        if (is_left && w0 >= i) {
          v = *reinterpret_cast<const float4*>(s + w0);
        } else {
          float e[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int w = w0 + k;
            e[k] = (w >= i) ? s[is_left ? w : w - i] : 0.f;
          }
          v = make_float4(e[0], e[1], e[2], e[3]);
        }
        *reinterpret_cast<float4*>(dst + h * W + w0) = v;
      } else {
        dst[h * W + q] = (q >= i) ? s[is_left ? q : q - i] : 0.f;
      }
    }
  }
}

}  // namespace lea

extern "C" int lea_build_cost_volume(const void* left, const void* right, void* cost, int B,
                                     int C, int H, int W, int D3, int dtype, void* stream) {
  using namespace lea;
  clear_error();
  LEA_CHECK_ARG(left && right && cost, "lea_build_cost_volume: null pointer");
  LEA_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0 && D3 > 0,
                "lea_build_cost_volume: bad shape B=%d C=%d H=%d W=%d D3=%d", B, C, H, W, D3);
  LEA_CHECK_ARG((long long)H * W < (1LL << 31) && (long long)B * 2 * C * D3 < (1LL << 31),
                "lea_build_cost_volume: shape too large");
  if (dtype != LEA_F32) {
    set_error("lea_build_cost_volume: dtype %d unsupported", dtype);
    return LEA_E_UNSUPPORTED;
  }
  const int planes = B * 2 * C * D3;
  const bool vec = (W % 4) == 0;
  const int per_plane = H * (vec ? W / 4 : W);
  const int threads = 256;
  // ~4 cells per thread (grid stride inside the plane): fewer, fatter workgroups
  const int gx = (per_plane + threads * 4 - 1) / (threads * 4);
  dim3 grid(gx, planes < 65535 ? planes : 65535);
  if (vec)
    cost_volume_f32<true><<<grid, threads, 0, as_stream(stream)>>>(
        (const float*)left, (const float*)right, (float*)cost, C, H, W, D3, planes);
  else
    cost_volume_f32<false><<<grid, threads, 0, as_stream(stream)>>>(
        (const float*)left, (const float*)right, (float*)cost, C, H, W, D3, planes);
  return launch_status("lea_build_cost_volume");
}
