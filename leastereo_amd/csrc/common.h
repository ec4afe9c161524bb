// Shared host/device helpers for libleastereo_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "leastereo_hip.h"
#include "leastereo_hip_tuning.h"

// Ablation switches (tools/wino2_ablate.sh, tools/wino2_stamps.py) knock phases out of
// the product kernels for timing; most of them make the outputs WRONG.  They only build
// together with LEA_ABLATION_BUILD, which the variant scripts set (never the Makefile).
#if !defined(LEA_ABLATION_BUILD) &&                                                      \
    (defined(LEA_EXP_STAMPS) || defined(LEA_EXP_NOWDMA) || defined(LEA_EXP_NOHALO) ||    \
     defined(LEA_EXP_NORES) || defined(LEA_EXP_NOSTORE) || defined(LEA_EXP_NOBAR1) ||    \
     defined(LEA_EXP_NOBAR2) || defined(LEA_EXP_NOVPASS) || defined(LEA_EXP_NOLDSRD) ||  \
     defined(LEA_EXP_NOXF) || defined(LEA_EXP_NOMFMA) || defined(LEA_EXP_NOWAIT) ||      \
     defined(LEA_EXP_STAGGER) || defined(LEA_EXP_NOUXF))
#error "LEA_EXP_* ablation switches give wrong outputs: build them only with -DLEA_ABLATION_BUILD"
#endif

namespace lea {

// Last error text of the calling host thread (lea_last_error()).
void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Map a launch result to the ABI return code, recording the HIP error string.
inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return LEA_OK;
}

#define LEA_CHECK_ARG(cond, ...)   \
  do {                             \
    if (!(cond)) {                 \
      ::lea::set_error(__VA_ARGS__); \
      return LEA_E_INVALID;        \
    }                              \
  } while (0)

// Epilogue flags an entry point accepts: LEA_PAIR_SUM where the entry has no
// pair form is LEA_E_UNSUPPORTED (the header's contract), any other bit outside `allowed`
// LEA_E_INVALID -- never silently a different computation.
#define LEA_CHECK_FLAGS(flags, allowed, who)                                                  \
  do {                                                                                       \
    const unsigned lea_f_ = (flags), lea_a_ = (allowed);                                     \
    if ((lea_f_ & LEA_PAIR_SUM) && !(lea_a_ & LEA_PAIR_SUM)) {                               \
      ::lea::set_error("%s: LEA_PAIR_SUM is not supported by this entry point", (who));      \
      return LEA_E_UNSUPPORTED;                                                              \
    }                                                                                        \
    if (lea_f_ & ~(lea_a_ | LEA_PAIR_SUM)) {                                                 \
      ::lea::set_error("%s: unknown flag bits 0x%x", (who), lea_f_ & ~(lea_a_ | LEA_PAIR_SUM)); \
      return LEA_E_INVALID;                                                                  \
    }                                                                                        \
  } while (0)

constexpr int kWave = 64;

// ---- trilinear interpolation with aten's source-index rule (UpSample.h:
// area_pixel_compute_scale / area_pixel_compute_source_index); shared by the
// resample kernel and the conv's resampling stager so both round identically.
struct Axis {
  int i0, i1;
  float l0, l1;
};

__host__ inline float axis_ratio(int in, int out, int ac) {
  if (ac) return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  return (float)in / (float)out;
}

__host__ __device__ __forceinline__ Axis axis_index(float ratio, int o, int in, int out, int ac) {
#pragma clang fp contract(off)
  Axis a;
  if (in == out) {
    a.i0 = a.i1 = o;
    a.l0 = 1.f;
    a.l1 = 0.f;
    return a;
  }
  float real = ac ? ratio * (float)o : ratio * ((float)o + 0.5f) - 0.5f;
  if (!ac && real < 0.f) real = 0.f;
  int i = (int)floorf(real);
  if (i > in - 1) i = in - 1;
  float lam = real - (float)i;
  lam = fminf(fmaxf(lam, 0.f), 1.f);
  a.i0 = i;
  a.i1 = i + ((i < in - 1) ? 1 : 0);
  a.l1 = lam;
  a.l0 = 1.f - lam;
  return a;
}

// Row-staged kernels (resample3d_rows/sep_f32, tapsum_hwpass_rows_f32): a workgroup owns
// output rows h0 .. h0 + R - 1 and stages the source rows that rows h0 - halo .. h0 + R - 1 +
// halo (clamped to the output) read.  The exact largest count over the blocks, from the
// kernels' own index expression on the host (the same IEEE float ops, contraction off), sizes
// their LDS; a kernel that ever sees more rows than this writes NaN instead of reading rows it
// never staged (lea_staged_rows exports it for the host sweep test).
__host__ inline int staged_rows(int Hi, int Ho, int ac, int R, int halo) {
  const float rh = axis_ratio(Hi, Ho, ac);
  int n = 0;
  for (int h0 = 0; h0 < Ho; h0 += R) {
    const int lo = axis_index(rh, h0 - halo > 0 ? h0 - halo : 0, Hi, Ho, ac).i0;
    const int e = h0 + R - 1 + halo;
    const int hi = axis_index(rh, e < Ho - 1 ? e : Ho - 1, Hi, Ho, ac).i1;
    n = hi - lo + 1 > n ? hi - lo + 1 : n;
  }
  return n;
}

// p{dz}{hy}: row pointers of source plane d_{dz}, row h_{hy}; nested-lerp order of
// aten's upsample_trilinear3d: t0*(h0*(w0*a + w1*b) + h1*(...)) + t1*(...)
__device__ __forceinline__ float trilerp(const Axis& ad, const Axis& ah, const Axis& aw,
                                         const float* p00, const float* p01, const float* p10,
                                         const float* p11) {
#pragma clang fp contract(off)
  return ad.l0 * (ah.l0 * (aw.l0 * p00[aw.i0] + aw.l1 * p00[aw.i1]) +
                  ah.l1 * (aw.l0 * p01[aw.i0] + aw.l1 * p01[aw.i1])) +
         ad.l1 * (ah.l0 * (aw.l0 * p10[aw.i0] + aw.l1 * p10[aw.i1]) +
                  ah.l1 * (aw.l0 * p11[aw.i0] + aw.l1 * p11[aw.i1]));
}

}  // namespace lea
