// Host-side AddressSanitizer run of the C-ABI boundary ("host ASan build of
// the argument checks").  Built by `make asan` from every csrc/*.hip unit compiled for
// the host only (-Xarch_host -fsanitize=address, no device code: nothing here launches
// a kernel), it drives each entry point through its argument validation -- null
// pointers, bad shapes, unsupported dtypes -- plus the pure host queries (sizes,
// workspace bytes, kernel names), and checks the documented error contract:
// LEA_E_INVALID / LEA_E_UNSUPPORTED with a non-empty lea_last_error(), 0 + "" after a
// good query.  Exit 0 = every check passed and ASan saw no error.
#include <cstdio>
#include <cstring>
#include <string>

#include "leastereo_hip.h"
#include "leastereo_hip_tuning.h"

static int g_fail = 0;

static void expect_err(const char* what, int rc, int want = LEA_E_INVALID) {
  const char* e = lea_last_error();
  if (rc != want || e == nullptr || e[0] == '\0') {
    std::printf("FAIL %s: rc=%d (want %d) err='%s'\n", what, rc, want, e ? e : "(null)");
    ++g_fail;
  }
}

static void expect_name(const char* what, const char* name, const char* prefix) {
  if (name == nullptr || std::strncmp(name, prefix, std::strlen(prefix)) != 0) {
    std::printf("FAIL %s: name '%s' (want prefix '%s')\n", what, name ? name : "(null)", prefix);
    ++g_fail;
  }
}

int main() {
  if (lea_abi_version() <= 0) {
    std::printf("FAIL abi version\n");
    ++g_fail;
  }
  // pure host queries: sizes, workspaces, the planner's kernel choices
  const size_t p3 = lea_conv3d_packed_floats(32, 64, 3), p1 = lea_conv3d_packed_floats(32, 64, 1);
  const size_t pw = lea_conv3d_wino_packed_floats(32, 64), p2 = lea_conv2d_packed_floats(32, 16);
  const size_t pb = lea_conv3d_packed_elems_bf16(32, 64, 3), p2b = lea_conv2d_packed_elems_bf16(32, 16);
  if (p3 < 32u * 64 * 27 || p1 < 32u * 64 || pw < 32u * 64 * 27 || p2 < 32u * 16 * 9 || pb < 32u * 64 * 27 ||
      p2b < 32u * 16 * 9) {
    std::printf("FAIL packed sizes %zu %zu %zu %zu %zu %zu\n", p3, p1, pw, p2, pb, p2b);
    ++g_fail;
  }
  if (lea_tapsum_workspace_bytes(1, 1, 96, 160, 64) == 0 || lea_standardize_workspace_bytes(2) == 0 ||
      lea_disparity_metrics_workspace_bytes(2, 576, 960) == 0) {
    std::printf("FAIL workspace queries\n");
    ++g_fail;
  }
  expect_name("wino name", lea_conv3d_wino_kernel_name(1, 128, 64, 32, 96, 160, 0), "conv3d_wino");
  expect_name("wino cv name", lea_conv3d_wino_kernel_name(1, 64, 32, 64, 192, 320, 1), "conv3d_wino");
  expect_name("direct name", lea_conv3d_kernel_name(1, 32, 16, 48, 80, 3, 0), "conv3d_");
  expect_name("direct 1x1 name", lea_conv3d_kernel_name(1, 32, 16, 48, 80, 1, 1), "conv");
  expect_name("cv name", lea_conv3d_costvolume_kernel_name(1, 32, 64, 192, 320), "conv3d_");
  expect_name("2d name", lea_conv2d_kernel_name(2, 32, 192, 320), "conv");
  expect_name("bf16 name", lea_conv3d_kernel_name_bf16(8, 64, 128, 32, 96, 160, 3, 0), "conv");

  // every compute entry: null pointers first, then a bad shape / dtype where the
  // pointers are valid host addresses (the checks never dereference them)
  float buf[64] = {};
  void* p = buf;
  float* f = buf;
  expect_err("cost volume null", lea_build_cost_volume(nullptr, p, p, 1, 4, 8, 8, 4, LEA_F32, nullptr));
  expect_err("cost volume shape", lea_build_cost_volume(p, p, f + 1, 0, 4, 8, 8, 4, LEA_F32, nullptr));
  expect_err("pack null", lea_conv3d_pack_weights(nullptr, f, 32, 64, 3, nullptr));
  expect_err("pack k", lea_conv3d_pack_weights(f, f + 1, 32, 64, 2, nullptr));
  expect_err("conv null", lea_conv3d_bnrelu(nullptr, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, p, 0,
                                            1, 4, 4, 4, 4, 4, 3, LEA_RELU, LEA_F32, nullptr));
  expect_err("conv shape", lea_conv3d_bnrelu(p, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, f + 8, 0,
                                             1, 4, 4, -1, 4, 4, 3, LEA_RELU, LEA_F32, nullptr));
  expect_err("conv scale/shift", lea_conv3d_bnrelu(p, 0, nullptr, 0, 0, f, f, nullptr, nullptr, 0, f + 8, 0,
                                                   1, 4, 4, 4, 4, 4, 3, LEA_RELU, LEA_F32, nullptr));
  expect_err("conv residual", lea_conv3d_bnrelu(p, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, f + 8, 0,
                                                1, 4, 4, 4, 4, 4, 3, LEA_RESIDUAL, LEA_F32, nullptr));
  expect_err("conv pair-sum", lea_conv3d_bnrelu(p, 0, f + 16, 0, 4, f, nullptr, nullptr, nullptr, 0, f + 8, 0,
                                                1, 8, 4, 4, 4, 4, 3, LEA_RELU | LEA_PAIR_SUM, LEA_F32, nullptr),
             LEA_E_UNSUPPORTED);
  expect_err("conv unknown flag", lea_conv3d_bnrelu(p, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, f + 8, 0,
                                                    1, 4, 4, 4, 4, 4, 3, 0x40u, LEA_F32, nullptr));
  expect_err("conv2d pair-sum", lea_conv2d_bnrelu(p, 0, f, nullptr, nullptr, nullptr, 0, f + 8, 0, 1, 4, 4, 4, 4,
                                                  LEA_PAIR_SUM, LEA_F32, nullptr),
             LEA_E_UNSUPPORTED);
  expect_err("resampled null", lea_conv3d_bnrelu_resampled(nullptr, 0, 2, 2, 2, f, nullptr, nullptr, nullptr, 0,
                                                           p, 0, 1, 4, 4, 4, 4, 4, 1, 0, LEA_F32, nullptr));
  expect_err("cv conv null", lea_conv3d_bnrelu_costvolume(nullptr, p, 0, f, nullptr, nullptr, p, 0, 1, 4, 4, 4,
                                                          4, 4, 0, LEA_F32, nullptr));
  expect_err("conv2d null", lea_conv2d_bnrelu(nullptr, 0, f, nullptr, nullptr, nullptr, 0, p, 0, 1, 4, 4, 4, 4,
                                              0, LEA_F32, nullptr));
  expect_err("conv2d pack null", lea_conv2d_pack_weights(nullptr, f, 4, 4, nullptr));
  expect_err("conv2d s3 null", lea_conv2d_s3_bnrelu(nullptr, 0, f, nullptr, nullptr, p, 0, 1, 3, 16, 9, 9, 0,
                                                    LEA_F32, nullptr));
  expect_err("stem null", lea_feature_stem_bnrelu(nullptr, 0, f, f, f, f, f, f, p, 0, 2, 3, 16, 32, 9, 9,
                                                  LEA_F32, nullptr));
  expect_err("resample null", lea_resample3d_trilinear(nullptr, 0, p, 0, 1, 4, 2, 2, 2, 4, 4, 4, 1, nullptr,
                                                       nullptr, 0, LEA_F32, nullptr));
  expect_err("resample alias", lea_resample3d_trilinear(p, 0, p, 0, 1, 4, 2, 2, 2, 4, 4, 4, 1, nullptr,
                                                        nullptr, 0, LEA_F32, nullptr));
  expect_err("resample dtype", lea_resample3d_trilinear(p, 0, f + 8, 0, 1, 4, 2, 2, 2, 4, 4, 4, 1, nullptr,
                                                        nullptr, 0, 77, nullptr),
             LEA_E_UNSUPPORTED);
  expect_err("tapsum null", lea_tapsum_upsample(nullptr, 0, p, 0, 1, 1, 2, 2, 2, 4, 4, 4, nullptr, nullptr, 0,
                                                p, LEA_F32, nullptr));
  expect_err("disparity null", lea_disparity_regression(nullptr, f, 1, 4, 4, 4, 12, LEA_F32, nullptr));
  expect_err("disparity shape", lea_disparity_regression(p, f, 1, 0, 4, 4, 12, LEA_F32, nullptr));
  expect_err("disparity dtype", lea_disparity_regression(p, f, 1, 4, 4, 4, 12, 77, nullptr), LEA_E_UNSUPPORTED);
  expect_err("bf16 pack null", lea_conv3d_pack_weights_bf16(nullptr, p, 16, 16, 3, nullptr));
  expect_err("bf16 conv null", lea_conv3d_bnrelu_bf16(nullptr, 0, nullptr, 0, 0, p, nullptr, nullptr, nullptr,
                                                      0, p, 0, 1, 16, 16, 4, 4, 4, 3, 0, nullptr));
  expect_err("bf16 conv cin", lea_conv3d_bnrelu_bf16(p, 0, nullptr, 0, 0, p, nullptr, nullptr, nullptr, 0,
                                                     f + 8, 0, 1, 12, 16, 4, 4, 4, 3, 0, nullptr));
  expect_err("bf16 cv null", lea_conv3d_bnrelu_costvolume_bf16(nullptr, p, 0, p, nullptr, nullptr, p, 0, 1, 16,
                                                               16, 4, 4, 4, 0, nullptr));
  expect_err("bf16 rs1x1 null", lea_conv1x1_resampled_bf16(nullptr, 0, 2, 2, 2, p, nullptr, nullptr, p, 0, 1,
                                                           32, 16, 4, 4, 4, 0, nullptr));
  expect_err("bf16 resample null", lea_resample3d_trilinear_bf16(nullptr, 0, p, 0, 1, 8, 2, 2, 2, 4, 4, 4, 1,
                                                                 nullptr, nullptr, 0, nullptr));
  expect_err("to_c8 null", lea_to_c8_bf16(nullptr, 0, p, 0, 1, 8, 64, nullptr));
  expect_err("from_c8 null", lea_from_c8_bf16(nullptr, 0, f, 0, 1, 8, 64, nullptr));
  expect_err("bf16 conv2d null", lea_conv2d_bnrelu_bf16(nullptr, 0, p, nullptr, nullptr, nullptr, 0, p, 0, 1, 16,
                                                        16, 4, 4, 0, nullptr));
  expect_err("bf16 conv2d pack null", lea_conv2d_pack_weights_bf16(nullptr, p, 16, 16, nullptr));
  expect_err("wino pack null", lea_conv3d_wino_pack_weights(nullptr, f, 32, 64, nullptr));
  expect_err("wino null", lea_conv3d_bnrelu_wino(nullptr, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, p,
                                                 0, 1, 8, 16, 4, 4, 4, 0, LEA_F32, nullptr));
  expect_err("wino cin", lea_conv3d_bnrelu_wino(p, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, f + 8, 0,
                                                1, 6, 16, 4, 4, 4, 0, LEA_F32, nullptr));
  expect_err("wino alias", lea_conv3d_bnrelu_wino(p, 0, nullptr, 0, 0, f, nullptr, nullptr, nullptr, 0, p, 0,
                                                  1, 8, 16, 4, 4, 4, 0, LEA_F32, nullptr));
  expect_err("wino cv null", lea_conv3d_bnrelu_costvolume_wino(nullptr, p, 0, f, nullptr, nullptr, p, 0, 1, 8,
                                                               16, 4, 4, 4, 0, LEA_F32, nullptr));
  expect_err("cv split null", lea_cv_stem_split_weights(nullptr, f, f, 32, 32, nullptr));
  expect_err("cv combine null", lea_cv_stem_combine(nullptr, 0, p, 0, nullptr, nullptr, p, 0, 1, 32, 4, 4, 8, 0,
                                                    LEA_F32, nullptr));
  expect_err("standardize null", lea_standardize_crop_u8(nullptr, p, 1, 8, 8, 3, f, f, 8, 8, p, nullptr));
  expect_err("metrics null", lea_disparity_metrics(nullptr, 0, f, 0, 1, 4, 4, 192.f, 0, 0, 1, 2, 3, nullptr,
                                                   nullptr, p, nullptr));
  // training backward (csrc/conv3d_grad.hip)
  if (lea_conv3d_wgrad_workspace_bytes(1, 16, 16, 4, 8, 70, 3) == 0 || lea_bn_workspace_bytes(16) == 0 ||
      lea_conv3d_wgrad_workspace_bytes(1, 16, 16, 4, 8, 70, 5) != 0) {
    std::printf("FAIL training workspace queries\n");
    ++g_fail;
  }
  expect_err("wgrad null", lea_conv3d_wgrad(nullptr, f, f, p, 1 << 20, 1, 16, 16, 4, 8, 70, 3, nullptr));
  expect_err("wgrad k", lea_conv3d_wgrad(f, f, f, p, 1 << 20, 1, 16, 16, 4, 8, 70, 5, nullptr));
  expect_err("wgrad workspace", lea_conv3d_wgrad(f, f, f, p, 4, 1, 16, 16, 4, 8, 70, 3, nullptr));
  expect_err("flip alias", lea_conv3d_flip_weights(f, f, 16, 16, 3, nullptr));
  expect_err("bn fwd null", lea_bn_forward_f32(nullptr, f, 1, 16, 64, nullptr, nullptr, nullptr, nullptr, 0.1f,
                                               1e-5f, 1, 0, f, f, p, nullptr));
  expect_err("bn fwd eval stats", lea_bn_forward_f32(f, f, 1, 16, 64, nullptr, nullptr, nullptr, nullptr, 0.1f,
                                                     1e-5f, 0, 0, f, f, p, nullptr));
  expect_err("bn bwd relu y", lea_bn_backward_f32(f, nullptr, f, f, 1, 16, 64, nullptr, f, f, 1, LEA_RELU,
                                                  nullptr, nullptr, p, nullptr));
  expect_err("resample bwd null", lea_resample3d_trilinear_backward(nullptr, f, p, 1 << 20, 1, 2, 4, 4, 4, 8, 8,
                                                                    8, 1, nullptr));
  expect_err("resample bwd ws", lea_resample3d_trilinear_backward(f, f + 64, p, 4, 1, 2, 4, 4, 4, 8, 8, 8, 1,
                                                                  nullptr));
  expect_err("disp bwd null", lea_disparity_regression_backward(nullptr, f, f, f, 1, 8, 4, 4, 24, nullptr));
  expect_err("cv bwd alias", lea_build_cost_volume_backward(f, f, f, 1, 4, 4, 4, 4, nullptr));
  // tuning hooks: out-of-range values are rejected
  expect_err("walk range", lea_conv3d_wino2_set_walk(-1));
  expect_err("resample batch range", lea_resample_bf16_set_batch(3));
  // after a good query the error string is cleared
  (void)lea_conv3d_wino2_set_walk(0);
  if (lea_last_error() == nullptr || lea_last_error()[0] != '\0') {
    std::printf("FAIL error not cleared: '%s'\n", lea_last_error() ? lea_last_error() : "(null)");
    ++g_fail;
  }
  std::printf("%s: %d failed checks\n", g_fail ? "FAIL" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
