"""ctypes binding of libleastereo_hip.so (include/leastereo_hip.h).

Loading fails loudly: there is no CPU or eager fallback for the hot path.
"""
from __future__ import annotations

import ctypes
import os
import threading

LIB_PATH = os.environ.get(
    "LEASTEREO_HIP_LIB",
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "libleastereo_hip.so"))

ABI_VERSION = 13
LEA_F32 = 0
LEA_BF16 = 1
LEA_RELU = 1
LEA_RESIDUAL = 2
LEA_PAIR_SUM = 4
LEA_E_INVALID = 1001

_p = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_u = ctypes.c_uint

# name -> (restype, argtypes); exactly the symbols include/leastereo_hip.h and
# include/leastereo_hip_tuning.h declare
SIGNATURES = {
    "lea_abi_version": (_i, []),
    "lea_last_error": (ctypes.c_char_p, []),
    "lea_build_cost_volume": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "lea_conv3d_packed_floats": (ctypes.c_size_t, [_i, _i, _i]),
    "lea_conv3d_pack_weights": (_i, [_p, _p, _i, _i, _i, _p]),
    "lea_conv3d_bnrelu": (_i, [_p, _i64, _p, _i64, _i, _p, _p, _p, _p, _i64, _p, _i64,
                               _i, _i, _i, _i, _i, _i, _i, _u, _i, _p]),
    "lea_conv3d_bnrelu_resampled": (_i, [_p, _i64, _i, _i, _i, _p, _p, _p, _p, _i64, _p, _i64,
                                         _i, _i, _i, _i, _i, _i, _i, _u, _i, _p]),
    "lea_conv3d_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i, _i, _i, _i]),
    "lea_conv3d_set_tile_override": (_i, [_i, _i, _i]),
    "lea_conv3d_bnrelu_costvolume": (_i, [_p, _p, _i64, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _i,
                                          _i, _u, _i, _p]),
    "lea_conv3d_costvolume_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i, _i]),
    "lea_conv2d_packed_floats": (ctypes.c_size_t, [_i, _i]),
    "lea_conv2d_pack_weights": (_i, [_p, _p, _i, _i, _p]),
    "lea_conv2d_bnrelu": (_i, [_p, _i64, _p, _p, _p, _p, _i64, _p, _i64, _i, _i, _i, _i, _i, _u,
                               _i, _p]),
    "lea_conv2d_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i]),
    "lea_conv2d_s3_bnrelu": (_i, [_p, _i64, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _i, _u, _i, _p]),
    "lea_feature_stem_bnrelu": (_i, [_p, _i64, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _i, _i,
                                     _i, _p]),
    "lea_resample3d_trilinear": (_i, [_p, _i64, _p, _i64, _i, _i, _i, _i, _i, _i, _i, _i,
                                      _i, _p, _p, _u, _i, _p]),
    "lea_tapsum_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i]),
    "lea_tapsum_upsample": (_i, [_p, _i64, _p, _i64, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _u,
                                 _p, _i, _p]),
    "lea_disparity_regression": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p]),
    # bf16 path (c8 layout)
    "lea_conv3d_packed_elems_bf16": (ctypes.c_size_t, [_i, _i, _i]),
    "lea_conv3d_pack_weights_bf16": (_i, [_p, _p, _i, _i, _i, _p]),
    "lea_conv3d_bnrelu_bf16": (_i, [_p, _i64, _p, _i64, _i, _p, _p, _p, _p, _i64, _p, _i64,
                                    _i, _i, _i, _i, _i, _i, _i, _u, _p]),
    "lea_conv3d_bnrelu_costvolume_bf16": (_i, [_p, _p, _i64, _p, _p, _p, _p, _i64, _i, _i, _i, _i,
                                               _i, _i, _u, _p]),
    "lea_conv3d_kernel_name_bf16": (ctypes.c_char_p, [_i, _i, _i, _i, _i, _i, _i, _i]),
    "lea_conv3d_bf16_pair_supported": (_i, [_i, _i, _i, _i, _i, _i]),
    "lea_conv3d_bf16_set_tile_override": (_i, [_i, _i, _i]),
    "lea_conv3d_bf16_set_variant": (_i, [_i]),
    "lea_resample3d_trilinear_bf16": (_i, [_p, _i64, _p, _i64, _i, _i, _i, _i, _i, _i, _i, _i,
                                           _i, _p, _p, _u, _p]),
    "lea_resample_bf16_set_batch": (_i, [_i]),
    "lea_resample_bf16_set_cols": (_i, [_i]),
    "lea_conv3d_wino_set_w22": (_i, [_i]),
    "lea_conv3d_bf16_set_pair_split": (_i, [_i]),
    "lea_disparity_set_register_form": (_i, [_i]),
    "lea_tapsum_set_rows": (_i, [_i]),
    "lea_staged_rows": (_i, [_i, _i, _i, _i, _i]),
    "lea_conv1x1_resampled_bf16": (_i, [_p, _i64, _i, _i, _i, _p, _p, _p, _p, _i64, _i, _i, _i, _i, _i,
                                        _i, _u, _p]),
    "lea_to_c8_bf16": (_i, [_p, _i64, _p, _i64, _i, _i, _i64, _p]),
    "lea_conv2d_packed_elems_bf16": (ctypes.c_size_t, [_i, _i]),
    "lea_conv2d_pack_weights_bf16": (_i, [_p, _p, _i, _i, _p]),
    "lea_conv2d_bnrelu_bf16": (_i, [_p, _i64, _p, _p, _p, _p, _i64, _p, _i64, _i, _i, _i, _i, _i,
                                    _u, _p]),
    "lea_from_c8_bf16": (_i, [_p, _i64, _p, _i64, _i, _i, _i64, _p]),
    # Winograd F(2,3)-along-W k=3 fp32 convs
    "lea_conv3d_wino_packed_floats": (ctypes.c_size_t, [_i, _i]),
    "lea_conv3d_wino_pack_weights": (_i, [_p, _p, _i, _i, _p]),
    "lea_conv3d_bnrelu_wino": (_i, [_p, _i64, _p, _i64, _i, _p, _p, _p, _p, _i64, _p, _i64,
                                    _i, _i, _i, _i, _i, _i, _u, _i, _p]),
    "lea_conv3d_bnrelu_costvolume_wino": (_i, [_p, _p, _i64, _p, _p, _p, _p, _i64, _i, _i, _i,
                                               _i, _i, _i, _u, _i, _p]),
    "lea_conv3d_wino_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i, _i, _i, _i]),
    "lea_conv3d_wino_set_tile_override": (_i, [_i, _i, _i]),
    "lea_conv3d_wino_set_variant": (_i, [_i]),
    "lea_conv3d_wino2_set_walk": (_i, [_i]),
    "lea_conv3d_wino2_set_halo16": (_i, [_i]),
    "lea_conv3d_wino2_set_lane_halo16": (_i, [_i]),
    "lea_conv3d_wino_set_fence": (_i, [_i]),
    "lea_resample_set_mode": (_i, [_i]),
    "lea_conv2d_set_small": (_i, [_i]),
    "lea_conv2d_kernel_name_cin": (ctypes.c_char_p, [_i, _i, _i, _i, _i]),
    "lea_conv2d_bnrelu_pair": (_i, [_p, _i64, _p, _p, _p, _p, _i64, _p, _i64, _p, _i64, _i, _i, _i, _i, _i,
                                    _i, _u, _p]),
    "lea_conv3d_wino2_set_pipeline": (_i, [_i]),
    "lea_conv3d_wino2p_set_wpre": (_i, [_i]),
    "lea_conv3d_wino44_set": (_i, [_i]),
    "lea_conv3d_wino44_set_upre": (_i, [_i]),
    "lea_conv3d_wino44_set_sched": (_i, [_i]),
    "lea_conv3d_wino44_set_group": (_i, [_i]),
    "lea_conv3d_wino_set_epi_buf": (_i, [_i]),
    "lea_conv3d_set_rs_gather": (_i, [_i]),
    "lea_conv1x1_set_vector": (_i, [_i]),
    "lea_conv3d_bf16_set_stream1x1": (_i, [_i]),
    "lea_conv3d_wino_set_small_cout": (_i, [_i]),
    "lea_conv3d_wino_set_block48": (_i, [_i]),
    # stem0 over the cost volume, factored through 2D maps
    "lea_cv_stem_split_weights": (_i, [_p, _p, _p, _i, _i, _p]),
    "lea_cv_stem_combine": (_i, [_p, _i64, _p, _i64, _p, _p, _p, _i64, _i, _i, _i, _i, _i, _u, _i,
                                 _p]),
    # host steps either side of forward: predict.py load_data/test_transform, metrics
    "lea_standardize_workspace_bytes": (ctypes.c_size_t, [_i]),
    "lea_standardize_crop_u8": (_i, [_p, _p, _i, _i, _i, _i, _p, _p, _i, _i, _p, _p]),
    "lea_disparity_metrics_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i]),
    "lea_disparity_metrics": (_i, [_p, _i64, _p, _i64, _i, _i, _i, ctypes.c_float, _i, _i,
                                   _i, _i, _i, _p, _p, _p, _p]),
    # training backward of ConvBR3d (csrc/conv3d_grad.hip)
    "lea_conv3d_wgrad_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i, _i, _i]),
    "lea_conv3d_wgrad": (_i, [_p, _p, _p, _p, ctypes.c_size_t, _i, _i, _i, _i, _i, _i, _i, _p]),
    "lea_conv2d_wgrad_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i]),
    "lea_conv2d_wgrad": (_i, [_p, _p, _p, _p, ctypes.c_size_t, _i, _i, _i, _i, _i, _p]),
    "lea_conv2d_s3_backward_data": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "lea_conv2d_s3_wgrad_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i]),
    "lea_conv2d_s3_wgrad": (_i, [_p, _p, _p, _p, ctypes.c_size_t, _i, _i, _i, _i, _i, _p]),
    "lea_conv3d_flip_weights": (_i, [_p, _p, _i, _i, _i, _p]),
    "lea_bn_workspace_bytes": (ctypes.c_size_t, [_i]),
    "lea_bn_forward_f32": (_i, [_p, _p, _i, _i, _i64, _p, _p, _p, _p, ctypes.c_float, ctypes.c_float,
                                _i, _u, _p, _p, _p, _p]),
    "lea_bn_backward_f32": (_i, [_p, _p, _p, _p, _i, _i, _i64, _p, _p, _p, _i, _u, _p, _p, _p, _p]),
    "lea_disparity_regression_backward": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "lea_build_cost_volume_backward": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "lea_resample3d_backward_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i, _i, _i, _i]),
    "lea_resample3d_trilinear_backward": (_i, [_p, _p, _p, ctypes.c_size_t, _i, _i, _i, _i, _i, _i, _i, _i,
                                               _i, _p]),
}

_lib = None
_lock = threading.Lock()


class HipKernelError(RuntimeError):
    pass


def load():
    """Load (once) and type the shared library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipKernelError(
                    f"{LIB_PATH} not found: build it with `make` (hipcc --offload-arch=gfx950); "
                    "the LEAStereo hot path has no fallback")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _apply_env_tuning(lib)
            _lib = lib
    return _lib


# A/B switches for the planners' tuning hooks (include/leastereo_hip_tuning.h; process-wide
# in the library), e.g. LEASTEREO_WINO2_WALK=1 to disable the depth walk
TUNING_ENV = {"LEASTEREO_WINO2_WALK": "lea_conv3d_wino2_set_walk",
              "LEASTEREO_HALO16": "lea_conv3d_wino2_set_halo16",
              "LEASTEREO_LANE_HALO16": "lea_conv3d_wino2_set_lane_halo16",
              "LEASTEREO_WINO_FENCE": "lea_conv3d_wino_set_fence",
              "LEASTEREO_RESAMPLE_MODE": "lea_resample_set_mode",
              "LEASTEREO_CONV2D_SMALL": "lea_conv2d_set_small",
              "LEASTEREO_WINO2_PIPE": "lea_conv3d_wino2_set_pipeline",
              "LEASTEREO_WINO2P_WPRE": "lea_conv3d_wino2p_set_wpre",
              "LEASTEREO_WINO44": "lea_conv3d_wino44_set",
              "LEASTEREO_WINO44_UPRE": "lea_conv3d_wino44_set_upre",
              "LEASTEREO_EPI_BUF": "lea_conv3d_wino_set_epi_buf",
              "LEASTEREO_RS_GATHER": "lea_conv3d_set_rs_gather",
              "LEASTEREO_1X1_VEC": "lea_conv1x1_set_vector",
              "LEASTEREO_BF16_1X1": "lea_conv3d_bf16_set_stream1x1",
              "LEASTEREO_RESAMPLE_K": "lea_resample_bf16_set_batch",
              "LEASTEREO_RESAMPLE_COLS": "lea_resample_bf16_set_cols",
              "LEASTEREO_W22": "lea_conv3d_wino_set_w22",
              "LEASTEREO_PAIR_SPLIT": "lea_conv3d_bf16_set_pair_split",
              "LEASTEREO_DISP_REG": "lea_disparity_set_register_form",
              "LEASTEREO_TAPSUM_ROWS": "lea_tapsum_set_rows"}


def _apply_env_tuning(lib):
    for var, fn in TUNING_ENV.items():
        if os.environ.get(var):
            if getattr(lib, fn)(int(os.environ[var])) != 0:
                raise HipKernelError(f"{var}={os.environ[var]}: {lib.lea_last_error().decode()}")


def check(rc: int, what: str):
    if rc != 0:
        msg = load().lea_last_error().decode(errors="replace")
        raise HipKernelError(f"{what} failed (rc={rc}): {msg}")
