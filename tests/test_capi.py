"""The C-ABI library loads and exports every symbol include/*.h declares (CPU:
only argument-checking paths are called, nothing launches)."""
import ctypes
import glob
import os
import re

import pytest

from leastereo_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(lea_\w+)\s*\(", src))
    return names


def test_header_and_binding_agree():
    assert declared_symbols() == set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.lea_abi_version() == _lib.ABI_VERSION


def test_invalid_arguments_are_rejected_before_launch():
    lib = _lib.load()
    assert lib.lea_build_cost_volume(None, None, None, 1, 1, 1, 1, 1, 0, None) == 1001
    assert b"null" in lib.lea_last_error()
    assert lib.lea_conv3d_bnrelu(None, 0, None, 0, 0, None, None, None, None, 0, None, 0,
                                 1, 1, 1, 1, 1, 1, 3, 1, 0, None) == 1001
    x = ctypes.c_void_p(16)
    y = ctypes.c_void_p(32)
    # scale without shift
    assert lib.lea_conv3d_bnrelu(x, 0, None, 0, 0, x, x, None, None, 0, y, 0,
                                 1, 1, 1, 1, 1, 1, 3, 1, 0, None) == 1001
    # second source announced but missing
    assert lib.lea_conv3d_bnrelu(x, 0, None, 0, 4, x, None, None, None, 0, y, 0,
                                 1, 8, 1, 1, 1, 1, 3, 1, 0, None) == 1001
    # output aliasing the input
    assert lib.lea_conv3d_bnrelu(x, 0, None, 0, 0, x, None, None, None, 0, x, 0,
                                 1, 1, 1, 1, 1, 1, 3, 1, 0, None) == 1001
    assert lib.lea_conv3d_bnrelu_resampled(x, 0, 0, 1, 1, x, None, None, None, 0, y, 0,
                                           1, 1, 1, 1, 1, 1, 1, 1, 0, None) == 1001
    assert b"input volume" in lib.lea_last_error()
    assert lib.lea_conv3d_kernel_name(1, 32, 64, 192, 320, 3, 0) == b"conv3d_dma_kernel<2, 2, 16, 2, 3, false>"
    assert lib.lea_conv3d_kernel_name(1, 32, 16, 48, 80, 3, 0) == b"conv3d_dma_kernel<2, 2, 16, 1, 3, false>"
    # tuning override: forced tile, then back to the planner; bad tiles rejected
    assert lib.lea_conv3d_set_tile_override(4, 64, 2) == 0
    assert lib.lea_conv3d_kernel_name(1, 32, 64, 192, 320, 3, 0) == b"conv3d_dma_kernel<2, 4, 64, 2, 3, false>"
    assert lib.lea_conv3d_set_tile_override(0, 0, 0) == 0
    assert lib.lea_conv3d_kernel_name(1, 32, 64, 192, 320, 3, 0) == b"conv3d_dma_kernel<2, 2, 16, 2, 3, false>"
    assert lib.lea_conv3d_set_tile_override(3, 16, 2) == 1001
    assert lib.lea_conv3d_kernel_name(1, 8, 16, 48, 80, 1, 1) == b"conv1x1_rs_f32_kernel<1>"
    assert lib.lea_conv3d_set_rs_gather(0) == 0
    try:
        assert lib.lea_conv3d_kernel_name(1, 8, 64, 192, 320, 1, 1).startswith(b"conv3d_reg_kernel<1, 1")
    finally:
        lib.lea_conv3d_set_rs_gather(1)
    assert lib.lea_conv3d_kernel_name(1, 8, 32, 96, 160, 1, 0) == b"conv1x1_kernel<1, 4>"
    assert lib.lea_conv1x1_set_vector(2) == 1001 and lib.lea_conv1x1_set_vector(1) == 0
    # unsupported dtype is reported as such
    assert lib.lea_disparity_regression(x, x, 1, 1, 1, 1, 1, 7, None) == 1002
    # LEA_PAIR_SUM on an entry without a pair form is LEA_E_UNSUPPORTED (the header's
    # contract; ADVICE r05: the direct engine had run a plain conv over the concatenation),
    # unknown flag bits LEA_E_INVALID -- both before any launch
    x2 = ctypes.c_void_p(48)
    pair, relu = 4, 1
    assert lib.lea_conv3d_bnrelu(x, 0, x2, 0, 4, x, None, None, None, 0, y, 0,
                                 1, 8, 4, 4, 4, 4, 3, relu | pair, 0, None) == 1002
    assert b"LEA_PAIR_SUM" in lib.lea_last_error()
    assert lib.lea_conv3d_bnrelu(x, 0, None, 0, 0, x, None, None, None, 0, y, 0,
                                 1, 8, 4, 4, 4, 4, 3, relu | 64, 0, None) == 1001
    assert b"unknown flag" in lib.lea_last_error()
    assert lib.lea_conv3d_bnrelu_resampled(x, 0, 2, 2, 2, x, None, None, None, 0, y, 0,
                                           1, 8, 4, 4, 4, 4, 1, pair, 0, None) == 1002
    assert lib.lea_conv2d_bnrelu(x, 0, x, None, None, None, 0, y, 0, 1, 8, 8, 4, 4, pair, 0, None) == 1002
    assert lib.lea_conv3d_bnrelu_costvolume(x, x2, 0, x, None, None, y, 0, 1, 8, 8, 4, 4, 4,
                                            pair, 0, None) == 1002
    assert lib.lea_resample3d_trilinear(x, 0, y, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, None, None, pair, 0,
                                        None) == 1002
    assert lib.lea_resample3d_trilinear(x, 0, y, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, None, None, 2, 0,
                                        None) == 1001
    # the pair entries still accept it (rejected later only for an unsupported shape)
    assert lib.lea_conv3d_bnrelu_wino(x, 0, None, 0, 0, x, None, None, None, 0, y, 0,
                                      1, 8, 4, 4, 4, 4, relu | 64, 0, None) == 1001
    assert lib.lea_resample3d_trilinear(x, 0, x, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, None, None, 0, 0,
                                        None) == 1001
    assert lib.lea_resample3d_trilinear(x, 0, y, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, x, None, 0, 0,
                                        None) == 1001


@pytest.mark.parametrize("cout,cin,k", [(32, 64, 3), (64, 128, 3), (16, 16, 3), (8, 8, 3), (3, 5, 3),
                                        (1, 32, 3), (16, 64, 1), (32, 128, 1), (8, 64, 1),
                                        (128, 256, 1), (80, 12, 3)])
def test_packed_sizes(cout, cin, k):
    n = _lib.load().lea_conv3d_packed_floats(cout, cin, k)
    cin_b = 4 if k == 3 else 32
    if cout <= 48:
        mt = -(-cout // 16)
    else:
        mt = 3 if -(-cout // 48) * 48 < -(-cout // 64) * 64 else 4
    cops = mt * 16  # no padding: 32/64-wide rows are XOR-swizzled instead
    if k == 3 and 2 < cout <= 8:  # depth-paired: 4 input planes x 9 taps, 16 = 2 planes x 8
        assert n == -(-cin // cin_b) * 36 * cin_b * 16
    else:
        assert n == -(-cout // (mt * 16)) * -(-cin // cin_b) * k ** 3 * cin_b * cops
    assert _lib.load().lea_conv3d_packed_floats(16, 8, 5) == 0


def test_tuning_setters_reject_out_of_range_values():
    """The round-6 tuning setters (include/leastereo_hip_tuning.h) take their documented ranges
    and refuse the rest with LEA_E_INVALID, leaving the setting as it was (CPU: no launch)."""
    lib = _lib.load()
    cases = [("lea_conv3d_wino44_set", (0, 3), 2), ("lea_conv3d_wino44_set_group", (-1, 16), -1),
             ("lea_conv3d_wino44_set_sched", (0, 3), 0), ("lea_conv3d_wino44_set_upre", (0, 1), 0),
             ("lea_conv3d_wino2p_set_wpre", (0, 1), 1), ("lea_disparity_set_register_form", (0, 4), 4)]
    for name, (lo, hi), default in cases:
        fn = getattr(lib, name)
        assert fn(lo - 1) == 1001 and fn(hi + 1) == 1001, name
        assert name.encode() in lib.lea_last_error(), lib.lea_last_error()
        assert fn(lo) == 0 and fn(hi) == 0 and fn(default) == 0, name
