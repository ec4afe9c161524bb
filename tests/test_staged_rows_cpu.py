"""The row-staged kernels' LDS bound, swept on the host.

resample3d_rows_f32 / resample3d_sep_f32 (every fp32 trilinear level change) and
tapsum_hwpass_rows_f32 (the head's up-sampled last_3) stage, per workgroup of R output
rows, the source rows those rows read (plus one output row either side for the tap-sum).
The LDS they get is ``lea_staged_rows`` (csrc/common.h staged_rows): the largest row
count over the blocks, from the kernels' own index rule.  This test restates aten's
source-index rule (UpSample.h area_pixel_compute_source_index, as oracle/torch_ref's
F.interpolate applies it) in numpy float32 and checks the exported bound is exactly that
maximum for every level change the configured shapes produce, plus a sweep of sizes; a
kernel meeting more rows than the bound writes NaN (never unstaged rows).
"""
import numpy as np
import pytest

from leastereo_amd import _lib
from leastereo_amd.arch import scale_dimension


def _source_rows(hi, ho, ac):
    """(i0, i1) per output row, float32 arithmetic as the kernels (contraction off)."""
    o = np.arange(ho, dtype=np.float32)
    if hi == ho:
        i = np.arange(ho)
        return i, i
    if ac:
        ratio = np.float32(hi - 1) / np.float32(ho - 1) if ho > 1 else np.float32(0)
        real = (np.float32(ratio) * o).astype(np.float32)
    else:
        ratio = np.float32(hi) / np.float32(ho)
        real = (np.float32(ratio) * (o + np.float32(0.5)).astype(np.float32)).astype(np.float32)
        real = (real - np.float32(0.5)).astype(np.float32)
        real = np.maximum(real, np.float32(0))
    i0 = np.minimum(np.floor(real).astype(np.int64), hi - 1)
    i1 = i0 + (i0 < hi - 1)
    return i0, i1


def _expected(hi, ho, ac, r, halo):
    i0, i1 = _source_rows(hi, ho, ac)
    n = 0
    for h0 in range(0, ho, r):
        lo = i0[max(h0 - halo, 0)]
        top = i1[min(h0 + r - 1 + halo, ho - 1)]
        # every row the block's outputs read lies in [lo, top]
        rows = np.concatenate([i0[max(h0 - halo, 0):min(h0 + r + halo, ho)],
                               i1[max(h0 - halo, 0):min(h0 + r + halo, ho)]])
        assert rows.min() >= lo and rows.max() <= top
        n = max(n, int(top - lo + 1))
    return n


def _configured_axes():
    """(Hi, Ho) of every trilinear H/W/D level change at the five configs:
    L0 <-> L1 <-> L2 <-> L3 by scale_dimension, and the head's up-samplings."""
    axes = set()
    for l0 in (32, 96, 192, 64, 128, 416, 320, 88, 336, 504, 16, 48):  # D3/H3/W3 of C1..C5, e2e
        n = l0
        for _ in range(3):
            down = scale_dimension(n, 0.5)
            axes |= {(n, down), (down, n), (down, scale_dimension(down, 2))}
            n = down
        axes |= {(l0 // 2, l0), (l0 // 4, l0 // 2), (l0 // 8, l0 // 4)}
    return sorted(a for a in axes if a[0] > 0 and a[1] > 0)


@pytest.mark.parametrize("halo,rs", [(0, (16, 8, 4, 2)), (1, (8, 4, 2))])
def test_staged_rows_bound_is_exact_on_configured_axes(halo, rs):
    lib = _lib.load()
    for hi, ho in _configured_axes():
        for r in rs:
            for ac in (1, 0):
                got = lib.lea_staged_rows(hi, ho, ac, r, halo)
                assert got == _expected(hi, ho, ac, r, halo), (hi, ho, ac, r, halo, got)


def test_staged_rows_sweep():
    lib = _lib.load()
    rng = np.random.default_rng(5)
    for _ in range(400):
        hi = int(rng.integers(1, 700))
        ho = int(rng.integers(1, 1400))
        r, halo, ac = int(rng.choice([2, 4, 8, 16])), int(rng.integers(0, 2)), int(rng.integers(0, 2))
        assert lib.lea_staged_rows(hi, ho, ac, r, halo) == _expected(hi, ho, ac, r, halo), (hi, ho, ac, r, halo)


def test_staged_rows_rejects_bad_arguments():
    lib = _lib.load()
    assert lib.lea_staged_rows(0, 4, 1, 8, 0) == -1
    assert b"lea_staged_rows" in lib.lea_last_error()
    assert lib.lea_staged_rows(4, 8, 2, 8, 0) == -1
