"""Host AddressSanitizer run of the C-ABI boundary: `make asan` builds every
unit with ASan on its host side (device code as usual, never launched) and runs
tests/asan/capi_asan.cpp, which drives each entry point through its argument checks
(null pointers, bad shapes, unsupported dtypes, aliased buffers) and the host queries
(packed sizes, workspaces, the planner's kernel names).  CPU only."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs make and hipcc")
def test_capi_argument_checks_under_asan():
    r = subprocess.run(["make", "-s", "-j8", "asan"], cwd=REPO, capture_output=True, text=True, timeout=1200)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "OK: 0 failed checks" in r.stdout, tail
    assert "AddressSanitizer" not in r.stderr, tail
