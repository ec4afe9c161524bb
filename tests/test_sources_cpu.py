"""Product-source hygiene: no LEA_EXP_* ablation switch in the library's
sources; the ablation builds' patches (tools/ablation/*.patch) still apply to them and
restore every switch (tools/build_variants.sh compiles that patched copy)."""
import os
import re
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "leastereo_amd", "csrc")


def test_product_sources_have_no_ablation_switches():
    for name in sorted(os.listdir(CSRC)):
        with open(os.path.join(CSRC, name)) as f:
            text = f.read()
        hits = re.findall(r"^\s*#\s*if(?:n?def)?\b.*LEA_EXP_", text, re.M)
        assert not hits, (name, hits)


def test_ablation_patches_apply(tmp_path):
    dst = tmp_path / "csrc"
    shutil.copytree(CSRC, dst)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "ablation.py"), "apply", str(dst)], check=True)
    with open(dst / "conv3d_wino2.hip") as f:
        patched = f.read()
    for sw in ("LEA_EXP_NOMFMA", "LEA_EXP_NOHALO", "LEA_EXP_STAMPS", "LEA_EXP_NOVPASS"):
        assert f"#ifdef {sw}" in patched or f"#ifndef {sw}" in patched, sw
    # resolving the switches again gives back the product source exactly
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import ablation
    for unit in ("conv3d_wino2.hip", "conv3d_wino.hip", "wino_common.h"):
        with open(dst / unit) as f, open(os.path.join(CSRC, unit)) as g:
            assert ablation.strip(f.read()) == g.read(), unit
