#!/usr/bin/env python3
"""Ablation builds kept out of the product sources.

The timing ablations of the Winograd engines (phases knocked out at compile time:
outputs WRONG, timing only) live as unified diffs under ``tools/ablation/`` against
the product sources in ``leastereo_amd/csrc``.  ``tools/build_variants.sh`` copies
the sources to ``build/var/src``, applies every patch there and compiles the variant
unit from that copy with ``-DLEA_ABLATION_BUILD``; the shipped library never sees an
``LEA_EXP_*`` switch.

    python tools/ablation.py strip UNIT...   # resolve LEA_EXP_* (undefined) in place,
                                            # writing tools/ablation/UNIT.patch
    python tools/ablation.py apply DIR       # patch the copy of csrc in DIR
"""
from __future__ import annotations

import difflib
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "leastereo_amd", "csrc")
PATCHES = os.path.join(REPO, "tools", "ablation")
_DIRECTIVE = re.compile(r"^\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b\s*(\S*)")


def strip(text: str) -> str:
    """The source with every ``#ifdef/#ifndef LEA_EXP_*`` block resolved as if the
    switch were undefined (nested non-ablation conditionals are kept verbatim)."""
    out, stack = [], []  # stack entries: [is_ablation, branch_kept]
    for line in text.splitlines(keepends=True):
        m = _DIRECTIVE.match(line)
        emitting = all(keep for abl, keep in stack if abl)
        if m:
            kind, arg = m.groups()
            if kind in ("ifdef", "ifndef") and arg.startswith("LEA_EXP_"):
                stack.append([True, kind == "ifndef"])
                continue
            if kind in ("if", "ifdef", "ifndef"):
                stack.append([False, True])
            elif stack and stack[-1][0]:
                if kind == "elif":
                    raise ValueError(f"#elif inside an ablation block: {line!r}")
                if kind == "else":
                    stack[-1][1] = not stack[-1][1]
                else:
                    stack.pop()
                continue
            elif kind == "endif":
                stack.pop()
        if emitting:
            out.append(line)
    if stack:
        raise ValueError("unbalanced conditionals")
    return "".join(out)


def cmd_strip(units):
    os.makedirs(PATCHES, exist_ok=True)
    for unit in units:
        path = os.path.join(CSRC, unit)
        with open(path) as f:
            full = f.read()
        prod = strip(full)
        if prod == full:
            print(f"{unit}: no ablation switches")
            continue
        diff = difflib.unified_diff(prod.splitlines(keepends=True), full.splitlines(keepends=True),
                                    f"a/{unit}", f"b/{unit}")
        with open(os.path.join(PATCHES, unit + ".patch"), "w") as f:
            f.writelines(diff)
        with open(path, "w") as f:
            f.write(prod)
        print(f"{unit}: {len(full.splitlines())} -> {len(prod.splitlines())} lines, patch written")


def cmd_apply(dest):
    for name in sorted(os.listdir(PATCHES)):
        if name.endswith(".patch"):
            subprocess.run(["patch", "-s", "-p1", "-d", dest, "-i", os.path.join(PATCHES, name)], check=True)


if __name__ == "__main__":
    if len(sys.argv) >= 3 and sys.argv[1] == "strip":
        cmd_strip(sys.argv[2:])
    elif len(sys.argv) == 3 and sys.argv[1] == "apply":
        cmd_apply(sys.argv[2])
    else:
        sys.exit(__doc__)
