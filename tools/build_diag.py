#!/usr/bin/env python3
"""Diagnostic builds of the lane analysis (never shipped): build/var/<name>.so
= the product library with k_ana.hip recompiled under -D<DEFINE> (e.g.
MELPE_DIAG_UNIFORM_PITCH: every frac_pch / frac_cor at one lag, so the
pitch-dependent window reads are the same address on every lane; the
output is wrong by construction).

  python tools/build_diag.py <name> <DEFINE> [<DEFINE> ...]
  MELPE_DIAG_TU=k_ana_mw python tools/build_diag.py ...   (another TU)
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pairphone_amd import build as b  # noqa: E402


def main(name, defs):
    tu = os.environ.get("MELPE_DIAG_TU", "k_ana")
    base = os.path.join(ROOT, "build", "obj", "libmelpe_amd")
    assert os.path.exists(os.path.join(base, tu + ".o")), "build the product library first"
    os.makedirs(os.path.join(ROOT, "build", "var"), exist_ok=True)
    od = os.path.join(ROOT, "build", "obj", name)
    os.makedirs(od, exist_ok=True)
    for f in os.listdir(base):
        if f.endswith(".o") and f != tu + ".o":
            shutil.copy2(os.path.join(base, f), os.path.join(od, f))
    b.build_engine(force=True, out=os.path.join(ROOT, "build", "var", name + ".so"), only=(tu,),
                   tus_defs={tu: list(defs)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
