#!/usr/bin/env python3
"""Knockout builds of the lane analysis (diagnostics, never shipped):
build/var/ko_<stage>.so = the product library with k_ana.hip recompiled
under -DMELPE_KO_<STAGE> (encoder.h: the stage is skipped, so the output is
wrong by construction).  tools/gpu_r04_ko.sh prices each stage on MI355X by
the kernel-time and PMC-traffic difference against the product build.

  python tools/build_ko.py bpvc pauto classify lsfvq pitchana gpitch analysis
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pairphone_amd import build as b  # noqa: E402


def main(stages):
    base = os.path.join(ROOT, "build", "obj", "libmelpe_amd")
    assert os.path.exists(os.path.join(base, "k_ana.o")), "build the product library first"
    os.makedirs(os.path.join(ROOT, "build", "var"), exist_ok=True)
    for st in stages:
        out = os.path.join(ROOT, "build", "var", "ko_%s.so" % st)
        od = os.path.join(ROOT, "build", "obj", "ko_%s" % st)
        os.makedirs(od, exist_ok=True)
        for f in os.listdir(base):
            if f.endswith(".o") and f != "k_ana.o":
                shutil.copy2(os.path.join(base, f), os.path.join(od, f))
        b.build_engine(force=True, out=out, only=("k_ana",),
                       tus_defs={"k_ana": ["MELPE_KO_" + st.upper()]})


if __name__ == "__main__":
    main(sys.argv[1:])
