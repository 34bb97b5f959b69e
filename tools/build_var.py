#!/usr/bin/env python3
"""A/B variant of the engine library: build/var/NAME.so, recompiling only the
named TUs (with extra -D defines) and linking them with the product build's
other objects (build/obj/libmelpe_amd/*.o, copied).  Several variants can
build in parallel (one hipcc per TU).

  python tools/build_var.py NAME TU[,TU...] [DEFINE ...]
  e.g. python tools/build_var.py noguard k_ana,k_ana_mw MELPE_FLAT_GUARD=0
"""
import glob
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pairphone_amd import build  # noqa: E402


def main(name, tus, defs):
    out = os.path.join(ROOT, "build", "var", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    objdir = os.path.join(ROOT, "build", "obj", name)
    os.makedirs(objdir, exist_ok=True)
    for o in glob.glob(os.path.join(ROOT, "build", "obj", "libmelpe_amd", "*.o")):
        shutil.copy(o, objdir)
    # compile from a snapshot of the sources: hipcc preprocesses the device
    # and host passes separately, minutes apart, and edits in between break
    # the build
    top = os.path.join(ROOT, "build", "src", name)
    snap = os.path.join(top, "pairphone_amd", "csrc")	# engine.hip includes ../../include
    shutil.rmtree(top, ignore_errors=True)
    shutil.copytree(build.CSRC, snap)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    build.CSRC = snap
    t0 = time.time()
    build.build_engine(force=True, defs=defs, out=out, only=tuple(tus))
    print("built %s in %.0f s" % (out, time.time() - t0), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2].split(","), sys.argv[3:])
