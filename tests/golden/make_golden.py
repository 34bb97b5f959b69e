#!/usr/bin/env python3
"""Generates the committed golden fixtures from the REFERENCE codec.

Runs only where /root/reference was compiled into oracle/_ref (the dev
container).  Inputs come from the integer generator csrc/synth.h (the same
generator the tests and the benchmark use), so every fixture is reproducible
from (seed, channel).  Each fixture stores the SHA-256 of the reference's
outputs (and, for small cases, the outputs themselves).

  npp.json   melpe_n over F frames per channel  (ref_tool npp)
  enc.json   melpe_a bitstreams, per channel     (ref_tool encgen)
  dec.json   melpe_s PCM of those bitstreams     (ref_tool decgen)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_tool")


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def ref(*args):
    subprocess.run([TOOL, "jobs", "8"] + [str(a) for a in args], check=True)


def gen(seed, ch, n, path):
    subprocess.run([TOOL, "gen", str(seed), str(ch), str(n), path], check=True)


def make_npp(tmp, seed=11, channels=8, frames=300):
    out = {"seed": seed, "channels": channels, "frames": frames, "sha256": []}
    for c in range(channels):
        inp = os.path.join(tmp, "n%d.pcm" % c)
        gen(seed, c, frames * 180 + 76, inp)
        ref("npp", inp, inp + ".out")
        y = np.fromfile(inp + ".out", dtype=np.int16)
        assert y.size == frames * 180
        out["sha256"].append(sha(y.tobytes()))
    return out


def main():
    if not os.path.exists(TOOL):
        sys.exit("oracle/_ref/ref_tool missing")
    which = sys.argv[1:] or ["npp"]
    with tempfile.TemporaryDirectory() as tmp:
        if "npp" in which:
            json.dump(make_npp(tmp), open(os.path.join(HERE, "npp.json"), "w"), indent=1)
    print("ok")


if __name__ == "__main__":
    main()
