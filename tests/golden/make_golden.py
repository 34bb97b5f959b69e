#!/usr/bin/env python3
"""Generates the committed golden fixtures from the REFERENCE codec.

Runs only where /root/reference was compiled into oracle/_ref (the dev
container).  Inputs come from the integer generator csrc/synth.h (the same
generator the tests and the benchmark use), so every fixture is reproducible
from (seed, channel).  Each fixture stores the SHA-256 of the reference's
outputs (and, for small cases, the outputs themselves).

  npp.json   melpe_n over F frames per channel  (ref_tool npp)
  enc.json   melpe_a bitstreams, per channel     (ref_tool encgen)
  dec_1024.json  melpe_s PCM of the enc_1024 bitstreams (ref_tool decgen)
  dec_fuzz.json  melpe_s PCM of uniformly random bitstreams (FEC, parity and
                 erasure paths), bits regenerated from numpy's PCG64(seed)
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


def make_enc(tmp, seed, channels, nsf, keep_bits=0):
    """melpe_a goldens: per-channel SHA-256 of the bitstream and of the NPP
    output the reference leaves in the caller's buffer."""
    bits = os.path.join(tmp, "e.bits")
    npp = os.path.join(tmp, "e.npp")
    ref("encgen", seed, 0, channels, nsf, bits, npp)
    b = np.fromfile(bits, dtype=np.uint8).reshape(channels, nsf * 11)
    y = np.fromfile(npp, dtype=np.int16).reshape(channels, nsf * 540)
    out = {"seed": seed, "channels": channels, "superframes": nsf,
           "bits_sha256": [sha(b[c].tobytes()) for c in range(channels)],
           "npp_sha256": [sha(y[c].tobytes()) for c in range(channels)]}
    if keep_bits:
        out["bits_hex"] = [b[c].tobytes().hex() for c in range(keep_bits)]
    return out


def make_dec(tmp, seed, channels, nsf):
    bits = os.path.join(tmp, "d.bits")
    ref("encgen", seed, 0, channels, nsf, bits)
    pcm = os.path.join(tmp, "d.pcm")
    ref("decgen", bits, channels, nsf, pcm)
    y = np.fromfile(pcm, dtype=np.int16).reshape(channels, nsf * 540)
    return {"seed": seed, "channels": channels, "superframes": nsf,
            "pcm_sha256": [sha(y[c].tobytes()) for c in range(channels)]}


def fuzz_bits(seed, channels, nsf):
    return np.random.Generator(np.random.PCG64(seed)).integers(
        0, 256, (channels, nsf * 11), dtype=np.uint8)


def make_dec_fuzz(tmp, seed, channels, nsf):
    bits = os.path.join(tmp, "f.bits")
    fuzz_bits(seed, channels, nsf).tofile(bits)
    pcm = os.path.join(tmp, "f.pcm")
    ref("decgen", bits, channels, nsf, pcm)
    y = np.fromfile(pcm, dtype=np.int16).reshape(channels, nsf * 540)
    return {"seed": seed, "channels": channels, "superframes": nsf,
            "pcm_sha256": [sha(y[c].tobytes()) for c in range(channels)],
            "pcm0_first_sf": y[0, :540].tolist()}


def main():
    if not os.path.exists(TOOL):
        sys.exit("oracle/_ref/ref_tool missing")
    which = sys.argv[1:] or ["npp"]
    with tempfile.TemporaryDirectory() as tmp:
        if "enc" in which:
            json.dump(make_enc(tmp, 1, 1024, 149, keep_bits=8),
                      open(os.path.join(HERE, "enc_1024.json"), "w"))
        if "dec" in which:
            json.dump(make_dec(tmp, 1, 1024, 149), open(os.path.join(HERE, "dec_1024.json"), "w"))
            json.dump(make_dec_fuzz(tmp, 77, 256, 200),
                      open(os.path.join(HERE, "dec_fuzz.json"), "w"))
        if "npp" in which:
            json.dump(make_npp(tmp), open(os.path.join(HERE, "npp.json"), "w"), indent=1)
    print("ok")


if __name__ == "__main__":
    main()
