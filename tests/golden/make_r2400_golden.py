#!/usr/bin/env python3
"""Golden fixtures of the 2400 bps MELP mode from the REFERENCE codec.

The reference never runs its RATE2400 code through melpe_i; oracle/ref_tool
enc24gen / dec24gen set the globals as melpe_i would for RATE2400 and call
the reference's own npp / analysis / synthesis per 180-sample frame
(oracle/ref_tool.c init2400).  Inputs from the integer generator
(csrc/synth.h) so every fixture is reproducible from (seed, channel).

  r2400.json  enc: per-channel SHA-256 of the 54-bit frames (7 bytes each)
                   and of the NPP output, full frames of the first channels
              dec: per-channel SHA-256 of the PCM those frames decode to
              fuzz: PCM SHA-256 of uniformly random 7-byte frames (the
                   erasure, Hamming and invalid-pitch paths), frames from
                   numpy's PCG64(seed)
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
SEED, CHANNELS, FRAMES, KEEP = 7, 64, 450, 4
FUZZ_SEED, FUZZ_CHANNELS, FUZZ_FRAMES = 99, 64, 300


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def ref(*args):
    subprocess.run([TOOL, "jobs", "8"] + [str(a) for a in args], check=True)


def fuzz_frames(seed=FUZZ_SEED, channels=FUZZ_CHANNELS, frames=FUZZ_FRAMES):
    b = np.random.default_rng(seed).integers(0, 256, (channels, frames, 7)).astype(np.uint8)
    b[:, :, 6] &= 0x3F          # 54 bits: the last byte carries bits 48..53
    return b


def main():
    with tempfile.TemporaryDirectory() as tmp:
        bits, npp, pcm = (os.path.join(tmp, n) for n in ("e.bits", "e.npp", "d.pcm"))
        ref("enc24gen", SEED, 0, CHANNELS, FRAMES, bits, npp)
        ref("dec24gen", bits, CHANNELS, FRAMES, pcm)
        b = np.fromfile(bits, np.uint8).reshape(CHANNELS, FRAMES * 7)
        y = np.fromfile(npp, np.int16).reshape(CHANNELS, FRAMES * 180)
        p = np.fromfile(pcm, np.int16).reshape(CHANNELS, FRAMES * 180)
        fz = fuzz_frames()
        fb, fp = os.path.join(tmp, "f.bits"), os.path.join(tmp, "f.pcm")
        fz.tofile(fb)
        ref("dec24gen", fb, FUZZ_CHANNELS, FUZZ_FRAMES, fp)
        q = np.fromfile(fp, np.int16).reshape(FUZZ_CHANNELS, FUZZ_FRAMES * 180)
    doc = {"what": "2400 bps MELP (RATE2400) via the reference's npp/analysis/synthesis, "
                   "oracle/ref_tool enc24gen/dec24gen",
           "seed": SEED, "channels": CHANNELS, "frames": FRAMES,
           "bits_sha256": [sha(b[c]) for c in range(CHANNELS)],
           "npp_sha256": [sha(y[c].tobytes()) for c in range(CHANNELS)],
           "pcm_sha256": [sha(p[c].tobytes()) for c in range(CHANNELS)],
           "bits_hex": [b[c].tobytes().hex() for c in range(KEEP)],
           "fuzz": {"seed": FUZZ_SEED, "channels": FUZZ_CHANNELS, "frames": FUZZ_FRAMES,
                    "pcm_sha256": [sha(q[c].tobytes()) for c in range(FUZZ_CHANNELS)]}}
    json.dump(doc, open(os.path.join(HERE, "r2400.json"), "w"), indent=1)
    print("wrote r2400.json")


if __name__ == "__main__":
    sys.exit(main())
