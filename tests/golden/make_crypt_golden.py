#!/usr/bin/env python3
"""Generates tests/golden/voice_crypt.json from the REFERENCE sponge.

VoiceEnc / VoiceDec (crp.c:986-1027) driven through the reference's own
crypto/sponge.c, compiled where it lies into oracle/_ref/libref_crypt.so by
oracle/Makefile (harness oracle/ref_crypt.c).  Runs only in the dev
container.  Inputs are regenerated from numpy's PCG64(seed) by `inputs()`
(tests import it), with edge cases patched in: counter wrap-around at
2^32, the counters the call state machine uses (7, 65534, crp.c:471,807),
an all-zero and an all-0xFF key, the polarity-inversion flag.
"""
import ctypes
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_crypt.so")
SEED, C, K = 2026, 64, 8


def inputs(seed=SEED, C=C, K=K):
    rng = np.random.Generator(np.random.PCG64(seed))
    pkts = rng.integers(0, 256, (C, K, 11), dtype=np.uint8)
    pkts[..., 10] &= 1
    ctr = rng.integers(0, 2**32, C, dtype=np.uint64).astype(np.uint32)
    keys = rng.integers(0, 256, (C, 16), dtype=np.uint8)
    inv = (rng.random(C) < 0.5).astype(np.uint8)
    if C >= 4:
        ctr[0], ctr[1], ctr[2], ctr[3] = 0xFFFFFFFC, 0, 7, 65534
        keys[1] = 0
        keys[2] = 0xFF
    return pkts, ctr, keys, inv


def ref_crypt(pkts, ctr, keys, inv, direction):
    lib = ctypes.CDLL(LIB)
    out = np.ascontiguousarray(pkts, dtype=np.uint8).copy()
    P = ctypes.c_void_p
    lib.ref_voice_crypt(P(out.ctypes.data), P(ctr.ctypes.data), P(keys.ctypes.data),
                        None if inv is None else P(inv.ctypes.data),
                        out.shape[0], out.shape[1], direction)
    return out


def main():
    pkts, ctr, keys, inv = inputs()
    enc = ref_crypt(pkts, ctr, keys, None, 0)
    dec = ref_crypt(pkts, ctr, keys, inv, 1)
    doc = {
        "what": "VoiceEnc/VoiceDec (crp.c:986-1027) via reference crypto/sponge.c",
        "seed": SEED, "channels": C, "packets": K,
        "enc_hex": enc.tobytes().hex(), "dec_invert_hex": dec.tobytes().hex(),
        "enc_sha256": hashlib.sha256(enc.tobytes()).hexdigest(),
    }
    with open(os.path.join(HERE, "voice_crypt.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote voice_crypt.json")


if __name__ == "__main__":
    main()
