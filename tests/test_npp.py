"""NPP (melpe_n, melpe/npp.c) parity.

CPU: the host-emulation build of the device sources against the committed
golden hashes (reference outputs).  GPU: the HIP kernel against the same
golden hashes and, on more channels, against the reference run live through
oracle/_ref/ref_tool (one process per channel, as the reference keeps its
state in process globals).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT, GOLDEN, run_ref

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
TABLES = os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin")


def golden():
    return json.load(open(os.path.join(GOLDEN, "npp.json")))


def make_input(seed, channels, frames):
    from pairphone_amd import synth_signal
    n = frames * 180 + 76
    return np.stack([synth_signal(seed, c, n) for c in range(channels)])


def emu():
    lib = ctypes.CDLL(EMU)
    lib.emu_create.restype = ctypes.c_void_p
    lib.emu_create.argtypes = [ctypes.c_int]
    lib.emu_npp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.emu_destroy.argtypes = [ctypes.c_void_p]
    assert lib.emu_load_tables(TABLES.encode()) == 0
    return lib


def sha(a):
    return hashlib.sha256(a.tobytes()).hexdigest()


def test_npp_hostemu_matches_golden():
    g = golden()
    ch = 2
    x = make_input(g["seed"], ch, g["frames"])
    lib = emu()
    e = lib.emu_create(ch)
    lib.emu_npp(e, x.ctypes.data, g["frames"], x.shape[1], 1)
    lib.emu_destroy(e)
    for c in range(ch):
        assert sha(x[c, :g["frames"] * 180]) == g["sha256"][c], "channel %d" % c


@pytest.mark.gpu
def test_npp_gpu_matches_golden():
    from pairphone_amd import MelpeEngine
    g = golden()
    x = make_input(g["seed"], g["channels"], g["frames"])
    eng = MelpeEngine(g["channels"])
    eng.npp(x, g["frames"])
    for c in range(g["channels"]):
        assert sha(x[c, :g["frames"] * 180]) == g["sha256"][c], "channel %d" % c


@pytest.mark.gpu
def test_npp_gpu_matches_reference_live(tmp_path, ref_tool):
    from pairphone_amd import MelpeEngine
    ch, frames, seed = 128, 120, 5
    x = make_input(seed, ch, frames)
    ref = []
    for c in range(ch):
        p = str(tmp_path / ("c%d.pcm" % c))
        x[c].tofile(p)
        run_ref("npp", p, p + ".out")
        ref.append(np.fromfile(p + ".out", dtype=np.int16))
    eng = MelpeEngine(ch)
    # two launches of half the frames each: state must carry across calls
    y = x.copy()
    a = np.ascontiguousarray(y[:, :60 * 180 + 76])
    eng.npp(a, 60)
    b = np.ascontiguousarray(y[:, 60 * 180:])
    eng.npp(b, 60)
    out = np.concatenate([a[:, :60 * 180], b[:, :60 * 180]], axis=1)
    for c in range(ch):
        np.testing.assert_array_equal(out[c], ref[c], err_msg="channel %d" % c)
