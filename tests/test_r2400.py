"""The 2400 bps MELP mode: 180 samples <-> 54 bits.

The reference compiles this path but cannot reach it (melpe_i pins
RATE1200, melpe/melpe.c:76; melpe_i2 / melpe_al are declared at
melpe/melpe.c:57-58 without bodies).  Oracle: the reference's own npp /
analysis / synthesis at RATE2400, driven by oracle/ref_tool enc24gen /
dec24gen (globals set as melpe_i would for RATE2400); goldens in
tests/golden/r2400.json (make_r2400_golden.py): 64 channels x 450 frames
(10 s) encoded and decoded, plus 64 channels x 300 uniformly random frames
decoded (erasures, Hamming-protected unvoiced frames, invalid pitch codes).

CPU: the host build of codec2400.h.  GPU: melpe_encode2400 / decode2400
through the C ABI, the drop-in melpe_i2 / melpe_al / melpe_s, and 65,536
channels against the live reference on sampled channels.
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, GOLDEN, REF_TOOL

sys.path.insert(0, GOLDEN)
from make_r2400_golden import fuzz_frames  # noqa: E402

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
TABLES = os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin")


def sha(a):
    return hashlib.sha256(a.tobytes()).hexdigest()


def golden():
    return json.load(open(os.path.join(GOLDEN, "r2400.json")))


def inputs(seed, C, nfr):
    from pairphone_amd import synth_signal
    return np.stack([synth_signal(seed, c, nfr * 180) for c in range(C)]).reshape(C, nfr, 180)


def emu():
    lib = ctypes.CDLL(EMU)
    vp = ctypes.c_void_p
    lib.emu_create.restype = vp
    lib.emu_create.argtypes = [ctypes.c_int]
    lib.emu_destroy.argtypes = [vp]
    lib.emu_encode2400.argtypes = [vp, vp, vp]
    lib.emu_decode2400.argtypes = [vp, vp, vp]
    assert lib.emu_load_tables(TABLES.encode()) == 0
    return lib


def run_emu(x, bits_in=None):
    """x: C x nfr x 180 (encode + decode of its bits), or bits_in: C x nfr x
    7 (decode only).  Returns (bits, npp out, pcm)."""
    lib = emu()
    C, nfr = (x.shape[:2] if bits_in is None else bits_in.shape[:2])
    e = lib.emu_create(C)
    d = lib.emu_create(C)
    bits = np.zeros((C, nfr, 7), np.uint8) if bits_in is None else bits_in
    npp = np.zeros((C, nfr, 180), np.int16)
    pcm = np.zeros((C, nfr, 180), np.int16)
    for k in range(nfr):
        if bits_in is None:
            sp = np.ascontiguousarray(x[:, k])
            b = np.zeros((C, 7), np.uint8)
            lib.emu_encode2400(e, b.ctypes.data, sp.ctypes.data)
            bits[:, k] = b
            npp[:, k] = sp
        bk = np.ascontiguousarray(bits[:, k])
        out = np.zeros((C, 180), np.int16)
        lib.emu_decode2400(d, out.ctypes.data, bk.ctypes.data)
        pcm[:, k] = out
    lib.emu_destroy(e)
    lib.emu_destroy(d)
    return bits, npp, pcm


def check(g, bits, npp, pcm, chans):
    for c in chans:
        assert sha(bits[c]) == g["bits_sha256"][c], "bits, channel %d" % c
        assert sha(npp[c]) == g["npp_sha256"][c], "NPP output, channel %d" % c
        assert sha(pcm[c]) == g["pcm_sha256"][c], "PCM, channel %d" % c
        if c < len(g["bits_hex"]):
            assert bits[c].tobytes().hex() == g["bits_hex"][c]


def test_r2400_hostemu_matches_golden():
    g = golden()
    C = 6
    x = inputs(g["seed"], C, g["frames"])
    bits, npp, pcm = run_emu(x)
    check(g, bits, npp, pcm, range(C))


def test_r2400_hostemu_fuzz_decode_matches_golden():
    g = golden()["fuzz"]
    fz = fuzz_frames(g["seed"], 8, g["frames"])
    _, _, pcm = run_emu(None, fz)
    for c in range(8):
        assert sha(pcm[c]) == g["pcm_sha256"][c], "fuzz PCM, channel %d" % c


@pytest.mark.gpu
def test_r2400_gpu_matches_golden():
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nfr = g["channels"], g["frames"]
    x = inputs(g["seed"], C, nfr)
    enc, dec = MelpeEngine(C), MelpeEngine(C)
    bits = np.zeros((C, nfr, 7), np.uint8)
    npp = np.zeros((C, nfr, 180), np.int16)
    pcm = np.zeros((C, nfr, 180), np.int16)
    for k in range(nfr):
        sp = np.ascontiguousarray(x[:, k])
        bits[:, k] = enc.encode2400(sp)
        npp[:, k] = sp
        pcm[:, k] = dec.decode2400(bits[:, k])
    check(g, bits, npp, pcm, range(C))
    # random frames: erasure / FEC / invalid-pitch paths
    f = g["fuzz"]
    fz = fuzz_frames(f["seed"], f["channels"], f["frames"])
    d2 = MelpeEngine(f["channels"])
    out = np.stack([d2.decode2400(np.ascontiguousarray(fz[:, k])) for k in range(f["frames"])], 1)
    for c in range(f["channels"]):
        assert sha(out[c]) == f["pcm_sha256"][c], "fuzz PCM, channel %d" % c


@pytest.mark.gpu
def test_r2400_dropin_melpe_i2_al_s():
    """melpe_i2 + melpe_al per 180 samples + melpe_s per 7 bytes (the
    single-stream drop-in at 2400 bps) reproduce golden channel 0; the
    encoder and decoder share one process-global instance, as in the
    reference, so encode runs first over the whole stream (as the
    reference's separate encoder process would) after a fresh reset"""
    from pairphone_amd import Melpe
    g = golden()
    x = inputs(g["seed"], 1, g["frames"])[0]
    m = Melpe()
    m.reset_process_state()
    m.lib.melpe_i2()
    bits = np.zeros((g["frames"], 7), np.uint8)
    npp = np.zeros((g["frames"], 180), np.int16)
    for k in range(g["frames"]):
        sp = np.ascontiguousarray(x[k])
        b = np.zeros(11, np.uint8)
        m.lib.melpe_al(b.ctypes.data_as(ctypes.c_void_p), sp.ctypes.data_as(ctypes.c_void_p))
        bits[k] = b[:7]
        npp[k] = sp
    assert bits.tobytes().hex() == g["bits_hex"][0]
    assert sha(npp) == g["npp_sha256"][0]
    m.reset_process_state()
    m.lib.melpe_i2()
    pcm = np.zeros((g["frames"], 180), np.int16)
    for k in range(g["frames"]):
        b = np.zeros(11, np.uint8)
        b[:7] = bits[k]
        out = np.zeros(540, np.int16)
        m.lib.melpe_s(out.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p))
        pcm[k] = out[:180]
        assert not out[180:].any()
    assert sha(pcm) == g["pcm_sha256"][0]
    m.reset_process_state()


@pytest.mark.gpu
def test_r2400_65536_channels_match_reference(tmp_path):
    """65,536 channels x 24 frames on one GPU (device buffers), 16 channels
    sampled across the range against the live reference"""
    import torch
    from pairphone_amd import MelpeEngine
    C, nfr, seed = 65536, 24, 2026
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    eng = MelpeEngine(C)
    eng.synth_seed(seed)
    pcm = torch.empty((nfr, C, 180), dtype=torch.int16, device=dev)
    for k in range(nfr):
        eng.synth_dev(pcm[k].data_ptr(), 180, s)
    bits = torch.zeros((nfr, C, 7), dtype=torch.uint8, device=dev)
    out = torch.zeros((nfr, C, 180), dtype=torch.int16, device=dev)
    for k in range(nfr):
        assert eng.lib.melpe_encode2400_dev(eng.h, bits[k].data_ptr(), pcm[k].data_ptr(), None,
                                            s) == 0
    for k in range(nfr):
        assert eng.lib.melpe_decode2400_dev(eng.h, out[k].data_ptr(), bits[k].data_ptr(), None,
                                            s) == 0
    torch.cuda.synchronize(dev)
    chans = sorted(set([0, C - 1] + [int(c) for c in np.linspace(1, C - 2, 14)]))
    b = bits[:, chans].cpu().numpy()
    o = out[:, chans].cpu().numpy()
    eng.close()
    for i, c in enumerate(chans):
        bf, pf = str(tmp_path / ("b%d" % c)), str(tmp_path / ("p%d" % c))
        subprocess.run([REF_TOOL, "enc24gen", str(seed), str(c), "1", str(nfr), bf], check=True)
        subprocess.run([REF_TOOL, "dec24gen", bf, "1", str(nfr), pf], check=True)
        np.testing.assert_array_equal(b[:, i], np.fromfile(bf, np.uint8).reshape(nfr, 7),
                                      err_msg="bits, channel %d" % c)
        np.testing.assert_array_equal(o[:, i], np.fromfile(pf, np.int16).reshape(nfr, 180),
                                      err_msg="pcm, channel %d" % c)
