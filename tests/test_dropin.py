"""Drop-in boundary, proven by linking: the reference's own callers of
melpe.h -- melpe/encoder.c, melpe/decoder.c (the standalone harnesses) and
melpe_dec.c (the VAD-framed decoder) -- compiled unchanged from
/root/reference and linked against libmelpe_amd.so instead of the
reference's libmelpe.a (pairphone_amd/build.py build_dropin, INTEGRATION.md
§1).  On the GPU box they must reproduce the reference's goldens (BASELINE
config 1: one channel, 10 s).

Also the melpe_n buffer contract (melpe/npp.c:176-193): only the first npp
call of a RATE1200 process reads 256 samples; every other call reads 180, so
a caller may hand a 180-sample buffer that ends at an unmapped page.
"""
import ctypes
import hashlib
import json
import mmap
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, GOLDEN

DROPIN = os.path.join(ROOT, "build", "dropin")
BINS = {"encoder": ("melpe_i", "melpe_a"), "decoder": ("melpe_i", "melpe_s"),
        "melpe_dec": ("melpe_i", "melpe_s")}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_dropin_binaries_link_the_engine():
    """no GPU: the relinked reference callers exist and resolve melpe_* from
    libmelpe_amd.so (not from a reference archive)"""
    for b, fns in BINS.items():
        p = os.path.join(DROPIN, b)
        assert os.path.exists(p), "run __graft_entry__.build() where /root/reference exists"
        ldd = subprocess.run(["ldd", p], capture_output=True, text=True).stdout
        assert "libmelpe_amd.so" in ldd, ldd
        syms = subprocess.run(["nm", p], capture_output=True, text=True).stdout
        for f in fns:
            assert ("U " + f) in syms, "%s must be imported, not defined, in %s" % (f, b)


@pytest.mark.gpu
def test_reference_encoder_decoder_relinked(tmp_path):
    from pairphone_amd import synth_signal
    ge = json.load(open(os.path.join(GOLDEN, "enc_1024.json")))
    gd = json.load(open(os.path.join(GOLDEN, "dec_1024.json")))
    nsf = ge["superframes"]
    for c in (0, 3):
        raw = tmp_path / ("in%d.raw" % c)
        synth_signal(ge["seed"], c, nsf * 540).tofile(str(raw))
        bits, pcm = tmp_path / ("b%d.bits" % c), tmp_path / ("p%d.raw" % c)
        subprocess.run([os.path.join(DROPIN, "encoder"), str(raw), str(bits)], check=True,
                       timeout=120)
        b = bits.read_bytes()
        assert len(b) == nsf * 11
        assert b.hex() == ge["bits_hex"][c], "bitstream of the relinked encoder, channel %d" % c
        assert sha(b) == ge["bits_sha256"][c]
        subprocess.run([os.path.join(DROPIN, "decoder"), str(bits), str(pcm)], check=True,
                       timeout=120)
        p = pcm.read_bytes()
        assert len(p) == nsf * 540 * 2
        assert sha(p) == gd["pcm_sha256"][c], "PCM of the relinked decoder, channel %d" % c


@pytest.mark.gpu
def test_reference_melpe_dec_relinked_matches_reference(tmp_path):
    """the VAD-framed stream decoder of the reference, relinked, gives the
    PCM of the reference's own build (oracle/_ref/melpe_dec)"""
    from pairphone_amd import stream_pack
    ge = json.load(open(os.path.join(GOLDEN, "enc_1024.json")))
    bits = np.frombuffer(bytes.fromhex(ge["bits_hex"][1]), np.uint8).reshape(-1, 11)
    votes = np.ones(bits.shape[0], np.uint8)
    votes[5:9] = 0
    votes[40:41] = 0
    votes[100:130] = 0
    f = tmp_path / "s.mlp"
    f.write_bytes(stream_pack(bits, votes))
    outs = []
    for exe in (os.path.join(DROPIN, "melpe_dec"), os.path.join(ROOT, "oracle", "_ref", "melpe_dec")):
        o = tmp_path / (os.path.basename(os.path.dirname(exe)) + ".raw")
        subprocess.run([exe, str(f), str(o)], check=True, timeout=120, capture_output=True)
        outs.append(o.read_bytes())
    assert len(outs[0]) == bits.shape[0] * 540 * 2
    assert outs[0] == outs[1]


def _guarded_buffer(nsamples):
    """an int16 view of `nsamples` that ends exactly at a PROT_NONE page"""
    page = mmap.PAGESIZE
    m = mmap.mmap(-1, 2 * page, prot=mmap.PROT_READ | mmap.PROT_WRITE)
    libc = ctypes.CDLL(None)
    base = ctypes.addressof(ctypes.c_char.from_buffer(m))
    assert libc.mprotect(ctypes.c_void_p(base + page), ctypes.c_size_t(page), 0) == 0
    off = page - 2 * nsamples
    return m, np.frombuffer(m, dtype=np.int16, count=nsamples, offset=off)


@pytest.mark.gpu
def test_melpe_n_reads_180_after_first_call():
    """the first call of a fresh RATE1200 process gets 256 samples; every
    later call a 180-sample buffer against a guard page (an over-read would
    fault); the outputs equal the golden NPP stream of that channel"""
    from pairphone_amd import Melpe, synth_signal
    g = json.load(open(os.path.join(GOLDEN, "npp.json")))
    m = Melpe()
    m.reset_process_state()
    m.melpe_i()
    x = synth_signal(g["seed"], 0, g["frames"] * 180 + 76)
    out = np.zeros(g["frames"] * 180, np.int16)
    first = np.ascontiguousarray(x[:256])
    m.lib.melpe_n(first.ctypes.data_as(ctypes.c_void_p))
    out[:180] = first[:180]
    mm, buf = _guarded_buffer(180)
    for k in range(1, g["frames"]):
        buf[:] = x[k * 180:(k + 1) * 180]
        m.lib.melpe_n(buf.ctypes.data_as(ctypes.c_void_p))
        out[k * 180:(k + 1) * 180] = buf
    del buf
    mm.close()
    assert sha(out.tobytes()) == g["sha256"][0]
    m.reset_process_state()
