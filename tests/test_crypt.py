"""Voice-frame crypt parity against the reference.

VoiceEnc / VoiceDec (crp.c:986-1027): each 81-bit packet XORed with the
Keccak sponge keystream of (counter, 16-byte key).  Oracle = the reference's
own crypto/sponge.c compiled into oracle/_ref/libref_crypt.so (harness
oracle/ref_crypt.c); golden fixture tests/golden/voice_crypt.json made from
it by tests/golden/make_crypt_golden.py (64 channels x 8 packets, counter
wrap-around, zero / 0xFF keys, polarity inversion).

CPU: the oracle and the host build of voice_crypt.h against the golden;
argument errors of the C ABI (rejected before any HIP call).
GPU: the HIP kernel through the C ABI against the golden, against the live
oracle at BASELINE config 4's 262,144 channels, and the enc -> dec round trip.
"""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, GOLDEN

sys.path.insert(0, GOLDEN)
from make_crypt_golden import inputs, ref_crypt, LIB as REF_LIB  # noqa: E402

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
P = ctypes.c_void_p


def golden():
    g = json.load(open(os.path.join(GOLDEN, "voice_crypt.json")))
    shape = (g["channels"], g["packets"], 11)
    enc = np.frombuffer(bytes.fromhex(g["enc_hex"]), np.uint8).reshape(shape)
    dec = np.frombuffer(bytes.fromhex(g["dec_invert_hex"]), np.uint8).reshape(shape)
    return g, enc, dec


def emu_crypt(pkts, ctr, keys, inv, direction):
    lib = ctypes.CDLL(EMU)
    out = pkts.copy()
    assert lib.emu_voice_crypt(P(out.ctypes.data), P(ctr.ctypes.data), P(keys.ctypes.data),
                               None if inv is None else P(inv.ctypes.data),
                               out.shape[0], out.shape[1], direction) == 0
    return out


def test_oracle_matches_golden():
    g, enc, dec = golden()
    pkts, ctr, keys, inv = inputs(g["seed"], g["channels"], g["packets"])
    assert np.array_equal(ref_crypt(pkts, ctr, keys, None, 0), enc)
    assert np.array_equal(ref_crypt(pkts, ctr, keys, inv, 1), dec)


def test_hostemu_matches_golden():
    g, enc, dec = golden()
    pkts, ctr, keys, inv = inputs(g["seed"], g["channels"], g["packets"])
    assert np.array_equal(emu_crypt(pkts, ctr, keys, None, 0), enc)
    assert np.array_equal(emu_crypt(pkts, ctr, keys, inv, 1), dec)
    # only the 81 packet bits change: byte 10's upper bits stay zero
    assert not (enc[..., 10] & 0xFE).any()


def test_abi_rejects_bad_arguments(engine_lib):
    lib = engine_lib
    # misaligned key pointer, zero channels, bad direction: refused before any HIP call
    assert lib.melpe_voice_crypt_dev(P(4096), P(4096), P(4097), None, 1, 1, 0, None) < 0
    assert b"aligned" in lib.melpe_last_error()
    assert lib.melpe_voice_crypt_dev(P(4096), P(4096), P(4096), None, 0, 1, 0, None) < 0
    assert lib.melpe_voice_crypt_dev(P(4096), P(4096), P(4096), None, 1, 1, 2, None) < 0


@pytest.mark.gpu
def test_gpu_matches_golden():
    from pairphone_amd import VoiceEnc, VoiceDec
    g, enc, dec = golden()
    pkts, ctr, keys, inv = inputs(g["seed"], g["channels"], g["packets"])
    assert np.array_equal(VoiceEnc(pkts, ctr, keys), enc)
    assert np.array_equal(VoiceDec(pkts, ctr, keys, inv), dec)


@pytest.mark.gpu
def test_gpu_262144_channels_match_reference_and_round_trip():
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    C, K = 262144, 2
    pkts, ctr, keys, inv = inputs(7, C, K)
    want = ref_crypt(pkts, ctr, keys, None, 0)
    dev = torch.device("cuda:0")
    d_p = torch.from_numpy(pkts.copy()).to(dev)
    d_c = torch.from_numpy(ctr.view(np.int32)).to(dev)
    d_k = torch.from_numpy(keys).to(dev)
    d_i = torch.from_numpy(inv).to(dev)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.melpe_voice_crypt_dev(d_p.data_ptr(), d_c.data_ptr(), d_k.data_ptr(), None,
                                     C, K, 0, s) == 0
    got = d_p.cpu().numpy()
    assert np.array_equal(got, want)
    # decrypting with the same counter and key restores the packets
    assert lib.melpe_voice_crypt_dev(d_p.data_ptr(), d_c.data_ptr(), d_k.data_ptr(), None,
                                     C, K, 1, s) == 0
    assert np.array_equal(d_p.cpu().numpy(), pkts)
    # a polarity-inverted channel carries the complement; invert=1 undoes it
    flip = want.copy()
    flip[..., :10] ^= 0xFF
    flip[..., 10] ^= 1
    d_p.copy_(torch.from_numpy(np.where(inv[:, None, None] != 0, flip, want)))
    assert lib.melpe_voice_crypt_dev(d_p.data_ptr(), d_c.data_ptr(), d_k.data_ptr(),
                                     d_i.data_ptr(), C, K, 1, s) == 0
    assert np.array_equal(d_p.cpu().numpy(), pkts)
    assert os.path.exists(REF_LIB)
