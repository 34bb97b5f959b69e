"""PairPhone's pseudo-voice BPSK modem: Modulate
(modem/modem.c:136, TX after the voice-frame crypt, tx.c:271) and Demodulate
(:186, RX before it, rx.c:294-297), batched per channel (csrc/modem.h).

Oracle: the reference's own modem/modem.c compiled by oracle/Makefile into
oracle/_ref/ref_modem, one process per channel (its state is file
statics).  CPU tests check the host build of modem.h against it; GPU tests
the HIP kernels (melpe_modulate_dev / melpe_demodulate_dev).

Channels for the demodulator: a modulated packet stream behind a random
lead-in, then impaired as a GSM-tandem-like path would: clean, gain + noise,
inverted polarity, sampling-rate drift (a sample dropped or repeated every
few hundred), no carrier (noise only), silence, clipping.  Every call's
12 output bytes (payload, lag, BER and lock flags) and its consumed-sample
count must equal the reference's.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, REF_DIR

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
REF_MODEM = os.path.join(REF_DIR, "ref_modem")
PKT = 3240
LOOKAHEAD = 1080


def packets(seed, C, K):
    b = np.random.default_rng(seed).integers(0, 256, (C, K, 11)).astype(np.uint8)
    b[:, :, 10] &= 1          # 81 bits: byte 10 carries bit 80 only (crp.c:997)
    return b


def emu():
    lib = ctypes.CDLL(EMU)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    lib.emu_modem_reset.argtypes = [vp, i32]
    lib.emu_modulate.argtypes = [vp, vp, vp, i32, i32]
    lib.emu_demodulate.argtypes = [vp, vp, ctypes.c_long, vp, vp, vp, vp, i32, i32]
    return lib


def p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def impair(x, kind, seed):
    """deterministic channel impairments of one int16 stream"""
    g = np.random.default_rng(seed)
    lead = int(g.integers(0, 3 * PKT))
    x = np.concatenate([(g.normal(0, 60, lead)).astype(np.int64), x.astype(np.int64)])
    if kind == "noise_gain":
        x = (0.6 * x + g.normal(0, 1500, len(x))).astype(np.int64)
    elif kind == "inverted":
        x = -x
    elif kind == "drift_fast":
        keep = np.ones(len(x), bool)
        keep[::397] = False
        x = x[keep]
    elif kind == "drift_slow":
        x = np.repeat(x, np.where(np.arange(len(x)) % 251 == 0, 2, 1))
    elif kind == "no_carrier":
        x = g.normal(0, 4000, len(x)).astype(np.int64)
    elif kind == "silence":
        x = np.zeros(len(x), np.int64)
    elif kind == "clipped":
        x = 3 * x
    return np.clip(x, -32768, 32767).astype(np.int16)


KINDS = ["clean", "noise_gain", "inverted", "drift_fast", "drift_slow", "no_carrier",
         "silence", "clipped"]


def ref_modulate(tmp, bits):
    out = []
    for c in range(bits.shape[0]):
        bf, pf = str(tmp / ("m%d.bits" % c)), str(tmp / ("m%d.pcm" % c))
        bits[c].tofile(bf)
        subprocess.run([REF_MODEM, "mod", bf, pf], check=True)
        out.append(np.fromfile(pf, np.int16))
    return np.stack(out)


def ref_demodulate(tmp, streams, calls):
    data, rets = [], []
    for c, x in enumerate(streams):
        xf, of = str(tmp / ("d%d.pcm" % c)), str(tmp / ("d%d.out" % c))
        x.tofile(xf)
        subprocess.run([REF_MODEM, "demod", xf, str(calls), of], check=True)
        r = np.fromfile(of, np.uint8).reshape(calls, 16)
        data.append(r[:, :12])
        rets.append(r[:, 12:].copy().view(np.int32)[:, 0])
    return np.stack(data), np.stack(rets)


def streams_for(bits):
    """modulated packet streams of every channel, impaired by channel kind,
    padded to one length; returns (C x L int16, calls)"""
    lib = emu()
    C, K = bits.shape[:2]
    st = np.zeros(C * lib.emu_modem_state_bytes(), np.uint8)
    lib.emu_modem_reset(p(st), C)
    pcm = np.zeros((C, K * PKT), np.int16)
    lib.emu_modulate(p(st), p(np.ascontiguousarray(bits)), p(pcm), C, K)
    xs = [impair(pcm[c], KINDS[c % len(KINDS)], 100 + c) for c in range(C)]
    L = max(len(x) for x in xs) + LOOKAHEAD
    out = np.zeros((C, L), np.int16)
    for c, x in enumerate(xs):
        out[c, :len(x)] = x
    calls = (min(len(x) for x in xs) - LOOKAHEAD) // 226
    return out, calls


def test_modulate_hostemu_matches_reference(tmp_path, ref_tool):
    bits = packets(7, 6, 24)
    lib = emu()
    st = np.zeros(6 * lib.emu_modem_state_bytes(), np.uint8)
    lib.emu_modem_reset(p(st), 6)
    got = np.zeros((6, 24 * PKT), np.int16)
    lib.emu_modulate(p(st), p(bits), p(got), 6, 24)
    np.testing.assert_array_equal(got, ref_modulate(tmp_path, bits))


def test_demodulate_hostemu_matches_reference(tmp_path, ref_tool):
    bits = packets(8, len(KINDS), 30)
    x, calls = streams_for(bits)
    want_d, want_r = ref_demodulate(tmp_path, list(x), calls)
    lib = emu()
    C = x.shape[0]
    st = np.zeros(C * lib.emu_modem_state_bytes(), np.uint8)
    lib.emu_modem_reset(p(st), C)
    pos = np.zeros(C, np.int32)
    data = np.zeros((C, 12), np.uint8)
    out = np.zeros((C, calls, 12), np.uint8)
    ret = np.zeros((C, calls), np.int32)
    lib.emu_demodulate(p(st), p(x), x.shape[1], p(pos), p(data), p(out), p(ret), C, calls)
    for c in range(C):
        np.testing.assert_array_equal(ret[c], want_r[c], err_msg="returns, %s" % KINDS[c])
        np.testing.assert_array_equal(out[c], want_d[c], err_msg="data, %s" % KINDS[c])
    # the clean channel synchronises and then delivers the packets sent
    # (received in inverted polarity here, which the crypto layer undoes)
    ok = np.nonzero((out[0, :, 11] & 0xC0) == 0xC0)[0]
    assert len(ok) > 10
    got = out[0, ok, :11].copy()
    got[:, 10] &= 1
    inv = bits[0] ^ np.uint8(0xFF)
    inv[:, 10] &= 1
    k0 = next(k for k in range(bits.shape[1]) if (inv[k] == got[0]).all())
    np.testing.assert_array_equal(got, inv[k0:k0 + len(ok)])


def _dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.gpu
def test_modem_gpu_matches_reference(tmp_path, ref_tool):
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    C, K = len(KINDS) * 2, 30
    bits = packets(9, C, K)
    sb = lib.melpe_modem_state_bytes()
    st = torch.zeros(C * sb, dtype=torch.uint8, device=dev)
    assert lib.melpe_modem_reset_dev(st.data_ptr(), C, None, s) == 0
    db = _dev(bits, dev)
    pcm = torch.zeros((C, K, PKT), dtype=torch.int16, device=dev)
    # two launches (packets 0..9, 10..29): the modulator state carries over
    for k0, k1 in ((0, 10), (10, K)):
        sub_b = db[:, k0:k1].contiguous()
        sub_p = torch.zeros((C, k1 - k0, PKT), dtype=torch.int16, device=dev)
        assert lib.melpe_modulate_dev(st.data_ptr(), sub_b.data_ptr(), sub_p.data_ptr(), C,
                                      k1 - k0, None, s) == 0, lib.melpe_last_error()
        pcm[:, k0:k1] = sub_p
    got = pcm.cpu().numpy().reshape(C, K * PKT)
    np.testing.assert_array_equal(got[:4], ref_modulate(tmp_path, bits[:4]))
    x, calls = streams_for(bits)
    want_d, want_r = ref_demodulate(tmp_path, list(x), calls)
    assert lib.melpe_modem_reset_dev(st.data_ptr(), C, None, s) == 0
    dx = _dev(x, dev)
    pos = torch.zeros(C, dtype=torch.int32, device=dev)
    data = torch.zeros((C, 12), dtype=torch.uint8, device=dev)
    out = torch.zeros((C, calls, 12), dtype=torch.uint8, device=dev)
    ret = torch.zeros((C, calls), dtype=torch.int32, device=dev)
    # in two launches of calls, as a receiver would run it
    h = calls // 2
    for a, n in ((0, h), (h, calls - h)):
        o = torch.zeros((C, n, 12), dtype=torch.uint8, device=dev)
        r = torch.zeros((C, n), dtype=torch.int32, device=dev)
        assert lib.melpe_demodulate_dev(st.data_ptr(), dx.data_ptr(), x.shape[1], pos.data_ptr(),
                                        data.data_ptr(), o.data_ptr(), r.data_ptr(), C, n,
                                        None, s) == 0, lib.melpe_last_error()
        out[:, a:a + n] = o
        ret[:, a:a + n] = r
    o, r = out.cpu().numpy(), ret.cpu().numpy()
    for c in range(C):
        np.testing.assert_array_equal(r[c], want_r[c], err_msg="returns, ch %d" % c)
        np.testing.assert_array_equal(o[c], want_d[c], err_msg="data, ch %d" % c)


@pytest.mark.gpu
def test_modem_round_trip_65536_channels():
    """size-independent property at scale: after synchronisation every
    clean channel's demodulator delivers exactly the packets its modulator
    sent, in order (rx.c reads a packet when buf[11] has the ready 0x80 and
    block-lock 0x40 flags)"""
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    C, K = 65536, 12
    g = torch.Generator(device="cpu").manual_seed(11)
    bits = torch.randint(0, 256, (C, K, 11), dtype=torch.uint8, generator=g)
    bits[:, :, 10] &= 1
    db = bits.to(dev)
    sb = lib.melpe_modem_state_bytes()
    st = torch.zeros(C * sb, dtype=torch.uint8, device=dev)
    assert lib.melpe_modem_reset_dev(st.data_ptr(), C, None, s) == 0
    L = K * PKT + LOOKAHEAD + 512
    pcm = torch.zeros((C, L), dtype=torch.int16, device=dev)
    tmp = torch.zeros((C, K, PKT), dtype=torch.int16, device=dev)
    assert lib.melpe_modulate_dev(st.data_ptr(), db.data_ptr(), tmp.data_ptr(), C, K, None, s) == 0
    pcm[:, :K * PKT] = tmp.view(C, K * PKT)
    del tmp
    calls = (K * PKT) // 216 - 8
    pos = torch.zeros(C, dtype=torch.int32, device=dev)
    data = torch.zeros((C, 12), dtype=torch.uint8, device=dev)
    out = torch.zeros((C, calls, 12), dtype=torch.uint8, device=dev)
    ret = torch.zeros((C, calls), dtype=torch.int32, device=dev)
    assert lib.melpe_demodulate_dev(st.data_ptr(), pcm.data_ptr(), L, pos.data_ptr(), data.data_ptr(),
                                    out.data_ptr(), ret.data_ptr(), C, calls, None, s) == 0
    torch.cuda.synchronize(dev)
    o = out.cpu()
    ok = ((o[:, :, 11] & 0xC0) == 0xC0)
    assert bool((ret.cpu() > 0).all())
    # every channel synchronises within a few packets; the packets it
    # delivers from then on are consecutive packets of the sent stream, in
    # one polarity (BPSK is received inverted or not; PairPhone's crypto
    # layer resolves it with its polarity flag, crp.c:1011-1015)
    sent = bits.view(C, K, 11)
    inv = sent ^ 0xFF
    inv[:, :, 10] &= 1
    for c in (0, 1, 4097, 30000, C - 1):
        idx = torch.nonzero(ok[c]).flatten()
        assert len(idx) >= K - 6, "channel %d delivered %d packets" % (c, len(idx))
        got = o[c, idx, :11].clone()
        got[:, 10] &= 1
        n = len(idx)
        hit = None
        for ref in (sent[c], inv[c]):
            for k in range(n - 1, K):
                if torch.equal(ref[k], got[-1]):
                    hit = torch.equal(got, ref[k - n + 1:k + 1])
        assert hit, "channel %d: delivered packets are not the sent sequence" % c
