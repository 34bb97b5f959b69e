"""melpe_s (decode) parity against the reference codec.

Goldens (tests/golden/make_golden.py, reference compiled by oracle/Makefile):
  dec_1024.json  SHA-256 of the PCM the reference decodes from the enc_1024
                 bitstreams (1024 channels x 149 superframes, synth seed 1)
  dec_fuzz.json  SHA-256 of the PCM decoded from uniformly random
                 bitstreams (256 channels x 200 superframes, PCG64 seed 77):
                 every parity / FEC / erasure branch of low_rate_chn_read
CPU: the host build of the device sources on a few channels, and the
single-stream melp_par / quant_par sharing against the reference's `duplex`.
GPU: the HIP engine on all channels, ragged masks, the drop-in API.
"""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, GOLDEN, REF_TOOL
from test_encode import emu, signals, run_superframes, golden as enc_golden

FUZZ_SEED = 77


def gold(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def sha(b):
    return hashlib.sha256(b.tobytes()).hexdigest()


def fuzz_bits(seed, channels, nsf):
    """same generator as tests/golden/make_golden.py:fuzz_bits"""
    return np.random.Generator(np.random.PCG64(seed)).integers(
        0, 256, (channels, nsf * 11), dtype=np.uint8)


def decode_all(decode, bits, nsf):
    C = bits.shape[0]
    pcm = np.zeros((C, nsf * 540), np.int16)
    for k in range(nsf):
        pcm[:, k * 540:(k + 1) * 540] = decode(np.ascontiguousarray(bits[:, k * 11:(k + 1) * 11]))
    return pcm


def emu_decoder(ch, fn="emu_decode"):
    lib = emu()
    f = getattr(lib, fn)
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    e = lib.emu_create(ch)

    def dec(b):
        sp = np.zeros((ch, 540), np.int16)
        f(e, sp.ctypes.data, b.ctypes.data)
        return sp
    return lib, e, dec


def test_decode_hostemu_matches_golden():
    g, ge = gold("dec_1024.json"), enc_golden()
    ch, nsf = 4, g["superframes"]
    bits = np.stack([np.frombuffer(bytes.fromhex(ge["bits_hex"][c]), np.uint8) for c in range(ch)])
    lib, e, dec = emu_decoder(ch)
    pcm = decode_all(dec, bits, nsf)
    lib.emu_destroy(e)
    for c in range(ch):
        assert sha(pcm[c]) == g["pcm_sha256"][c], "channel %d" % c


def test_decode_hostemu_random_bitstreams_match_golden():
    g = gold("dec_fuzz.json")
    ch, nsf = 8, g["superframes"]
    bits = fuzz_bits(g["seed"], g["channels"], nsf)[:ch]
    lib, e, dec = emu_decoder(ch)
    pcm = decode_all(dec, bits, nsf)
    lib.emu_destroy(e)
    assert pcm[0, :540].tolist() == g["pcm0_first_sf"]
    for c in range(ch):
        assert sha(pcm[c]) == g["pcm_sha256"][c], "channel %d" % c


def test_decode2_hostemu_matches_goldens():
    """The two-wave decoder's phase program (decoder.h dec2_phase: wave A the
    channel read and the excitation, wave B the filters, dispersion and
    postfilter one frame behind, each on its own copy of the record, the
    hand-over buffers pattern-filled) against the decode goldens and the
    random-bitstream fuzz set."""
    g, ge = gold("dec_1024.json"), enc_golden()
    ch, nsf = 4, g["superframes"]
    bits = np.stack([np.frombuffer(bytes.fromhex(ge["bits_hex"][c]), np.uint8) for c in range(ch)])
    lib, e, dec = emu_decoder(ch, "emu_decode2")
    pcm = decode_all(dec, bits, nsf)
    lib.emu_destroy(e)
    for c in range(ch):
        assert sha(pcm[c]) == g["pcm_sha256"][c], "channel %d" % c
    g = gold("dec_fuzz.json")
    ch, nsf = 8, g["superframes"]
    bits = fuzz_bits(g["seed"], g["channels"], nsf)[:ch]
    lib, e, dec = emu_decoder(ch, "emu_decode2")
    pcm = decode_all(dec, bits, nsf)
    lib.emu_destroy(e)
    for c in range(ch):
        assert sha(pcm[c]) == g["pcm_sha256"][c], "fuzz channel %d" % c


def test_duplex_sharing_hostemu_matches_reference(tmp_path, ref_tool):
    """melpe_a and melpe_s interleaved in one process share melp_par /
    quant_par / chbuf in the reference; the engine's hand-over (k_share_params)
    must reproduce that, including for corrupted received bits."""
    nsf = 60
    x = signals(4, 1, nsf)[0]
    rx = fuzz_bits(5, 1, nsf)[0]
    rx[: 30 * 11] = np.frombuffer(bytes.fromhex(enc_golden()["bits_hex"][1]), np.uint8)[: 30 * 11]
    x.tofile(str(tmp_path / "x.pcm"))
    rx.tofile(str(tmp_path / "rx.bits"))
    subprocess.run([ref_tool, "duplex", str(tmp_path / "x.pcm"), str(tmp_path / "rx.bits"),
                    str(tmp_path / "tx.bits"), str(tmp_path / "y.pcm")], check=True)
    want_tx = np.fromfile(str(tmp_path / "tx.bits"), np.uint8)
    want_y = np.fromfile(str(tmp_path / "y.pcm"), np.int16)
    lib = emu()
    lib.emu_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_share.argtypes = [ctypes.c_void_p, ctypes.c_int]
    e = lib.emu_create(1)
    tx, y = [], []
    for k in range(nsf):
        sp = x[k * 540:(k + 1) * 540].copy()
        b = np.zeros(11, np.uint8)
        lib.emu_encode(e, b.ctypes.data, sp.ctypes.data)
        tx.append(b)
        lib.emu_share(e, 0)
        out = np.zeros(540, np.int16)
        r = rx[k * 11:(k + 1) * 11].copy()
        lib.emu_decode(e, out.ctypes.data, r.ctypes.data)
        lib.emu_share(e, 1)
        y.append(out)
    lib.emu_destroy(e)
    np.testing.assert_array_equal(np.concatenate(tx), want_tx)
    np.testing.assert_array_equal(np.concatenate(y), want_y)


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [1, 2])
def test_decode_gpu_mappings_match_golden_and_fuzz(waves):
    """Both decoder mappings forced on every superframe: one lane per
    channel (k_decode, the 262,144-channel headline's) and the two-wave
    decoder (k_decode2, the default up to 65,536 channels), against the
    1,024-channel goldens and the random-bitstream fuzz set."""
    from pairphone_amd import MelpeEngine
    g, ge = gold("dec_1024.json"), enc_golden()
    C, nsf = g["channels"], g["superframes"]
    eng = MelpeEngine(C)
    eng.set_dec_waves(waves)
    x = signals(g["seed"], C, nsf)
    enc = MelpeEngine(C)
    bits, _ = run_superframes(enc.encode, x, nsf)
    enc.close()
    assert [c for c in range(C) if sha(bits[c]) != ge["bits_sha256"][c]] == []
    pcm = decode_all(eng.decode, bits, nsf)
    eng.close()
    bad = [c for c in range(C) if sha(pcm[c]) != g["pcm_sha256"][c]]
    assert not bad, "decoder mismatch on %d channels, first %s" % (len(bad), bad[:8])
    gf = gold("dec_fuzz.json")
    fb = fuzz_bits(gf["seed"], gf["channels"], gf["superframes"])
    eng = MelpeEngine(gf["channels"])
    eng.set_dec_waves(waves)
    pcm = decode_all(eng.decode, fb, gf["superframes"])
    eng.close()
    bad = [c for c in range(gf["channels"]) if sha(pcm[c]) != gf["pcm_sha256"][c]]
    assert not bad, "fuzz mismatch on %d channels, first %s" % (len(bad), bad[:8])


@pytest.mark.gpu
def test_decode_gpu_1024_channels_match_golden():
    from pairphone_amd import MelpeEngine
    g, ge = gold("dec_1024.json"), enc_golden()
    C, nsf = g["channels"], g["superframes"]
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    bits, _ = run_superframes(eng.encode, x, nsf)
    bad = [c for c in range(C) if sha(bits[c]) != ge["bits_sha256"][c]]
    assert not bad, "encoder mismatch on %d channels, first %s" % (len(bad), bad[:8])
    pcm = decode_all(eng.decode, bits, nsf)
    bad = [c for c in range(C) if sha(pcm[c]) != g["pcm_sha256"][c]]
    assert not bad, "decoder mismatch on %d channels, first %s" % (len(bad), bad[:8])


@pytest.mark.gpu
def test_decode_gpu_random_bitstreams_match_golden():
    from pairphone_amd import MelpeEngine
    g = gold("dec_fuzz.json")
    C, nsf = g["channels"], g["superframes"]
    bits = fuzz_bits(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    pcm = decode_all(eng.decode, bits, nsf)
    bad = [c for c in range(C) if sha(pcm[c]) != g["pcm_sha256"][c]]
    assert not bad, "mismatch on %d channels, first %s" % (len(bad), bad[:8])


@pytest.mark.gpu
def test_decode_gpu_ragged_mask():
    """Inactive channels keep state and output untouched."""
    from pairphone_amd import MelpeEngine
    g = gold("dec_fuzz.json")
    C, nsf = 8, 40
    bits = fuzz_bits(g["seed"], g["channels"], g["superframes"])[:C]
    full = decode_all(MelpeEngine(C).decode, bits, nsf)
    rng = np.random.default_rng(11)
    act = rng.random((nsf + 20, C)) < 0.6
    eng = MelpeEngine(C)
    pos = np.zeros(C, int)
    out = [[] for _ in range(C)]
    for k in range(act.shape[0]):
        m = np.array([act[k, c] and pos[c] < nsf for c in range(C)], np.uint8)
        b = np.stack([bits[c, pos[c] * 11:(pos[c] + 1) * 11] if pos[c] < nsf else np.zeros(11, np.uint8)
                      for c in range(C)])
        sp = eng.decode(b, m)
        for c in range(C):
            if m[c]:
                out[c].append(sp[c].copy())
                pos[c] += 1
            else:
                assert (sp[c] == 0).all()
    for c in range(C):
        np.testing.assert_array_equal(np.concatenate(out[c]), full[c, :pos[c] * 540], err_msg="ch %d" % c)


@pytest.mark.gpu
def test_single_stream_duplex_matches_reference(tmp_path, ref_tool):
    """melpe_i, then melpe_a / melpe_s alternately through include/melpe.h,
    against the reference doing the same in one process."""
    from pairphone_amd import Melpe
    nsf = 40
    x = signals(6, 1, nsf)[0]
    rx = fuzz_bits(8, 1, nsf)[0]
    rx[: 20 * 11] = np.frombuffer(bytes.fromhex(enc_golden()["bits_hex"][2]), np.uint8)[: 20 * 11]
    x.tofile(str(tmp_path / "x.pcm"))
    rx.tofile(str(tmp_path / "rx.bits"))
    subprocess.run([ref_tool, "duplex", str(tmp_path / "x.pcm"), str(tmp_path / "rx.bits"),
                    str(tmp_path / "tx.bits"), str(tmp_path / "y.pcm")], check=True)
    m = Melpe()
    m.reset_process_state()   # a fresh reference process per test
    m.melpe_i()
    tx, y = [], []
    for k in range(nsf):
        tx.append(m.melpe_a(x[k * 540:(k + 1) * 540].copy()))
        y.append(m.melpe_s(rx[k * 11:(k + 1) * 11]))
    np.testing.assert_array_equal(np.concatenate(tx), np.fromfile(str(tmp_path / "tx.bits"), np.uint8))
    np.testing.assert_array_equal(np.concatenate(y), np.fromfile(str(tmp_path / "y.pcm"), np.int16))


@pytest.mark.gpu
def test_duplex_encoder_decoder_on_own_streams_match_goldens():
    """An encoder engine and a decoder engine, each on a stream (hardware
    queue) of its own (melpe_engine_set_own_stream), driven from two caller
    streams: superframe k is encoded on one while superframe k - 1's bits
    are decoded on the other, the decoder's stream waiting only for the
    bits it reads.  Both outputs match the 1,024-channel goldens (the
    encoder's bitstream and NPP output, the PCM the reference decodes
    from it); whether the two engines' kernels overlap is timed by
    bench.py --duplex."""
    import torch
    from pairphone_amd import MelpeEngine
    ge, gd = enc_golden(), gold("dec_1024.json")
    C, nsf = ge["channels"], ge["superframes"]
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(np.ascontiguousarray(
        signals(ge["seed"], C, nsf).reshape(C, nsf, 540).transpose(1, 0, 2))).to(dev)
    enc, dec = MelpeEngine(C), MelpeEngine(C)
    enc.set_own_stream(True)
    dec.set_own_stream(True)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sa.wait_stream(torch.cuda.current_stream(dev))
    bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
    pcm = torch.zeros((nsf, C, 540), dtype=torch.int16, device=dev)
    for k in range(nsf + 1):
        if k < nsf:
            enc.encode_dev(bits[k].data_ptr(), x[k].data_ptr(), None, sa.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(sa)
        if k > 0:
            dec.decode_dev(pcm[k - 1].data_ptr(), bits[k - 1].data_ptr(), None, sb.cuda_stream)
        if k < nsf:
            sb.wait_event(ev)
    torch.cuda.synchronize(dev)
    enc.close()
    dec.close()
    b = bits.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 11)
    n = x.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 540)
    p = pcm.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 540)
    assert [c for c in range(C) if sha(b[c]) != ge["bits_sha256"][c]] == []
    assert [c for c in range(C) if sha(n[c]) != ge["npp_sha256"][c]] == []
    assert [c for c in range(C) if sha(p[c]) != gd["pcm_sha256"][c]] == []


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [1, 2])
def test_duplex_pipe_dev_matches_goldens(waves):
    """melpe_duplex_pipe_dev on one engine: superframe k's analysis, k+1's
    NPP and the decode of superframe k-1's bits on three internal streams
    (the config-3 round trip as bench.py times it), both decoder mappings:
    the bits, the NPP output and the decoded PCM match the 1,024-channel
    goldens, as the same calls serialised do."""
    import torch
    from pairphone_amd import MelpeEngine
    ge, gd = enc_golden(), gold("dec_1024.json")
    C, nsf = ge["channels"], ge["superframes"]
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    x = torch.from_numpy(np.ascontiguousarray(
        signals(ge["seed"], C, nsf).reshape(C, nsf, 540).transpose(1, 0, 2))).to(dev)
    bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
    pcm = torch.zeros((nsf, C, 540), dtype=torch.int16, device=dev)
    eng = MelpeEngine(C)
    eng.set_dec_waves(waves)
    eng.encode_npp_dev(x[0].data_ptr(), None, s)
    for k in range(nsf):
        eng.duplex_pipe_dev(bits[k].data_ptr(), x[k].data_ptr(),
                            x[k + 1].data_ptr() if k + 1 < nsf else None,
                            pcm[k - 1].data_ptr() if k > 0 else None,
                            bits[k - 1].data_ptr() if k > 0 else None, stream=s)
    eng.decode_dev(pcm[nsf - 1].data_ptr(), bits[nsf - 1].data_ptr(), None, s)
    torch.cuda.synchronize(dev)
    eng.close()
    b = bits.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 11)
    n = x.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 540)
    p = pcm.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 540)
    assert [c for c in range(C) if sha(b[c]) != ge["bits_sha256"][c]] == []
    assert [c for c in range(C) if sha(n[c]) != ge["npp_sha256"][c]] == []
    assert [c for c in range(C) if sha(p[c]) != gd["pcm_sha256"][c]] == []
