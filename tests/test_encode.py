"""melpe_a (encode) parity against the reference codec.

Goldens (tests/golden/enc_1024.json, made by tests/golden/make_golden.py from
the reference compiled by oracle/Makefile): SHA-256 of each channel's
bitstream and of the NPP output melpe_a leaves in the caller's buffer, for
1024 channels x 149 superframes (10 s) of the csrc/synth.h signal, seed 1.

CPU: the host build of the device sources on a few channels.
GPU: the HIP engine on all 1024 channels (BASELINE config 2), edge signals
against the live reference, ragged activity masks and the drop-in
single-stream API.
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

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
TABLES = os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin")


def golden():
    return json.load(open(os.path.join(GOLDEN, "enc_1024.json")))


def sha(b):
    return hashlib.sha256(b.tobytes()).hexdigest()


def signals(seed, channels, nsf, first=0):
    from pairphone_amd import synth_signal
    return np.stack([synth_signal(seed, first + c, nsf * 540) for c in range(channels)])


def emu():
    lib = ctypes.CDLL(EMU)
    lib.emu_create.restype = ctypes.c_void_p
    lib.emu_create.argtypes = [ctypes.c_int]
    lib.emu_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_destroy.argtypes = [ctypes.c_void_p]
    assert lib.emu_load_tables(TABLES.encode()) == 0
    return lib


def run_superframes(encode, x, nsf):
    """x: [C, nsf*540] -> (bits [C, nsf*11], npp [C, nsf*540])"""
    C = x.shape[0]
    bits = np.zeros((C, nsf * 11), np.uint8)
    npp = np.zeros((C, nsf * 540), np.int16)
    for k in range(nsf):
        sp = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        b = encode(sp)
        bits[:, k * 11:(k + 1) * 11] = b
        npp[:, k * 540:(k + 1) * 540] = sp
    return bits, npp


def emu_encode_all(x, nsf):
    lib = emu()
    e = lib.emu_create(x.shape[0])

    def enc(sp):
        b = np.zeros((x.shape[0], 11), np.uint8)
        lib.emu_encode(e, b.ctypes.data, sp.ctypes.data)
        return b
    out = run_superframes(enc, x, nsf)
    lib.emu_destroy(e)
    return out


def test_encode_hostemu_matches_golden():
    """16 golden channels x 10 s through the host build of the device code"""
    g = golden()
    ch, nsf = 16, g["superframes"]
    bits, npp = emu_encode_all(signals(g["seed"], ch, nsf), nsf)
    for c in range(ch):
        if c < len(g["bits_hex"]):
            assert bits[c].tobytes().hex() == g["bits_hex"][c], "channel %d bits" % c
        assert sha(bits[c]) == g["bits_sha256"][c], "channel %d bits" % c
        assert sha(npp[c]) == g["npp_sha256"][c], "channel %d npp" % c


def test_encode_hostemu_edge_signals_match_live_reference(tmp_path, ref_tool):
    """saturating / degenerate inputs through the host build,
    against the reference compiled by oracle/Makefile"""
    nsf = 24
    sig = edge_signals(nsf * 540)
    names = sorted(sig)
    bits, _ = emu_encode_all(np.stack([sig[k] for k in names]), nsf)
    for i, k in enumerate(names):
        p = str(tmp_path / (k + ".pcm"))
        sig[k].tofile(p)
        subprocess.run([ref_tool, "enc", p, p + ".bits"], check=True)
        np.testing.assert_array_equal(bits[i], np.fromfile(p + ".bits", dtype=np.uint8), err_msg=k)


@pytest.mark.gpu
def test_encode_gpu_1024_channels_match_golden():
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], g["superframes"]
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    bits, npp = run_superframes(eng.encode, x, nsf)
    bad = [c for c in range(C) if sha(bits[c]) != g["bits_sha256"][c]]
    badn = [c for c in range(C) if sha(npp[c]) != g["npp_sha256"][c]]
    assert not bad, "bitstream mismatch on %d channels, first %s" % (len(bad), bad[:8])
    assert not badn, "NPP output mismatch on %d channels, first %s" % (len(badn), badn[:8])


@pytest.mark.gpu
def test_encode_gpu_lane_kernel_alone_1024_channels_match_golden():
    """The headline's lane-per-channel analysis (k_enc_ana -> k_enc_harm ->
    k_enc_tail) forced on every superframe (set_ana_waves(1)): at 1,024
    channels the automatic choice would run the four-wave kernel instead."""
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], g["superframes"]
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    eng.set_ana_waves(1)
    bits, npp = run_superframes(eng.encode, x, nsf)
    assert eng.last_ana_waves() == 1
    eng.close()
    bad = [c for c in range(C) if sha(bits[c]) != g["bits_sha256"][c]]
    badn = [c for c in range(C) if sha(npp[c]) != g["npp_sha256"][c]]
    assert not bad, "bitstream mismatch on %d channels, first %s" % (len(bad), bad[:8])
    assert not badn, "NPP output mismatch on %d channels, first %s" % (len(badn), badn[:8])


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [0, 1])
def test_encode_pipe_dev_matches_golden(waves):
    """The pipelined encode (melpe_encode_pipe_dev: superframe k's analysis
    beside superframe k+1's NPP on the engine's second stream) over the
    1,024-channel goldens x 149 superframes: the bits and the NPP output
    melpe_a leaves in the buffer, channel by channel -- with the automatic
    mapping (the four-wave analysis at this size) and the lane kernel."""
    import torch
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], g["superframes"]
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    x = torch.from_numpy(np.ascontiguousarray(
        signals(g["seed"], C, nsf).reshape(C, nsf, 540).transpose(1, 0, 2))).to(dev)
    bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
    eng = MelpeEngine(C)
    if waves:
        eng.set_ana_waves(waves)
    eng.encode_npp_dev(x[0].data_ptr(), None, s)
    for k in range(nsf):
        eng.encode_pipe_dev(bits[k].data_ptr(), x[k].data_ptr(),
                            x[k + 1].data_ptr() if k + 1 < nsf else None, stream=s)
    torch.cuda.synchronize(dev)
    eng.close()
    b = bits.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 11)
    n = x.cpu().numpy().transpose(1, 0, 2).reshape(C, nsf * 540)
    bad = [c for c in range(C) if sha(b[c]) != g["bits_sha256"][c]]
    badn = [c for c in range(C) if sha(n[c]) != g["npp_sha256"][c]]
    assert not bad, "bitstream mismatch on %d channels, first %s" % (len(bad), bad[:8])
    assert not badn, "NPP output mismatch on %d channels, first %s" % (len(badn), badn[:8])


@pytest.mark.gpu
def test_encode_host_two_threads_one_engine():
    """Two host threads calling melpe_encode_host on one engine at once,
    each on its own half of the channels (disjoint masks): every call holds
    the engine's lock while it stages PCM, mask and bits through the
    engine's shared buffers, so each thread gets exactly the bits and NPP
    output of one engine running all channels alone (ctypes releases the
    GIL during the calls, so the calls do overlap)."""
    import threading
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], 40
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    halves = [np.arange(C) % 2 == h for h in (0, 1)]
    out = [None, None]
    err = []

    def worker(h):
        try:
            xs = x.copy()
            bits = np.zeros((C, nsf * 11), np.uint8)
            for k in range(nsf):
                sp = np.ascontiguousarray(xs[:, k * 540:(k + 1) * 540])
                bits[:, k * 11:(k + 1) * 11] = eng.encode(sp, active=halves[h])
                xs[:, k * 540:(k + 1) * 540] = sp
            out[h] = (bits, xs)
        except Exception as e:  # noqa: BLE001
            err.append(e)
    th = [threading.Thread(target=worker, args=(h,)) for h in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    eng.close()
    assert not err, err
    ref = MelpeEngine(C)
    want, wnpp = run_superframes(ref.encode, x.copy(), nsf)
    ref.close()
    for h in (0, 1):
        bits, npp = out[h]
        np.testing.assert_array_equal(bits[halves[h]], want[halves[h]])
        np.testing.assert_array_equal(npp[halves[h]], wnpp[halves[h]])


@pytest.mark.gpu
def test_encode_host_async_matches_sync():
    """The host-fed pipeline (melpe_encode_host_async: two device slots,
    copies and kernels on three streams) against melpe_encode_host, on
    pinned and on pageable buffers, with a ragged mask on some superframes:
    the same bits and in-place NPP output"""
    import torch
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = 256, 12
    x = signals(g["seed"], C, nsf)
    rng = np.random.default_rng(3)
    masks = [None if k % 3 else (rng.random(C) < 0.6).astype(np.uint8) for k in range(nsf)]
    ref = MelpeEngine(C)
    want_b = np.zeros((nsf, C, 11), np.uint8)
    want_p = np.zeros((nsf, C, 540), np.int16)
    for k in range(nsf):
        sp = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        bits = np.full((C, 11), 0xAB, np.uint8)
        ref._raw_encode(sp, bits, masks[k])
        want_b[k], want_p[k] = bits, sp
    ref.close()
    for pinned in (True, False):
        eng = MelpeEngine(C)
        pcm = torch.from_numpy(np.ascontiguousarray(
            x[:, :nsf * 540].reshape(C, nsf, 540).transpose(1, 0, 2)))
        bits = torch.full((nsf, C, 11), 0xAB, dtype=torch.uint8)
        mk = torch.from_numpy(np.stack([m if m is not None else np.ones(C, np.uint8) for m in masks]))
        if pinned:
            pcm, bits, mk = pcm.pin_memory(), bits.pin_memory(), mk.pin_memory()
        for k in range(nsf):
            eng.encode_host_async(bits[k].data_ptr(), pcm[k].data_ptr(),
                                  None if masks[k] is None else mk[k].data_ptr())
        eng.encode_host_wait()
        eng.close()
        np.testing.assert_array_equal(bits.numpy(), want_b, err_msg="bits, pinned=%s" % pinned)
        np.testing.assert_array_equal(pcm.numpy(), want_p, err_msg="NPP output, pinned=%s" % pinned)


def edge_signals(n):
    rng = np.random.default_rng(5)
    t = np.arange(n)
    return {
        "zeros": np.zeros(n, np.int16),
        "noise_fs": rng.integers(-32768, 32767, n).astype(np.int16),
        "sine1k_fs": (32767 * np.sin(2 * np.pi * 1000 * t / 8000)).astype(np.int16),
        "square": np.where((t // 20) % 2 == 0, 32767, -32768).astype(np.int16),
        "dc_pos": np.full(n, 32767, np.int16),
        "dc_neg": np.full(n, -32768, np.int16),
        "impulses": np.where(t % 57 == 0, 30000, 0).astype(np.int16),
        "sweep": (20000 * np.sin(2 * np.pi * np.cumsum(np.linspace(50, 3900, n)) / 8000)).astype(np.int16),
        "speech_loud": np.clip(np.asarray(signals(9, 1, n // 540)[0], np.int32) * 4, -32768, 32767).astype(np.int16),
    }


@pytest.mark.gpu
def test_encode_gpu_edge_signals_match_live_reference(tmp_path, ref_tool):
    from pairphone_amd import MelpeEngine
    nsf = 40
    sig = edge_signals(nsf * 540)
    names = sorted(sig)
    x = np.stack([sig[k] for k in names])
    eng = MelpeEngine(len(names))
    bits, npp = run_superframes(eng.encode, x, nsf)
    for i, k in enumerate(names):
        p = str(tmp_path / (k + ".pcm"))
        sig[k].tofile(p)
        subprocess.run([REF_TOOL, "enc", p, p + ".bits"], check=True)
        rb = np.fromfile(p + ".bits", dtype=np.uint8)
        np.testing.assert_array_equal(bits[i], rb, err_msg=k)


@pytest.mark.gpu
def test_encode_gpu_ragged_mask():
    """Inactive channels keep state, PCM and bits untouched: a channel that
    is paused for some superframes equals the same channel fed only its
    active superframes."""
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = 8, 30
    x = signals(g["seed"], C, nsf)
    rng = np.random.default_rng(3)
    act = rng.random((nsf + 10, C)) < 0.7
    eng = MelpeEngine(C)
    pos = np.zeros(C, int)
    out = [[] for _ in range(C)]
    for k in range(act.shape[0]):
        sp = np.zeros((C, 540), np.int16)
        for c in range(C):
            if act[k, c] and pos[c] < nsf:
                sp[c] = x[c, pos[c] * 540:(pos[c] + 1) * 540]
        m = np.array([act[k, c] and pos[c] < nsf for c in range(C)], np.uint8)
        b0 = np.full((C, 11), 0xAB, np.uint8)
        sp_before = sp.copy()
        b = eng._raw_encode(sp, b0, m)
        for c in range(C):
            if m[c]:
                out[c].append(b[c].copy())
                pos[c] += 1
            else:
                assert (b[c] == 0xAB).all() and (sp[c] == sp_before[c]).all()
    for c in range(C):
        got = np.concatenate(out[c])[:pos[c] * 11]
        want = bytes.fromhex(g["bits_hex"][c])[:pos[c] * 11]
        assert got.tobytes() == want, "channel %d" % c


@pytest.mark.gpu
def test_single_stream_dropin_matches_golden():
    """melpe_i + melpe_a through include/melpe.h, as melpe/encoder.c does."""
    from pairphone_amd import Melpe
    g = golden()
    nsf = 60
    x = signals(g["seed"], 1, nsf)[0]
    m = Melpe()
    m.reset_process_state()   # a fresh reference process per test
    m.melpe_i()
    out = []
    for k in range(nsf):
        sp = x[k * 540:(k + 1) * 540].copy()
        out.append(m.melpe_a(sp))
    assert np.concatenate(out).tobytes() == bytes.fromhex(g["bits_hex"][0])[:nsf * 11]


def emu_encode_split(x, nsf, fn="emu_encode_ana_split"):
    """the split lane analysis (encoder.h analysis_a / analysis_b, as
    k_enc_ana / k_enc_harm / k_enc_tail run it), NPP first"""
    lib = emu()
    lib.emu_encode_npp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    f = getattr(lib, fn)
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    e = lib.emu_create(x.shape[0])

    def enc(sp):
        b = np.zeros((x.shape[0], 11), np.uint8)
        lib.emu_encode_npp(e, sp.ctypes.data)
        assert f(e, b.ctypes.data, sp.ctypes.data) == 0
        return b
    out = run_superframes(enc, x, nsf)
    lib.emu_destroy(e)
    return out


def test_split_analysis_hostemu_matches_golden(fn="emu_encode_ana_split"):
    """8 golden channels x 10 s through analysis_a, find_harm on the written
    residuals, analysis_b: the goldens' bits and NPP samples"""
    g = golden()
    ch, nsf = 8, g["superframes"]
    bits, npp = emu_encode_split(signals(g["seed"], ch, nsf), nsf, fn)
    for c in range(ch):
        assert sha(bits[c]) == g["bits_sha256"][c], "channel %d bits" % c
        assert sha(npp[c]) == g["npp_sha256"][c], "channel %d npp" % c


def test_split_analysis_hostemu_edge_signals_match_serial(fn="emu_encode_ana_split"):
    nsf = 16
    sig = edge_signals(nsf * 540)
    x = np.stack([sig[k] for k in sorted(sig)])
    want, _ = emu_encode_all(x.copy(), nsf)
    got, _ = emu_encode_split(x.copy(), nsf, fn)
    np.testing.assert_array_equal(got, want)
