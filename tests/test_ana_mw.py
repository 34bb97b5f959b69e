"""The multi-wave analysis (pairphone_amd/csrc/ana_mw.h, k_enc_ana_mw):
analysis() of one channel split over 1, 2 or 4 waves of a workgroup, each
wave on its own copy of the state, meeting only through the exchange block
and the HBM record between phases.

CPU: the host build runs the same phase program with one private copy per
physical wave and checks the bitstream against the reference's goldens
(tests/golden/enc_1024.json) and the edge signals against the serial host
build.  GPU: k_enc_ana_mw at each wave count against the goldens, and the
32,768-channel configuration (BASELINE config 4's 8-GPU shard) against the
live reference on sampled channels.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

from test_encode import emu, golden, signals, sha, run_superframes, edge_signals

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def emu_mw(nw):
    lib = emu()
    lib.emu_encode_npp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_encode_ana_mw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return lib


def emu_encode_mw(x, nsf, nw):
    lib = emu_mw(nw)
    e = lib.emu_create(x.shape[0])

    def enc(sp):
        b = np.zeros((x.shape[0], 11), np.uint8)
        lib.emu_encode_npp(e, sp.ctypes.data)
        assert lib.emu_encode_ana_mw(e, b.ctypes.data, sp.ctypes.data, nw) == 0
        return b
    out = run_superframes(enc, x, nsf)
    lib.emu_destroy(e)
    return out


@pytest.mark.parametrize("nw", [1, 2, 4])
def test_mw_hostemu_matches_golden(nw):
    """8 golden channels x 10 s, the phase program on nw waves"""
    g = golden()
    ch, nsf = 8, g["superframes"]
    bits, npp = emu_encode_mw(signals(g["seed"], ch, nsf), nsf, nw)
    for c in range(ch):
        assert sha(bits[c]) == g["bits_sha256"][c], "channel %d bits (nw %d)" % (c, nw)
        assert sha(npp[c]) == g["npp_sha256"][c], "channel %d npp (nw %d)" % (c, nw)


def test_mw_hostemu_edge_signals_match_serial():
    from test_encode import emu_encode_all
    nsf = 16
    sig = edge_signals(nsf * 540)
    x = np.stack([sig[k] for k in sorted(sig)])
    want, _ = emu_encode_all(x.copy(), nsf)
    got, _ = emu_encode_mw(x.copy(), nsf, 4)
    np.testing.assert_array_equal(got, want)


def _gpu_encode(C, nsf, waves, seed):
    """C channels x nsf superframes of the synth signal, encoded on the GPU
    with `waves` analysis waves per 64 channels (0 = the engine's choice);
    returns bits [nsf, C, 11] on the host"""
    import torch
    from pairphone_amd import MelpeEngine
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    eng.set_ana_waves(waves)
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.synth_seed(seed)
    pcm = torch.empty((C, 540), dtype=torch.int16, device=dev)
    bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
    for k in range(nsf):
        eng.synth_dev(pcm.data_ptr(), 540, s)
        eng.encode_dev(bits[k].data_ptr(), pcm.data_ptr(), None, s)
    torch.cuda.synchronize(dev)
    eng.close()
    return bits.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("nw", [4])
def test_mw_gpu_1024_channels_match_golden(nw):
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], g["superframes"]
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    eng.set_ana_waves(nw)
    bits, npp = run_superframes(eng.encode, x, nsf)
    bad = [c for c in range(C) if sha(bits[c]) != g["bits_sha256"][c]]
    assert not bad, "nw %d: bitstream mismatch on %d channels, first %s" % (nw, len(bad), bad[:8])


@pytest.mark.gpu
def test_mw_gpu_32768_channels_match_reference(tmp_path, ref_tool):
    """BASELINE config 4's per-GPU shard at N=8 (262,144 / 8 channels), the
    channel count the multi-wave kernel is for, over the whole 10 s stream:
    64 channels sampled across the range against the reference codec."""
    from test_scale import _sampled, _ref_channels, SEED
    C, nsf = 32768, 149
    b = _gpu_encode(C, nsf, 0, SEED)
    chans = _sampled(C, 64)
    ref = _ref_channels(tmp_path, chans, nsf, decode=False)
    for c in chans:
        np.testing.assert_array_equal(b[:, c, :], ref[c][0], err_msg="bits, channel %d" % c)


@pytest.mark.gpu
def test_mw_gpu_wave_counts_agree():
    """1 and 4 waves per channel group give the same bits on a batch that
    mixes every voicing pattern (4,096 channels x 24 superframes)"""
    C, nsf = 4096, 24
    ref = _gpu_encode(C, nsf, 1, 77)
    for nw in (4,):
        np.testing.assert_array_equal(_gpu_encode(C, nsf, nw, 77), ref, err_msg="nw %d" % nw)


@pytest.mark.gpu
@pytest.mark.parametrize("nw", [1, 4])
def test_two_streams_disjoint_masks(nw):
    """One engine, encode_dev on two streams at once with disjoint channel
    masks (the header allows it: *_dev calls are ordered by their stream
    only): the engine's lane-order scratch is shared by both calls, so the
    second call's sort must wait for the first call's kernel.  Every channel
    must get the bits of a plain one-stream run."""
    import torch
    from pairphone_amd import MelpeEngine
    C, nsf = 2048, 12
    want = _gpu_encode(C, nsf, nw, 91)
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    eng.set_ana_waves(nw)
    s0 = torch.cuda.current_stream(dev)
    eng.synth_seed(91)
    pcm = torch.empty((nsf, C, 540), dtype=torch.int16, device=dev)
    for k in range(nsf):
        eng.synth_dev(pcm[k].data_ptr(), 540, s0.cuda_stream)
    even = (torch.arange(C, device=dev) % 2 == 0).to(torch.uint8)
    odd = (1 - even).to(torch.uint8)
    bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sa.wait_stream(s0)
    sb.wait_stream(s0)
    for k in range(nsf):
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), even.data_ptr(), sa.cuda_stream)
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), odd.data_ptr(), sb.cuda_stream)
    torch.cuda.synchronize(dev)
    np.testing.assert_array_equal(bits.cpu().numpy(), want)
    eng.close()


def test_mw_hostemu_many_channels_match_serial():
    """64 synthetic channels (another seed) x 40 superframes: every voicing
    pattern, so every lsf_vq path of the multi-wave search, against the
    serial host build"""
    from test_encode import emu_encode_all
    nsf = 40
    x = signals(4242, 64, nsf)
    want, _ = emu_encode_all(x.copy(), nsf)
    got, _ = emu_encode_mw(x.copy(), nsf, 4)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_mw_gpu_mapping_alternates_between_superframes():
    """The two analysis mappings on the same records, switched between
    superframes (lane, four-wave, lane, ...): the 1,024-channel goldens.
    Both mappings read and write the channel records in one layout, so any
    superframe can run on either (engine.hip ana_launch's live-count pick
    relies on that)."""
    from pairphone_amd import MelpeEngine
    g = golden()
    C, nsf = g["channels"], g["superframes"]
    x = signals(g["seed"], C, nsf)
    eng = MelpeEngine(C)
    k = [0]

    def enc(sp):
        eng.set_ana_waves(1 if (k[0] // 3) % 2 == 0 else 4)
        k[0] += 1
        return eng.encode(sp)
    bits, npp = run_superframes(enc, x, nsf)
    bad = [c for c in range(C) if sha(bits[c]) != g["bits_sha256"][c]]
    assert not bad, "bitstream mismatch on %d channels, first %s" % (len(bad), bad[:8])


def _gpu_encode_masked(C, masks, live_max, waves, seed, choice=None):
    """C channels under per-superframe activity masks [nsf, C]; returns bits
    [nsf, C, 11] (0xAB where a channel was inactive); `choice`, a list,
    receives the mapping each superframe's analysis ran (the device's
    record, after each superframe)"""
    import torch
    from pairphone_amd import MelpeEngine
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    eng.set_ana_waves(waves)
    eng.set_mw_live_max(live_max)
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.synth_seed(seed)
    nsf = masks.shape[0]
    pcm = torch.empty((C, 540), dtype=torch.int16, device=dev)
    bits = torch.full((nsf, C, 11), 0xAB, dtype=torch.uint8, device=dev)
    m = torch.from_numpy(masks.astype(np.uint8)).to(dev)
    for k in range(nsf):
        eng.synth_dev(pcm.data_ptr(), 540, s)
        eng.encode_dev(bits[k].data_ptr(), pcm.data_ptr(), m[k].data_ptr(), s)
        if choice is not None:
            choice.append(eng.last_ana_waves())
    torch.cuda.synchronize(dev)
    eng.close()
    return bits.cpu().numpy()


@pytest.mark.gpu
def test_mw_gpu_live_count_pick_ragged():
    """65,536 channels (above the four-wave kernel's channel count) under
    ragged masks whose live count crosses 32,768 both ways: with the
    live-count pick on (the default) every superframe with <= 32,768 live
    channels runs k_enc_ana_mw, the others the lane kernels, decided on the
    device (both enqueued, each gated on the sort's live count; the device
    records which ran).  Every channel's bits equal the lane kernels' alone
    (pick off) and the four-wave kernel's alone."""
    C, nsf = 65536, 10
    rng = np.random.default_rng(12)
    live = [60000, 20000, 32768, 32769, 1000, 45000, 30000, 64, 65536, 16000]
    masks = np.zeros((nsf, C), bool)
    for k, n in enumerate(live):
        masks[k, rng.choice(C, n, replace=False)] = True
    choice = []
    got = _gpu_encode_masked(C, masks, 32768, 0, 5, choice)
    assert choice == [4 if n <= 32768 else 1 for n in live], choice
    lane = _gpu_encode_masked(C, masks, 0, 0, 5)
    np.testing.assert_array_equal(got, lane)
    mw = _gpu_encode_masked(C, masks, 0, 4, 5)
    np.testing.assert_array_equal(got, mw)


_SCRATCH_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from pairphone_amd import MelpeEngine
dev = torch.device("cuda", 0)
C = 65536
hog, size = [], 1 << 30
while size >= (1 << 22):
    try:
        hog.append(torch.empty(size, dtype=torch.uint8, device=dev))
    except RuntimeError:
        size //= 2
try:
    MelpeEngine(C)
    print("CREATED")
except RuntimeError as e:
    print("CREATE FAILED:", e)
"""


@pytest.mark.gpu
def test_engine_create_fails_cleanly_without_scratch():
    """The engine's buffers and its kernels' private-segment scratch are
    had at melpe_engine_create (engine.hip engine_reserve: one dispatch of
    each kernel with a real launch's grid): on a device torch has filled,
    create fails with an error message instead of the first encode
    faulting mid-stream.  Run in a child process, so the filled device and
    any queue the runtime tears down stay out of this suite."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", _SCRATCH_CHILD, ROOT], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "CREATE FAILED" in r.stdout, r.stdout[-2000:]
