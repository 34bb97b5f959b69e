"""TX voice-activity gate parity against the reference.

The AMR VAD option 2 (vad/vad2.c) that PairPhone runs on six 80-sample
windows per superframe (tx.c:234-239, melpe_enc.c:48-53).  Oracle = the
reference's own vad/*.c compiled into oracle/_ref/libref_vad.so (harness
oracle/ref_vad.c, fresh vad2_reset state per channel); golden fixture
tests/golden/vad.json (make_vad_golden.py): 56 speech-like channels + 8 edge
channels x 149 superframes, votes = sum of the six decisions.

CPU: oracle and the host build of vad.h against the golden.
GPU: k_vad through the C ABI against the golden (host ABI, superframe by
superframe), at 65,536 channels against the live oracle through the device
ABI, ragged activity masks and per-channel reset.
"""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, GOLDEN

sys.path.insert(0, GOLDEN)
from make_vad_golden import inputs, ref_vad  # noqa: E402

EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
P = ctypes.c_void_p


def golden():
    g = json.load(open(os.path.join(GOLDEN, "vad.json")))
    v = np.frombuffer(bytes.fromhex(g["votes_hex"]), np.uint8)
    return g, v.reshape(g["channels"], g["superframes"])


def emu_vad(x, nsf):
    lib = ctypes.CDLL(EMU)
    C = x.shape[0]
    st = np.zeros(C * lib.emu_vad_state_bytes(), np.uint8)
    votes = np.zeros((C, nsf), np.uint8)
    x = np.ascontiguousarray(x, np.int16)
    lib.emu_vad(P(st.ctypes.data), P(x.ctypes.data), P(votes.ctypes.data), C, nsf)
    return votes


def test_oracle_matches_golden():
    g, want = golden()
    assert np.array_equal(ref_vad(inputs(g["channels"], g["superframes"], g["seed"]),
                                  g["superframes"]), want)


def test_hostemu_matches_golden():
    g, want = golden()
    got = emu_vad(inputs(g["channels"], g["superframes"], g["seed"]), g["superframes"])
    assert np.array_equal(got, want)
    assert (want == 0).any() and (want == 6).any()     # both gate outcomes covered


@pytest.mark.gpu
def test_gpu_matches_golden():
    from pairphone_amd import Vad
    g, want = golden()
    C, nsf = g["channels"], g["superframes"]
    x = inputs(C, nsf, g["seed"]).reshape(C, nsf, 540)
    vad = Vad(C)
    got = np.stack([vad.superframe(x[:, k]) for k in range(nsf)], axis=1)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_65536_channels_ragged_match_reference():
    import torch
    from pairphone_amd import load_library, synth_signal
    lib = load_library()
    C, nsf = 65536, 6
    rng = np.random.default_rng(5)
    # distinct channels: generator channels 0..255 cycled, scaled per channel
    base = np.stack([synth_signal(3, c, nsf * 540) for c in range(256)])
    gain = rng.integers(1, 5, C)
    x = (base[np.arange(C) % 256].astype(np.int32) * gain[:, None] // 2)
    x = np.clip(x, -32768, 32767).astype(np.int16)
    want = ref_vad(x, nsf)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    st = torch.zeros(C * lib.melpe_vad_state_bytes(), dtype=torch.uint8, device=dev)
    assert lib.melpe_vad_reset_dev(st.data_ptr(), C, None, s) == 0
    d_x = torch.from_numpy(x.reshape(C, nsf, 540)).to(dev)
    votes = torch.full((nsf, C), 255, dtype=torch.uint8, device=dev)
    for k in range(nsf):
        sp = d_x[:, k].contiguous()
        assert lib.melpe_vad_dev(st.data_ptr(), sp.data_ptr(), votes[k].data_ptr(), C,
                                 None, s) == 0
    assert np.array_equal(votes.cpu().numpy().T, want)
    # ragged: odd channels skip superframe 0 (state and vote untouched), so
    # they see superframes 1..5 as their first five
    mask = (np.arange(C) % 2 == 0).astype(np.uint8)
    d_m = torch.from_numpy(mask).to(dev)
    assert lib.melpe_vad_reset_dev(st.data_ptr(), C, None, s) == 0
    votes.fill_(255)
    for k in range(nsf):
        sp = d_x[:, k].contiguous()
        m = d_m.data_ptr() if k == 0 else None
        assert lib.melpe_vad_dev(st.data_ptr(), sp.data_ptr(), votes[k].data_ptr(), C, m,
                                 s) == 0
    got = votes.cpu().numpy().T
    assert np.array_equal(got[0::2], want[0::2])
    assert (got[1::2, 0] == 255).all()
    want_odd = ref_vad(x.reshape(C, nsf, 540)[1::2, 1:].reshape(C // 2, -1), nsf - 1)
    assert np.array_equal(got[1::2, 1:], want_odd)


@pytest.mark.gpu
def test_gpu_tx_front_end_vad_gated_ragged_matches_reference(tmp_path, ref_tool):
    """BASELINE config 5 in miniature: ragged stream lengths, the VAD gate
    and melpe_a on the superframes it opens (melpe_tx_dev), against the
    reference VAD + the reference codec run only on the gated superframes
    (ref_tool encgate)."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor
    import torch
    from pairphone_amd import MelpeEngine, load_library, synth_signal
    lib = load_library()
    C, nsf = 96, 14
    rng = np.random.default_rng(11)
    x = np.stack([synth_signal(9, c, nsf * 540) for c in range(C)]).reshape(C, nsf, 540)
    # silent stretches (low noise) so that the gate closes on some superframes
    for c in range(C):
        for k in rng.choice(nsf, size=rng.integers(0, 6), replace=False):
            x[c, k] = rng.integers(-20, 21, 540)
    lengths = rng.integers(3, nsf + 1, C)
    want_votes = np.zeros((C, nsf), np.uint8)
    for c in range(C):
        L = lengths[c]
        want_votes[c, :L] = ref_vad(x[c, :L].reshape(1, -1), L)[0]

    def ref_bits(c):
        L = lengths[c]
        pcm, gate, out = (str(tmp_path / ("%s%d" % (n, c))) for n in ("p", "g", "b"))
        x[c, :L].tofile(pcm)
        (want_votes[c, :L] > 0).astype(np.uint8).tofile(gate)
        subprocess.run([ref_tool, "encgate", pcm, gate, out], check=True)
        return np.fromfile(out, np.uint8).reshape(L, 11)
    with ThreadPoolExecutor(8) as ex:
        want_bits = list(ex.map(ref_bits, range(C)))

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    acts = torch.from_numpy(np.stack([(lengths > k).astype(np.uint8) for k in range(nsf)])).to(dev)
    # melpe_tx_dev per superframe, then the pipelined form (melpe_tx_npp_dev,
    # melpe_tx_pipe_dev: superframe k's analysis beside k+1's VAD and NPP)
    for pipe in (False, True):
        eng = MelpeEngine(C)
        st = torch.zeros(C * lib.melpe_vad_state_bytes(), dtype=torch.uint8, device=dev)
        assert lib.melpe_vad_reset_dev(st.data_ptr(), C, None, s) == 0
        d_x = torch.from_numpy(np.ascontiguousarray(x.transpose(1, 0, 2))).to(dev)   # nsf x C x 540
        bits = torch.zeros((nsf, C, 11), dtype=torch.uint8, device=dev)
        votes = torch.zeros((nsf, C), dtype=torch.uint8, device=dev)
        gate = torch.zeros((nsf, C), dtype=torch.uint8, device=dev)
        if pipe:
            eng.tx_npp_dev(st.data_ptr(), d_x[0].data_ptr(), votes[0].data_ptr(), gate[0].data_ptr(),
                           acts[0].data_ptr(), s)
        for k in range(nsf):
            if not pipe:
                eng.tx_dev(st.data_ptr(), bits[k].data_ptr(), d_x[k].data_ptr(), votes[k].data_ptr(),
                           gate[k].data_ptr(), acts[k].data_ptr(), s)
                continue
            nx = k + 1 < nsf
            eng.tx_pipe_dev(st.data_ptr(), bits[k].data_ptr(), d_x[k].data_ptr(), gate[k].data_ptr(),
                            d_x[k + 1].data_ptr() if nx else None, votes[k + 1].data_ptr() if nx else None,
                            gate[k + 1].data_ptr() if nx else None, acts[k + 1].data_ptr() if nx else None,
                            stream=s)
        torch.cuda.synchronize()
        eng.close()
        got_votes = votes.cpu().numpy().T
        got_gate = gate.cpu().numpy().T
        got_bits = bits.cpu().numpy().transpose(1, 0, 2)
        closed = 0
        for c in range(C):
            L = lengths[c]
            assert np.array_equal(got_votes[c, :L], want_votes[c, :L]), (pipe, c)
            assert np.array_equal(got_gate[c], (np.arange(nsf) < L) & (want_votes[c] > 0)), (pipe, c)
            assert np.array_equal(got_bits[c, :L], want_bits[c]), (pipe, c)
            assert not got_bits[c, L:].any()
            closed += int((want_votes[c, :L] == 0).sum())
        assert closed > 0      # the gate did close somewhere
