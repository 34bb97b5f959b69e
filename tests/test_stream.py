"""VAD-framed stream format (melpe_enc.c:55-72 / melpe_dec.c:33-49) against
the reference's own decoder.

Streams are built by melpe_stream_pack from reference-gated bitstreams (the
reference VAD's votes, then ref_tool encgate: melpe_a on the voiced
superframes only) and fed to the reference's unchanged melpe_dec
(oracle/_ref/melpe_dec, built from /root/reference/melpe_dec.c).  Its PCM
must equal the reference decoder run on the voiced superframes alone with
540 zeros per silent one, which pins the framing (a mis-framed stream
desynchronises melpe_dec).  melpe_stream_unpack must invert the packing.
GPU: the engine decodes the unpacked frames to melpe_dec's PCM.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, GOLDEN, REF_DIR

sys.path.insert(0, GOLDEN)
from make_vad_golden import ref_vad  # noqa: E402

MELPE_DEC = os.path.join(REF_DIR, "melpe_dec")
C, NSF = 4, 24


def signals():
    from pairphone_amd import synth_signal
    rng = np.random.default_rng(21)
    x = np.stack([synth_signal(4, c, NSF * 540) for c in range(C)]).reshape(C, NSF, 540)
    for c in range(C):
        for k in rng.choice(NSF, size=6 + c, replace=False):
            x[c, k] = rng.integers(-15, 16, 540)
    return x


def gated_reference(tmp_path, ref_tool, x, c):
    votes = ref_vad(x[c].reshape(1, -1), NSF)[0]
    pcm, gate, out = (str(tmp_path / ("%s%d" % (n, c))) for n in ("p", "g", "b"))
    x[c].tofile(pcm)
    (votes > 0).astype(np.uint8).tofile(gate)
    subprocess.run([ref_tool, "encgate", pcm, gate, out], check=True)
    return votes, np.fromfile(out, np.uint8).reshape(NSF, 11)


def ref_melpe_dec(tmp_path, stream, c):
    fi, fo = str(tmp_path / ("s%d" % c)), str(tmp_path / ("o%d" % c))
    open(fi, "wb").write(stream)
    subprocess.run([MELPE_DEC, fi, fo], check=True, capture_output=True)
    return np.fromfile(fo, np.int16)


def test_pack_matches_reference_decoder_and_unpack_inverts(tmp_path, ref_tool):
    from pairphone_amd import stream_pack, stream_unpack
    x = signals()
    silent = 0
    for c in range(C):
        votes, bits = gated_reference(tmp_path, ref_tool, x, c)
        stream = stream_pack(bits, votes)
        v = votes > 0
        assert len(stream) == int(v.sum()) * 11 + int((~v).sum())
        # expected PCM: the reference decoder on the voiced superframes only
        vb = str(tmp_path / ("vb%d" % c))
        bits[v].tofile(vb)
        subprocess.run([ref_tool, "dec", vb, vb + ".pcm"], check=True)
        dec_v = np.fromfile(vb + ".pcm", np.int16).reshape(-1, 540)
        want = np.zeros((NSF, 540), np.int16)
        want[v] = dec_v
        got = ref_melpe_dec(tmp_path, stream, c).reshape(-1, 540)
        assert np.array_equal(got, want), c
        ub, uv = stream_unpack(stream)
        assert np.array_equal(uv, v.astype(np.uint8))
        assert np.array_equal(ub[v], bits[v]) and not ub[~v].any()
        silent += int((~v).sum())
    assert silent > 0


def test_unpack_edges(engine_lib):
    from pairphone_amd import stream_unpack
    b, v = stream_unpack(b"")
    assert len(b) == 0 and len(v) == 0
    b, v = stream_unpack(bytes([2, 3, 0xFF]))       # three silence descriptors
    assert list(v) == [0, 0, 0]
    with pytest.raises(RuntimeError):
        stream_unpack(bytes([1] + [0] * 5))          # truncated voiced frame


@pytest.mark.gpu
def test_gpu_decodes_stream_like_reference_decoder(tmp_path, ref_tool):
    from pairphone_amd import MelpeEngine, stream_pack, stream_unpack
    x = signals()
    for c in range(C):
        votes, bits = gated_reference(tmp_path, ref_tool, x, c)
        stream = stream_pack(bits, votes)
        want = ref_melpe_dec(tmp_path, stream, c).reshape(-1, 540)
        ub, uv = stream_unpack(stream)
        eng = MelpeEngine(1)
        got = np.zeros_like(want)
        for k in range(len(uv)):
            if uv[k]:
                got[k] = eng.decode(ub[k:k + 1])[0]
        eng.close()
        assert np.array_equal(got, want), c
