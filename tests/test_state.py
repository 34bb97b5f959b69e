"""Per-channel state records (melpe_engine_export / melpe_engine_import) and
stream-ordered reset (melpe_engine_reset_dev).

The reference keeps one codec instance in process globals (SURVEY.md §5:
"checkpointing becomes trivial once state is explicit"); here a channel's
whole encoder / decoder state is one record, so a channel can be
checkpointed, resumed, or moved to another engine (another GPU, a re-balanced
ragged shard) mid-stream and continue bit-exactly.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _input(C, nsf):
    from pairphone_amd import synth_signal
    ge = json.load(open(os.path.join(GOLDEN, "enc_1024.json")))
    return ge, np.stack([synth_signal(ge["seed"], c, nsf * 540) for c in range(C)])


@pytest.mark.gpu
def test_state_migration_between_engines_is_bit_exact():
    from pairphone_amd import MelpeEngine
    C, nsf, cut = 8, 30, 11
    ge, x = _input(C, nsf)
    a = MelpeEngine(C)
    ref_bits = np.zeros((nsf, C, 11), np.uint8)
    ref_pcm = np.zeros((nsf, C, 540), np.int16)
    mig_bits = np.zeros_like(ref_bits)
    mig_pcm = np.zeros_like(ref_pcm)
    for k in range(cut):
        sp = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        ref_bits[k] = a.encode(sp)
        ref_pcm[k] = a.decode(ref_bits[k])
    enc = a.export_state(1)
    dec = a.export_state(2)
    assert enc.shape == (C, a.lib.melpe_engine_state_bytes(1))
    # channels land in reversed slots of a fresh engine with 3 extra channels
    b = MelpeEngine(C + 3)
    perm = np.arange(C)[::-1] + 2
    for c in range(C):
        b.import_state(1, enc[c:c + 1], first=int(perm[c]))
        b.import_state(2, dec[c:c + 1], first=int(perm[c]))
    for k in range(cut, nsf):
        sp = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        ref_bits[k] = a.encode(sp.copy())
        ref_pcm[k] = a.decode(ref_bits[k])
        spb = np.zeros((C + 3, 540), np.int16)
        spb[perm] = sp
        bb = b.encode(spb)
        mig_bits[k] = bb[perm]
        mig_pcm[k] = b.decode(bb)[perm]
    np.testing.assert_array_equal(mig_bits[cut:], ref_bits[cut:])
    np.testing.assert_array_equal(mig_pcm[cut:], ref_pcm[cut:])
    for c in range(C):   # and the unmigrated stream is the reference's
        assert ref_bits[:, c].tobytes().hex() == ge["bits_hex"][c][:nsf * 22]
    a.close()
    b.close()


@pytest.mark.gpu
def test_reset_dev_is_stream_ordered():
    """encode on a torch stream, then reset channel 1 on that same stream
    with no host sync, then encode again: channel 1 restarts from fresh
    state (its bits equal superframe 0's), the others continue"""
    import torch
    from pairphone_amd import MelpeEngine
    C, nsf = 4, 6
    _, x = _input(C, nsf)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    eng = MelpeEngine(C)
    pcm = torch.from_numpy(x.reshape(C, nsf, 540).transpose(1, 0, 2).copy()).to(dev)
    bits = torch.zeros((nsf + 1, C, 11), dtype=torch.uint8, device=dev)
    mask = torch.tensor([0, 1, 0, 0], dtype=torch.uint8, device=dev)
    first = pcm[0].clone()
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(st):
        s = st.cuda_stream
        for k in range(nsf):
            eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
        eng.reset_dev(mask.data_ptr(), 3, s)
        eng.encode_dev(bits[nsf].data_ptr(), first.data_ptr(), mask.data_ptr(), s)
    st.synchronize()
    b = bits.cpu().numpy()
    np.testing.assert_array_equal(b[nsf, 1], b[0, 1])
    np.testing.assert_array_equal(b[nsf, [0, 2, 3]], 0)   # masked off: untouched
    eng.close()


@pytest.mark.gpu
def test_import_rejects_foreign_records():
    """a record of another layout (here: a corrupted format tag, as a
    checkpoint of an older build would carry) is refused, nothing written"""
    from pairphone_amd import MelpeEngine
    a = MelpeEngine(2)
    rec = a.export_state(1)
    before = rec.copy()
    bad = rec.copy()
    bad[1, -4:] ^= 0x5a
    with pytest.raises(RuntimeError, match="layout"):
        a.import_state(1, bad)
    np.testing.assert_array_equal(a.export_state(1), before)
    a.import_state(1, rec)    # its own records go back in
    a.close()
