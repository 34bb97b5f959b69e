"""The pitch-class lane order (engine.hip, melpe_engine_set_lane_order).

Before each analysis / synthesis launch the engine sorts the live channels by
pitch class, so lane g of the kernel runs channel perm[g], and a ragged mask
is packed into the fewest waves.  The order must never change a channel's
result: these tests run the same streams through an engine with the order on
and one with it off, under sparse ragged masks and over enough superframes
for the classes to move, and require identical bits, NPP output and PCM.
The order-off engine is itself pinned to the reference by the golden tests
(test_encode.py / test_decode.py run with the default order on).
"""
import numpy as np
import pytest


def _streams(C, nsf, seed=2026):
    from pairphone_amd import synth_signal
    return np.stack([synth_signal(seed, c, nsf * 540) for c in range(C)])


@pytest.mark.gpu
def test_lane_order_is_invisible_under_ragged_masks():
    from pairphone_amd import MelpeEngine
    C, nsf = 1536, 16
    x = _streams(C, nsf)
    rng = np.random.default_rng(5)
    on, off = MelpeEngine(C), MelpeEngine(C)
    on.set_lane_order(True)
    off.set_lane_order(False)
    for k in range(nsf):
        # every channel runs its first superframes, then a ragged 35% / 100%
        # mix, so the live set is sparse and scattered across waves
        m = (rng.random(C) < (0.35 if k % 3 else 1.0)).astype(np.uint8)
        if k < 2:
            m[:] = 1
        sp_on = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        sp_off = sp_on.copy()
        b_on = on.encode(sp_on, m)
        b_off = off.encode(sp_off, m)
        np.testing.assert_array_equal(b_on, b_off, err_msg="bits, superframe %d" % k)
        np.testing.assert_array_equal(sp_on, sp_off, err_msg="NPP output, superframe %d" % k)
        assert (b_on[m == 0] == 0).all(), "an inactive channel's bits were written"
        p_on = on.decode(b_on, m)
        p_off = off.decode(b_off, m)
        np.testing.assert_array_equal(p_on, p_off, err_msg="PCM, superframe %d" % k)
        assert (p_on[m == 0] == 0).all(), "an inactive channel's PCM was written"


@pytest.mark.gpu
def test_lane_order_with_no_live_channel():
    """An all-zero mask leaves an empty order: the kernels launch and exit."""
    from pairphone_amd import MelpeEngine
    C = 256
    eng = MelpeEngine(C)
    eng.set_lane_order(True)
    sp = np.ascontiguousarray(_streams(C, 1))
    before = sp.copy()
    m = np.zeros(C, np.uint8)
    bits = eng.encode(sp, m)
    assert (bits == 0).all()
    np.testing.assert_array_equal(sp, before)
    assert (eng.decode(bits, m) == 0).all()
