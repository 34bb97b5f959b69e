"""The device-only helpers behind the codec's sample streams and exact
correlators (pairphone_amd/csrc/dsp.h:30-330, analysis.h fp_sums9; driven by
csrc/helpers_eval.h): P16 pair streams, PairStream / P16C chunked pairs,
xcorr_pairs for the lag-block shapes find_pitch, corPeak and frac_cor use,
fp_sums9, and the primitive ops sdot2 / sdot2_sat / pair_mid / pk_hi8 /
pk_lo8 / perm_b32 -- at every start alignment of both streams and lengths
from 0 to 200 (odd, even, below the 4-pair groups).

Checked against plain integer arithmetic in numpy (the helpers' definition:
sums wrap modulo 2^32, as v_dot2_i32_i16 without clamp does; the split
correlators sum hi8 = x >> 8 and lo8 = x & 255 separately).  CPU: the host
build of the same header; GPU: melpe_helpers_eval_dev, each lane on its
own private array, so a wave mixes alignments exactly as the codec's lanes
do.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

HE_N, HE_OUT = 464, 512
EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")

# (NA, NB, oa(k), ob(k), K, split) of the lag-block shapes (dsp.h FpLags,
# analysis.h CpLags / FcLags11)
def _fp(K):
    bmax = (K - 1) - K // 2
    return (K // 2 + 1, bmax + 1, lambda k: (k + 1) // 2, lambda k: (k + 1) // 2 - k + bmax, K, False)


SHAPES = {3: _fp(8), 4: (4, 5, lambda k: k // 2, lambda k: 4 - (k + 1) // 2, 8, True),
          5: (6, 6, lambda n: (n + 1) // 2, lambda n: (n + 1) // 2 - n + 5, 11, True),
          6: _fp(12)}


def wrap32(v):
    return ((np.asarray(v, np.int64) + 2**31) % 2**32 - 2**31).astype(np.int64)


def cases(mode, n, seed):
    g = np.random.default_rng(seed + mode)
    src = g.integers(-32768, 32768, (n, HE_N)).astype(np.int16)
    # a quarter of the lanes at full-scale extremes (sums that wrap)
    ext = g.random((n, HE_N)) < 0.05
    src[ext] = np.where(g.random(ext.sum()) < 0.5, -32768, 32767)
    args = np.zeros((n, 4), np.int32)
    for i in range(n):
        if mode == 8:
            a, b = 2 * g.integers(0, 200), 2 * g.integers(0, 200)
            sel = g.integers(0, 8, 4)
            ln = int(g.integers(-2**31, 2**31)) if i % 2 else int(sel[0] | sel[1] << 8 | sel[2] << 16 | sel[3] << 24)
        else:
            ln = int(g.integers(0, 201)) if i % 3 else int(g.integers(0, 12))
            a = int(g.integers(0, 40)) + (i & 1)
            b = int(g.integers(0, 40)) + ((i >> 1) & 1)
        args[i, :3] = (a, b, ln)
    return src, args


def want(mode, src, args):
    n = src.shape[0]
    out = np.zeros((n, HE_OUT), np.int64)
    for i in range(n):
        a, b, ln = (int(v) for v in args[i, :3])
        x = src[i].astype(np.int64)
        if mode == 0:
            out[i, :ln] = x[a:a + ln]
        elif mode in (1, 2):
            m = (ln + 1) // 2
            pairs = np.zeros(2 * m, np.int64)
            pairs[:ln] = x[a:a + ln]
            if mode == 1:
                out[i, :2 * m] = pairs
            else:
                nfull = (ln - 1) // 2 if a % 2 else ln // 2
                G = max((nfull - 1) // 4, 0)
                out[i, 2:2 + 8 * G] = pairs[2:2 + 8 * G]
        elif mode in SHAPES:
            NA, NB, oa, ob, K, split = SHAPES[mode]
            for k in range(K):
                pa, pb = x[a + oa(k):a + oa(k) + ln], x[b + ob(k):b + ob(k) + ln]
                if split:
                    out[i, k] = wrap32(np.sum((pa >> 8) * pb))
                    out[i, K + k] = wrap32(np.sum((pa & 255) * pb))
                else:
                    out[i, k] = wrap32(np.sum(pa * pb))
        elif mode == 7:
            pa, b0, b1, b2 = x[a:a + ln], x[b:b + ln], x[b + 1:b + 1 + ln], x[b + 2:b + 2 + ln]
            out[i, :9] = wrap32([np.sum(pa * pa), np.sum(b0 * b0), np.sum(pa * b0), np.sum(pa * b1),
                                 np.sum(pa * b2), np.sum(b1 * b2), np.sum(b1 * b1), np.sum(b2 * b2),
                                 np.sum(b0 * b1)])
        else:
            xa = (int(src[i, a]) & 0xffff) | (int(src[i, a + 1]) & 0xffff) << 16
            xb = (int(src[i, b]) & 0xffff) | (int(src[i, b + 1]) & 0xffff) << 16
            s = ln + int(x[a]) * int(x[b]) + int(x[a + 1]) * int(x[b + 1])
            hi8 = ((int(x[a]) >> 8) & 0xffff) | ((int(x[a + 1]) >> 8) & 0xffff) << 16
            v = xb | xa << 32
            sel = ln & 0x07070707
            perm = sum(((v >> (8 * ((sel >> (8 * k)) & 7))) & 0xff) << (8 * k) for k in range(4))
            out[i, :6] = wrap32([s, min(max(s, -2**31), 2**31 - 1), (xb >> 16) | (xa << 16) & 0xffffffff,
                                 hi8, xa & 0x00ff00ff, perm])
    return out


MODES = list(range(9))


@pytest.mark.parametrize("mode", MODES)
def test_helpers_hostemu(mode):
    lib = ctypes.CDLL(EMU)
    n = 96
    src, args = cases(mode, n, 11)
    out = np.zeros((n, HE_OUT), np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert lib.emu_helpers_eval(mode, p(src), p(args), p(out), n) == 0
    np.testing.assert_array_equal(out.astype(np.int64), want(mode, src, args))


@pytest.mark.gpu
def test_helpers_device():
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    n = 512
    for mode in MODES:
        src, args = cases(mode, n, 23)
        ds = torch.from_numpy(src).to(dev)
        da = torch.from_numpy(args).to(dev)
        do = torch.zeros((n, HE_OUT), dtype=torch.int32, device=dev)
        assert lib.melpe_helpers_eval_dev(mode, ds.data_ptr(), da.data_ptr(), do.data_ptr(), n, s) == 0
        got = do.cpu().numpy().astype(np.int64)
        np.testing.assert_array_equal(got, want(mode, src, args), err_msg="mode %d" % mode)
