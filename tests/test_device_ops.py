"""Device basic-op parity: the saturating operators as compiled for gfx950
(ops.h through engine.hip k_ops_eval, melpe_ops_eval_dev) against the
reference's own operators (melpe/mathhalf_i.h:120-2170, melpe/mathdp31.c:71,
compiled by oracle/Makefile into oracle/_ref/libref_ops.so, ref_ops_eval).

Domains: every int16 first operand against every shift in [-40, 40] (shifts)
or against 96 second operands covering the edges (two-operand 16-bit ops);
every int16 for the unary 16-bit ops; 2M edge-weighted random 32-bit and
40-bit cases for the others.  Saturation corners that speech rarely reaches
(L_sub(0, MIN32), L_mult(MIN16, MIN16), divide_s(x, x), 40-bit clamps) are
in the edge sets.  The op ids are pairphone_amd/csrc/ops_eval.h's.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import REF_DIR

OPS = ["add", "sub", "L_add", "L_sub", "L_mult", "extract_h", "extract_l", "mult", "L_mac",
       "L_msu", "r_ound", "msu_r", "negate", "L_negate", "abs_s", "L_abs", "shl", "shr",
       "L_shr", "L_shl", "shift_r", "L_shift_r", "norm_l", "norm_s", "divide_s", "L40_add",
       "L40_sub", "L40_mac", "L40_msu", "L40_shl", "L40_shr", "L40_negate", "norm32",
       "L_sat32", "L_mpy_ls"]
ID = {n: i for i, n in enumerate(OPS)}

E16 = np.array([0, 1, -1, 2, -2, 3, 7, 15, 16, 255, 256, 0x3fff, 0x4000, -0x4000, -0x4001,
                0x7ffe, 0x7fff, -0x7fff, -0x8000, 100, -100, 12345, -12345, 181, -182],
               np.int64)
E32 = np.array([0, 1, -1, 2, -2, 0x7fffffff, -0x80000000, 0x7ffffffe, -0x7fffffff,
                0x40000000, -0x40000000, 0x3fffffff, -0x40000001, 0x8000, 0x7fff, -0x8000,
                0xffff, 0x10000, 0x7fff8000, 0x7fff7fff, -0x7fff8000], np.int64)


def rng():
    return np.random.default_rng(20261016)


def r32(g, n):
    k = g.integers(0, 8, n)
    v = g.integers(-2**31, 2**31, n, dtype=np.int64)
    sh = g.integers(0, 32, n)
    v = np.where(k == 1, v >> sh, v)
    v = np.where(k == 0, E32[g.integers(0, len(E32), n)], v)
    return v


def r16(g, n):
    v = r32(g, n) >> g.integers(0, 2, n) * 16
    return ((v + 2**15) % 2**16 - 2**15).astype(np.int64)


def r40(g, n):
    v = g.integers(-2**39, 2**39 + 1, n, dtype=np.int64) >> g.integers(0, 40, n)
    edge = np.array([2**39, -2**39, 2**39 - 1, -2**39 + 1, 2**31, -2**31, 2**31 - 1,
                     -2**31 - 1, 2**30, -2**30, 1, -1, 0], np.int64)
    return np.where(g.integers(0, 8, n) == 0, edge[g.integers(0, len(edge), n)], v)


def all16():
    return np.arange(-32768, 32768, dtype=np.int64)


def second16(g):
    return np.unique(np.concatenate([E16, r16(g, 80)]))


def cases(name, g):
    """(a, b, c) int64/int32 arrays for op `name`"""
    N = 2_000_000
    if name in ("shl", "shr", "shift_r"):
        a, b = np.meshgrid(all16(), np.arange(-40, 41), indexing="ij")
        return a.ravel(), b.ravel(), None
    if name in ("L_shl", "L_shr", "L_shift_r", "L40_shl", "L40_shr"):
        base = r40(g, 30000) if name.startswith("L40") else r32(g, 30000)
        a, b = np.meshgrid(np.concatenate([base, E32]), np.arange(-45, 46), indexing="ij")
        return a.ravel(), b.ravel(), None
    if name in ("add", "sub", "mult", "L_mult", "divide_s"):
        a, b = np.meshgrid(all16(), second16(g), indexing="ij")
        a, b = a.ravel(), b.ravel()
        if name == "divide_s":   # the reference's domain: 0 <= num <= den
            a = np.concatenate([a, np.abs(b) // 3, np.abs(b)])
            b = np.concatenate([b, np.abs(b), np.abs(b)])
            # every denominator, with the numerators at the edges of the
            # quotient's correction (0, 1, den - 1, den, halves) and random
            # ones: the device's reciprocal-and-correct quotient (ops.h)
            d = np.arange(1, 32768, dtype=np.int64)
            nums = [np.zeros_like(d), np.minimum(1, d), d - 1, d, d // 2, (d + 1) // 2, d // 3]
            nums += [(g.random(len(d)) * d).astype(np.int64) for _ in range(32)]
            a = np.concatenate([a] + nums)
            b = np.concatenate([b] + [d] * len(nums))
        return a, b, None
    if name in ("negate", "abs_s", "norm_s"):
        return all16(), None, None
    if name in ("L_add", "L_sub"):
        a, b = r32(g, N), r32(g, N)
        a[:len(E32)] = 0
        b[:len(E32)] = E32
        return a, b, None
    if name in ("L_mac", "L_msu", "msu_r"):
        return r32(g, N), r16(g, N), r16(g, N)
    if name in ("L40_mac", "L40_msu"):
        return r40(g, N), r16(g, N), r16(g, N)
    if name in ("L40_add", "L40_sub"):
        return r40(g, N), r32(g, N), None
    if name in ("L40_negate", "norm32", "L_sat32"):
        return r40(g, N), None, None
    if name == "L_mpy_ls":
        return r32(g, N), r16(g, N), None
    return r32(g, N), None, None    # extract_h/l, r_ound, L_negate, L_abs, norm_l


def ref_eval(lib, op, a, b, c):
    n = len(a)
    out = np.zeros(n, np.int64)
    a = np.ascontiguousarray(a, np.int64)
    bb = None if b is None else np.ascontiguousarray(b, np.int32)
    cc = None if c is None else np.ascontiguousarray(c, np.int32)
    p = lambda x: None if x is None else x.ctypes.data_as(ctypes.c_void_p)
    assert lib.ref_ops_eval(op, p(a), p(bb), p(cc), p(out), ctypes.c_long(n)) == 0
    return out


@pytest.mark.gpu
def test_device_basic_ops_match_reference():
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    ref = ctypes.CDLL(os.path.join(REF_DIR, "libref_ops.so"))
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    g = rng()
    total = 0
    bad = []
    for name in OPS:
        a, b, c = cases(name, g)
        want = ref_eval(ref, ID[name], a, b, c)
        da = torch.from_numpy(np.ascontiguousarray(a, np.int64)).to(dev)
        db = None if b is None else torch.from_numpy(np.ascontiguousarray(b, np.int32)).to(dev)
        dc = None if c is None else torch.from_numpy(np.ascontiguousarray(c, np.int32)).to(dev)
        out = torch.empty(len(a), dtype=torch.int64, device=dev)
        rc = lib.melpe_ops_eval_dev(ID[name], da.data_ptr(), None if db is None else db.data_ptr(),
                                    None if dc is None else dc.data_ptr(), out.data_ptr(),
                                    len(a), s.cuda_stream)
        assert rc == 0, lib.melpe_last_error()
        got = out.cpu().numpy()
        total += len(a)
        if not np.array_equal(got, want):
            i = int(np.nonzero(got != want)[0][0])
            bad.append("%s(%d, %s, %s) = %d, reference %d" % (
                name, a[i], None if b is None else b[i], None if c is None else c[i],
                got[i], want[i]))
    assert not bad, "; ".join(bad)
    assert total > 30_000_000


def ref_divide_s_digests(ref):
    """for den = 1 .. 32,767: sum over num = 0 .. den of the reference's
    divide_s(num, den) * (num * 0x9E3779B97F4A7C15 + 1) mod 2^64, the
    reference evaluated over all ~537 M pairs in blocks of denominators"""
    out = np.zeros(32767, np.uint64)
    mul = np.uint64(0x9E3779B97F4A7C15)
    for d0 in range(1, 32768, 512):
        dens = np.arange(d0, min(d0 + 512, 32768), dtype=np.int64)
        cnt = dens + 1
        b = np.repeat(dens, cnt)
        start = np.repeat(np.cumsum(cnt) - cnt, cnt)
        a = np.arange(len(b), dtype=np.int64) - start
        q = ref_eval(ref, ID["divide_s"], a, b, None).astype(np.uint64)
        with np.errstate(over="ignore"):
            w = q * (a.astype(np.uint64) * mul + np.uint64(1))
        out[dens - 1] = np.add.reduceat(w, np.cumsum(cnt) - cnt)
    return out


@pytest.mark.gpu
def test_device_divide_s_exhaustive():
    """divide_s (device: float reciprocal + integer correction, ops.h) over
    its whole domain 0 <= num <= den < 2^15 against the reference's
    (melpe/mathhalf_i.h:175-190): one launch digests each denominator's
    quotients, the reference's quotients give the same digests"""
    import torch
    from pairphone_amd import load_library
    lib = load_library()
    ref = ctypes.CDLL(os.path.join(REF_DIR, "libref_ops.so"))
    dev = torch.device("cuda", 0)
    d = torch.zeros(32767, dtype=torch.int64, device=dev)
    assert lib.melpe_divide_s_sweep_dev(d.data_ptr(), torch.cuda.current_stream(dev).cuda_stream) == 0
    got = d.cpu().numpy().view(np.uint64)
    want = ref_divide_s_digests(ref)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, "divide_s differs for denominators %s" % (bad[:8] + 1)
