"""diagnostic: first frame where the GPU 2400 decoder's DecState departs from
the host build's, on golden channel 0"""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_r2400 as t
from pairphone_amd import MelpeEngine
g = t.golden()
bits = np.frombuffer(bytes.fromhex(g["bits_hex"][0]), np.uint8).reshape(-1, 7)
lib = t.emu()
lib.emu_export.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.emu_state_bytes.restype = ctypes.c_long
d = lib.emu_create(1)
eng = MelpeEngine(1)
n = lib.emu_state_bytes(2)
assert n == eng.lib.melpe_engine_state_bytes(2), (n, eng.lib.melpe_engine_state_bytes(2))
for k in range(bits.shape[0]):
    b = np.ascontiguousarray(bits[k:k + 1])
    out = np.zeros((1, 180), np.int16)
    lib.emu_decode2400(d, out.ctypes.data, b.ctypes.data)
    got = eng.decode2400(b)
    hs = np.zeros(n, np.uint8)
    lib.emu_export(d, 2, 0, hs.ctypes.data)
    gs = eng.export_state(2)[0]
    if not np.array_equal(out, got) or not np.array_equal(hs, gs):
        diff = np.nonzero(hs != gs)[0]
        print("frame", k, "pcm equal", np.array_equal(out, got), "first pcm diff",
              np.nonzero(out[0] != got[0])[0][:5], "state byte diffs", diff[:40], len(diff))
        print("host", hs[diff[:20]], "gpu", gs[diff[:20]])
        break
else:
    print("no difference in", bits.shape[0], "frames")
