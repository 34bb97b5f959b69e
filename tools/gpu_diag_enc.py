"""Debug aid (GPU box): HIP engine vs the host build of the device sources,
superframe by superframe: NPP output and bitstream mismatches per channel."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pairphone_amd as pa
from test_encode import emu, signals

C, nsf = int(sys.argv[1]), int(sys.argv[2])
x = signals(1, C, nsf)
lib = emu()
e = lib.emu_create(C)
eng = pa.MelpeEngine(C)
for k in range(nsf):
    a = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
    b = a.copy()
    ba = np.zeros((C, 11), np.uint8)
    lib.emu_encode(e, ba.ctypes.data, a.ctypes.data)
    bb = eng.encode(b)
    npp_bad = [c for c in range(C) if not np.array_equal(a[c], b[c])]
    bit_bad = [c for c in range(C) if not np.array_equal(ba[c], bb[c])]
    print("sf %d: npp mismatch %d %s  bits mismatch %d %s" % (k, len(npp_bad), npp_bad[:4],
          len(bit_bad), bit_bad[:4]), flush=True)
    if npp_bad:
        c = npp_bad[0]
        i = np.nonzero(a[c] != b[c])[0]
        print("  ch %d first diff at %d: emu %s gpu %s" % (c, i[0], a[c][i[0]:i[0]+6], b[c][i[0]:i[0]+6]))
    if bit_bad:
        c = bit_bad[0]
        print("  ch %d emu %s gpu %s" % (c, ba[c].tobytes().hex(), bb[c].tobytes().hex()))
