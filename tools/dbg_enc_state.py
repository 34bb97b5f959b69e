"""Debug aid (GPU box): the first superframe where the GPU encoder's
EncState departs from the host build's, with the differing fields
(tools/enc_fields.json: offsets from state.h)."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pairphone_amd import MelpeEngine
from test_encode import emu, signals

C, nsf = int(sys.argv[1]), int(sys.argv[2])
fields = json.load(open(os.path.join(ROOT, "tools", "enc_fields.json")))
x = signals(1, C, nsf)
lib = emu()
lib.emu_export.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.emu_state_bytes.restype = ctypes.c_long
e = lib.emu_create(C)
eng = MelpeEngine(C)
n = lib.emu_state_bytes(1)
assert n == fields["_size"][0], (n, fields["_size"])


def field(off):
    for k, (o, s) in fields.items():
        if o <= off < o + s:
            return "%s+%d" % (k, off - o)
    return "?%d" % off


for k in range(nsf):
    a = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
    b = a.copy()
    ba = np.zeros((C, 11), np.uint8)
    lib.emu_encode(e, ba.ctypes.data, a.ctypes.data)
    eng.encode(b)
    gs = eng.export_state(1)
    bad = 0
    for c in range(C):
        hs = np.zeros(n, np.uint8)
        lib.emu_export(e, 1, c, hs.ctypes.data)
        d = np.nonzero(hs != gs[c])[0]
        if len(d):
            bad += 1
            if bad <= 3:
                names = []
                for off in d:
                    f = field(int(off)).split("+")[0]
                    if f not in names:
                        names.append(f)
                print("sf %d ch %d: %d bytes differ; fields %s; first %s" % (k, c, len(d), names[:12],
                      [field(int(o)) for o in d[:6]]), flush=True)
    print("sf %d: %d/%d channels differ" % (k, bad, C), flush=True)
    if bad:
        break
