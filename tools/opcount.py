"""Basic-op census W (ops per channel-superframe) for the roofline figure.

Runs the host count build of the device sources (build/libmelpe_opcount.so,
-DMELPE_OPCOUNT) over the benchmark's own synthetic input (bench.py RUN_SEED,
channels 0..N-1, 149 superframes each), counting every saturating basic op
entered from codec code and not from inside another op.
Encode = melpe_a (NPP x3 + analysis + packing), split as the GPU runs it:
W_enc_npp (k_enc_npp) and W_enc_ana (k_enc_ana); decode = melpe_s of the
resulting bitstreams (k_decode).  Writes profiles/opcount.json, which bench.py reads.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def vad_census(lib, x, nsf):
    """W of the TX VAD gate (six vad2 windows per superframe, vad.h) on the
    same input, same counting rule over the AMR basic ops"""
    lib.emu_vad_opcount.restype = ctypes.c_uint64
    C = x.shape[0]
    st = np.zeros(C * lib.emu_vad_state_bytes(), np.uint8)
    votes = np.zeros((C, nsf), np.uint8)
    x = np.ascontiguousarray(x, np.int16)
    lib.emu_vad_opcount()
    lib.emu_vad(ctypes.c_void_p(st.ctypes.data), ctypes.c_void_p(x.ctypes.data),
                ctypes.c_void_p(votes.ctypes.data), C, nsf)
    return {"W_vad_per_sf": float(lib.emu_vad_opcount()) / (C * nsf)}


def vad_only(channels=32, nsf=149):
    """refresh only W_vad_per_sf in profiles/opcount.json"""
    from pairphone_amd.build import build_opcount
    from pairphone_amd import synth_signal
    import bench
    lib = ctypes.CDLL(build_opcount())
    x = np.stack([synth_signal(bench.RUN_SEED, c, nsf * 540) for c in range(channels)])
    path = os.path.join(ROOT, "profiles", "opcount.json")
    res = json.load(open(path))
    res.update(vad_census(lib, x, nsf))
    json.dump(res, open(path, "w"), indent=1)
    print("W_vad %.0f ops/superframe" % res["W_vad_per_sf"])


def main(channels=32, nsf=149):
    from pairphone_amd.build import build_opcount
    from pairphone_amd import synth_signal
    import bench
    lib = ctypes.CDLL(build_opcount())
    lib.emu_create.restype = ctypes.c_void_p
    lib.emu_create.argtypes = [ctypes.c_int]
    for f in ("emu_encode", "emu_decode"):
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_opcount.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.emu_op_names.restype = ctypes.c_char_p
    assert lib.emu_load_tables(os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin").encode()) == 0
    names = lib.emu_op_names().decode().split()
    cnt = np.zeros(64, np.uint64)
    lib.emu_opcount(cnt.ctypes.data, 64)
    x = np.stack([synth_signal(bench.RUN_SEED, c, nsf * 540) for c in range(channels)])
    e = lib.emu_create(channels)
    enc = np.zeros(64, np.uint64)
    dec = np.zeros(64, np.uint64)
    lib.emu_encode_npp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_encode_ana.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    npp = np.zeros(64, np.uint64)
    by_sf = {"npp": [], "ana": [], "dec": []}
    for k in range(nsf):
        sp = np.ascontiguousarray(x[:, k * 540:(k + 1) * 540])
        b = np.zeros((channels, 11), np.uint8)
        lib.emu_encode_npp(e, sp.ctypes.data)
        lib.emu_opcount(cnt.ctypes.data, 64)
        npp += cnt
        enc += cnt
        by_sf["npp"].append(float(cnt.sum()) / channels)
        lib.emu_encode_ana(e, b.ctypes.data, sp.ctypes.data)
        lib.emu_opcount(cnt.ctypes.data, 64)
        enc += cnt
        by_sf["ana"].append(float(cnt.sum()) / channels)
        out = np.zeros((channels, 540), np.int16)
        lib.emu_decode(e, out.ctypes.data, b.ctypes.data)
        lib.emu_opcount(cnt.ctypes.data, 64)
        dec += cnt
        by_sf["dec"].append(float(cnt.sum()) / channels)
    n = channels * nsf
    res = {
        "rule": "saturating basic ops entered from codec code (nested op calls not counted), "
                "host count build of the device sources, SURVEY.md 8(d)",
        "input": "bench.py synthetic signal, run seed %d, channels 0..%d, %d superframes each"
                 % (bench.RUN_SEED, channels - 1, nsf),
        "channel_superframes": n,
        "W_enc_per_sf": float(enc.sum()) / n,
        "W_enc_npp_per_sf": float(npp.sum()) / n,
        "W_enc_ana_per_sf": float(enc.sum() - npp.sum()) / n,
        "W_dec_per_sf": float(dec.sum()) / n,
        "enc_by_op": {names[i]: float(enc[i]) / n for i in np.argsort(-enc.astype(np.float64))[:len(names)] if enc[i]},
        # per superframe index (mean over the channels): bench.py averages
        # these over exactly the superframes it times
        "W_enc_npp_by_sf": by_sf["npp"],
        "W_enc_ana_by_sf": by_sf["ana"],
        "W_dec_by_sf": by_sf["dec"],
        "dec_by_op": {names[i]: float(dec[i]) / n for i in np.argsort(-dec.astype(np.float64))[:len(names)] if dec[i]},
    }
    res.update(vad_census(lib, x, nsf))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "profiles", "opcount.json"), "w"), indent=1)
    print("W_enc %.0f  W_dec %.0f ops/superframe" % (res["W_enc_per_sf"], res["W_dec_per_sf"]))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--vad"]:
        vad_only(*[int(a) for a in sys.argv[2:]])
    else:
        main(*[int(a) for a in sys.argv[1:]])
