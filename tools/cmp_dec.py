"""Debug aid (CPU): host-emulated decoder vs the reference, superframe by
superframe.  Bitstream = reference encoding of a synth signal (default) or
uniformly random bytes (--random, exercises the FEC / erasure paths)."""
import ctypes, os, subprocess, sys, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.cmp_enc import TOOL, PAR_NAMES, emu_lib


def main(seed=1, ch=0, nsf=149, random_bits=False, quiet=False):
    tmp = tempfile.mkdtemp()
    if random_bits:
        bits = np.random.default_rng(seed * 1000 + ch).integers(0, 256, nsf * 11, dtype=np.uint8)
        bits.tofile(tmp + "/x.bits")
    else:
        subprocess.run([TOOL, "gen", str(seed), str(ch), str(nsf * 540), tmp + "/x.pcm"], check=True)
        subprocess.run([TOOL, "enc", tmp + "/x.pcm", tmp + "/x.bits"], check=True)
        bits = np.fromfile(tmp + "/x.bits", dtype=np.uint8)
    subprocess.run([TOOL, "dec", tmp + "/x.bits", tmp + "/y.pcm", tmp + "/y.dump"], check=True)
    ref = np.fromfile(tmp + "/y.pcm", dtype=np.int16).reshape(nsf, 540)
    rpar = np.fromfile(tmp + "/y.dump", dtype=np.int16).reshape(nsf, 90)
    lib = emu_lib()
    lib.emu_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_dec_params.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    e = lib.emu_create(1)
    bad = 0
    for k in range(nsf):
        b = bits[k * 11:(k + 1) * 11].copy()
        sp = np.zeros(540, np.int16)
        lib.emu_decode(e, sp.ctypes.data, b.ctypes.data)
        prm = np.zeros(90, np.int16)
        lib.emu_dec_params(e, 0, prm.ctypes.data)
        msgs = []
        if not np.array_equal(prm, rpar[k]):
            i = np.nonzero(prm != rpar[k])[0]
            msgs.append("par differs: " + ", ".join("f%d.%s emu %d ref %d" % (j // 30, PAR_NAMES[j % 30], prm[j], rpar[k][j]) for j in i[:6]))
        if not np.array_equal(sp, ref[k]):
            i = np.nonzero(sp != ref[k])[0]
            msgs.append("pcm differs at %d samples (first %d: emu %d ref %d)" % (i.size, i[0], sp[i[0]], ref[k][i[0]]))
        if msgs:
            bad += 1
            if not quiet:
                print("sf %d: %s" % (k, "; ".join(msgs)))
            if bad >= 3:
                break
    if not quiet or bad:
        print("seed %d ch %d random=%s: %s" % (seed, ch, random_bits, "OK" if not bad else "MISMATCH"))
    return bad == 0


if __name__ == "__main__":
    rnd = "--random" in sys.argv
    args = [int(a) for a in sys.argv[1:] if not a.startswith("--")]
    ok = main(*args, random_bits=rnd)
    sys.exit(0 if ok else 1)
