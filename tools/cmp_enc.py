"""Debug aid (CPU): host-emulated encoder vs the reference, superframe by
superframe, reporting the first differing stage (NPP output, melp_par,
quant_par, bitstream)."""
import ctypes, os, subprocess, sys, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_tool")
EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")

PAR_NAMES = ["pitch"] + ["lsf%d" % i for i in range(10)] + ["gain0", "gain1", "jitter"] + \
    ["bpvc%d" % i for i in range(5)] + ["uv"] + ["fsmag%d" % i for i in range(10)]
Q_NAMES = ["pitch_index"] + ["lsf_index%d%d" % (i, j) for i in range(3) for j in range(4)] + \
    ["gain_index0", "gain_index1", "jit0", "jit1", "jit2", "bpvc0", "bpvc1", "bpvc2", "fs_index",
     "uv0", "uv1", "uv2", "msvq0", "msvq1", "msvq2", "msvq3", "fsvq"]


def emu_lib():
    lib = ctypes.CDLL(EMU)
    lib.emu_create.restype = ctypes.c_void_p
    lib.emu_create.argtypes = [ctypes.c_int]
    lib.emu_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.emu_enc_params.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    assert lib.emu_load_tables(os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin").encode()) == 0
    return lib


def main(seed=1, ch=0, nsf=149, pcm=None):
    tmp = tempfile.mkdtemp()
    if pcm is None:
        n = nsf * 540
        subprocess.run([TOOL, "gen", str(seed), str(ch), str(n), tmp + "/x.pcm"], check=True)
        x = np.fromfile(tmp + "/x.pcm", dtype=np.int16)
    else:
        x = np.fromfile(pcm, dtype=np.int16)
        nsf = (x.size + 539) // 540
        x = np.concatenate([x, np.zeros(nsf * 540 - x.size, np.int16)])
        x.tofile(tmp + "/x.pcm")
    subprocess.run([TOOL, "enc", tmp + "/x.pcm", tmp + "/x.bits", tmp + "/x.dump"], check=True)
    rec = 180 + 60 + 12 + 1080
    dump = np.fromfile(tmp + "/x.dump", dtype=np.uint8).reshape(-1, rec)
    lib = emu_lib()
    e = lib.emu_create(1)
    bad = 0
    for k in range(nsf):
        sp = x[k * 540:(k + 1) * 540].copy()
        bits = np.zeros(11, np.uint8)
        lib.emu_encode(e, bits.ctypes.data, sp.ctypes.data)
        prm = np.zeros(120, np.int16)
        lib.emu_enc_params(e, 0, prm.ctypes.data)
        d = dump[k]
        rpar = d[:180].view(np.int16)
        rq = d[180:240].view(np.int16)
        rbits = d[240:251]
        rsp = d[252:].view(np.int16)
        msgs = []
        if not np.array_equal(sp, rsp):
            i = np.nonzero(sp != rsp)[0]
            msgs.append("NPP out differs at %d samples (first %d: emu %d ref %d)" % (i.size, i[0], sp[i[0]], rsp[i[0]]))
        if not np.array_equal(prm[:90], rpar):
            i = np.nonzero(prm[:90] != rpar)[0]
            msgs.append("melp_par: " + ", ".join("f%d.%s emu %d ref %d" % (j // 30, PAR_NAMES[j % 30], prm[j], rpar[j]) for j in i[:8]))
        if not np.array_equal(prm[90:120], rq):
            i = np.nonzero(prm[90:120] != rq)[0]
            msgs.append("quant_par: " + ", ".join("%s emu %d ref %d" % (Q_NAMES[j], prm[90 + j], rq[j]) for j in i[:8]))
        if not np.array_equal(bits, rbits):
            msgs.append("bits differ")
        if msgs:
            print("superframe %d:" % k)
            for m in msgs:
                print("   ", m)
            bad += 1
            if bad >= 3:
                break
    print("done: %d/%d superframes checked, %s" % (k + 1, nsf, "MISMATCH" if bad else "all match"))


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "--pcm":
        main(pcm=a[1])
    else:
        main(*(int(v) for v in a))
