"""GPU stage profile (diagnostics): runs the stage-timer build
(libmelpe_amd_prof.so) over the bench input and prints, per instrumented
function, the wave-cycles it took per superframe (inclusive of callees),
as a share of encode_superframe / decode_superframe.

  python tools/stage_prof.py [channels] [superframes] [same]

same=1 gives every channel synthetic channel 0's signal (no divergence
inside a wave), so a stage's share against the default run prices the
divergence of its channels.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MELPE_AMD_LIB", os.path.join(ROOT, "pairphone_amd", "libmelpe_amd_prof.so"))

import numpy as np  # noqa: E402


def main(C=65536, nsf=4, same=0):
    import torch
    import bench
    from pairphone_amd import MelpeEngine, load_library
    lib = load_library()
    names = open(os.path.join(ROOT, "pairphone_amd", "csrc", "prof_names.txt")).read().split()
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    s = torch.cuda.current_stream(dev).cuda_stream
    pcm = torch.empty((nsf, C, 540), dtype=torch.int16, device=dev)
    bits = torch.empty((nsf, C, 11), dtype=torch.uint8, device=dev)
    out = torch.empty((nsf, C, 540), dtype=torch.int16, device=dev)
    eng.synth_seed(bench.RUN_SEED)
    for k in range(nsf):
        eng.synth_dev(pcm[k].data_ptr(), 540, s)
    if same:
        pcm[:] = pcm[:, :1, :]
    buf = np.zeros(64, np.uint64)
    lib.melpe_prof_read(buf.ctypes.data, 64)
    for k in range(nsf):
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    enc = np.zeros(64, np.uint64)
    lib.melpe_prof_read(enc.ctypes.data, 64)
    for k in range(nsf):
        eng.decode_dev(out[k].data_ptr(), bits[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    dec = np.zeros(64, np.uint64)
    lib.melpe_prof_read(dec.ctypes.data, 64)
    waves = C // 64
    for title, v, tot in (("encode", enc, ("npp_frame", "analysis")),
                          ("decode", dec, ("decode_superframe",))):
        t = float(sum(v[names.index(n)] for n in tot))
        print("%s: %d channels, %d superframes%s; wave-cycles per superframe, inclusive"
              % (title, C, nsf, ", every channel channel 0's signal" if same else ""))
        for i in np.argsort(-v.astype(np.float64)):
            if i < len(names) and v[i]:
                print("  %-20s %12.0f  %5.1f%%" % (names[i], v[i] / waves / nsf, 100 * v[i] / t))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
