"""Phase profile of the multi-wave analysis kernel (diagnostics): runs the
stage-timer build (libmelpe_amd_prof.so) with MELPE_ANA_NW waves per 64
channels and prints, per phase, the wall time wave 0 saw (barrier
included) and each virtual wave's busy time, in wave-cycles per workgroup
per superframe (k_ana.hip MW_SLOT).

  MELPE_ANA_NW=4 python tools/mw_prof.py [channels] [superframes]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MELPE_AMD_LIB", os.path.join(ROOT, "pairphone_amd", "libmelpe_amd_prof.so"))

import numpy as np  # noqa: E402

LQ_SLOTS = 7
PHASES = (["frame 0", "frame 1", "frame 2", "lsf prelude+step 0|bands2"]
          + [n % k for k in range(1, LQ_SLOTS) for n in ("lsf compute %d", "lsf scan %d")]
          + ["sc_ana+pvq prelude", "pvq slices", "pvq finish..", "find_harm", "pack"])


def main(C=32768, nsf=4):
    import torch
    import bench
    from pairphone_amd import MelpeEngine, load_library
    lib = load_library()
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    s = torch.cuda.current_stream(dev).cuda_stream
    pcm = torch.empty((nsf + 2, C, 540), dtype=torch.int16, device=dev)
    bits = torch.empty((nsf + 2, C, 11), dtype=torch.uint8, device=dev)
    eng.synth_seed(bench.RUN_SEED)
    for k in range(nsf + 2):
        eng.synth_dev(pcm[k].data_ptr(), 540, s)
    for k in range(2):     # warm up past the first superframes
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    buf = np.zeros(256, np.uint64)
    lib.melpe_prof_read(buf.ctypes.data, 256)
    for k in range(2, nsf + 2):
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    v = np.zeros(256, np.uint64)
    lib.melpe_prof_read(v.ctypes.data, 256)
    wg = C // 64 * nsf
    nw = int(os.environ.get("MELPE_ANA_NW", "0"))
    print("k_enc_ana_mw, %d channels, MELPE_ANA_NW=%d, cycles per workgroup per superframe" % (C, nw))
    print("  %-16s %10s %10s %10s %10s %10s" % ("phase", "wall(w0)", "v0", "v1", "v2", "v3"))
    tot = 0
    for p, name in enumerate(PHASES):
        row = [v[64 + 5 * p + k] / wg for k in range(5)]
        tot += row[4]
        print("  %-16s %10.0f %10.0f %10.0f %10.0f %10.0f" % (name, row[4], *row[:4]))
    nwv = max(nw, 1)
    print("  copy-in per wave %.0f, dc_rmv per wave %.0f, write-back per wave %.0f, sum of phase "
          "walls %.0f" % (v[64 + 5 * len(PHASES)] / wg / nwv, v[64 + 5 * len(PHASES) + 2] / wg / nwv,
                          v[64 + 5 * len(PHASES) + 1] / wg / nwv, tot))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
