#!/usr/bin/env python3
"""GPU stage profile per quarter of the lane order (diagnostics): the
stage-timer build with -DMELPE_PROF_QUART adds each scope's wave-cycles to
slot k + 64 q, q the wave's quarter of the grid -- for the lane analysis
kernel, the quarter of the pitch-class order (light -> heavy classes).
Prints, per stage, the wave-cycles per wave and superframe in each quarter,
and the heavy-minus-light difference, largest first.

  MELPE_AMD_LIB=build/var/profq.so python tools/stage_prof_q.py [channels] [superframes]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main(C=262144, nsf=6):
    import torch
    import bench
    from pairphone_amd import MelpeEngine, load_library
    lib = load_library()
    names = open(os.path.join(ROOT, "pairphone_amd", "csrc", "prof_names.txt")).read().split()
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    s = torch.cuda.current_stream(dev).cuda_stream
    pcm = torch.empty((nsf + 2, C, 540), dtype=torch.int16, device=dev)
    bits = torch.empty((nsf + 2, C, 11), dtype=torch.uint8, device=dev)
    eng.synth_seed(bench.RUN_SEED)
    for k in range(nsf + 2):
        eng.synth_dev(pcm[k].data_ptr(), 540, s)
    for k in range(2):	# warm-up superframes: the lane order needs a history
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    buf = np.zeros(256, np.uint64)
    lib.melpe_prof_read(buf.ctypes.data, 256)
    for k in range(2, nsf + 2):
        eng.encode_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
    torch.cuda.synchronize()
    v = np.zeros(256, np.uint64)
    lib.melpe_prof_read(v.ctypes.data, 256)
    q = v.reshape(4, 64).astype(np.float64) / (C // 64 / 4) / nsf	# per wave, superframe
    print("encode: %d channels, %d superframes; wave-cycles per wave and superframe by quarter of "
          "the lane order (q0 light .. q3 heavy), inclusive" % (C, nsf))
    print("  %-20s %10s %10s %10s %10s %10s" % ("stage", "q0", "q1", "q2", "q3", "q3-q0"))
    for i in np.argsort(-(q[3] - q[0])):
        if i < len(names) and q[:, i].any():
            print("  %-20s %10.0f %10.0f %10.0f %10.0f %10.0f" % (names[i], *q[:, i], q[3, i] - q[0, i]))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
