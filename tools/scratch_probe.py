#!/usr/bin/env python3
"""Diagnostic: how the HIP runtime holds the codec kernels' scratch.
Prints the device's scratch limits (hipExtLimitScratchMin/Max/Current) and
the time of single synchronised encode steps on a fresh engine -- lane
mapping, then the four-wave mapping, then the lane mapping again -- so a
per-dispatch scratch (re)allocation shows as wall time far above the
kernels' own.

  python tools/scratch_probe.py [channels]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def limits(hip):
    out = {}
    for name, k in (("min", 0x1000), ("max", 0x1001), ("current", 0x1002)):
        v = ctypes.c_size_t(0)
        rc = hip.hipDeviceGetLimit(ctypes.byref(v), k)
        out[name] = (rc, v.value / 2**30)
    return out


def main(C=65536):
    import torch
    from pairphone_amd import MelpeEngine
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize(dev)
    print("limits before (rc, GiB):", limits(hip), flush=True)
    eng = MelpeEngine(C)
    print("limits after create:", limits(hip), flush=True)
    s = torch.cuda.current_stream(dev).cuda_stream
    pcm = torch.zeros((C, 540), dtype=torch.int16, device=dev)
    bits = torch.zeros((C, 11), dtype=torch.uint8, device=dev)
    eng.synth_seed(1)
    for waves in (1, 4, 1, 4):
        eng.set_ana_waves(waves)
        ts = []
        for k in range(4):
            eng.synth_dev(pcm.data_ptr(), 540, s)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            eng.encode_dev(bits.data_ptr(), pcm.data_ptr(), None, s)
            torch.cuda.synchronize(dev)
            ts.append(1e3 * (time.perf_counter() - t0))
        print("waves %d: encode step ms %s" % (waves, " ".join("%.1f" % t for t in ts)), flush=True)
    eng.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
