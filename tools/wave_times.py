#!/usr/bin/env python3
"""Diagnostics: how the lane analysis launch's waves finish (k_ana.hip
MELPE_WAVE_TIMES build).  Runs the headline's encode step over a few
superframes and reads, for the last analysis launch, each wave's start and
end on the chip-wide 100 MHz counter: the distribution of end times against
the launch's span says how much of the launch runs with SIMDs already idle
(its tail).

  MELPE_AMD_LIB=build/var/wt.so python tools/wave_times.py [channels] [superframes]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(C=262144, nsf=6, dump=None):
    import torch
    import bench
    from pairphone_amd import MelpeEngine, load_library
    lib = load_library()
    lib.kl_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    eng = MelpeEngine(C)
    s = torch.cuda.current_stream(dev).cuda_stream
    pcm = torch.empty((nsf, C, 540), dtype=torch.int16, device=dev)
    bits = torch.empty((nsf, C, 11), dtype=torch.uint8, device=dev)
    eng.synth_seed(bench.RUN_SEED)
    for k in range(nsf):
        eng.synth_dev(pcm[k].data_ptr(), 540, s)
    out = []
    W = (C + 63) // 64
    for k in range(nsf):
        eng.encode_npp_dev(pcm[k].data_ptr(), None, s)
        eng.encode_ana_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
        torch.cuda.synchronize(dev)
        t = np.zeros(2 * W, np.uint64)
        lib.kl_wave_times(t.ctypes.data, 2 * W)
        st, en = t[0::2].astype(np.float64), t[1::2].astype(np.float64)
        t0 = st.min()
        span = (en.max() - t0) / 1e5           # ms (100 MHz)
        ends = (en - t0) / 1e5
        starts = (st - t0) / 1e5
        dur = ends - starts
        # busy wave-time / (span x waves): the fraction of the launch's
        # wave slots doing work
        util = float(dur.sum() / (span * W))
        out.append({"superframe": k, "span_ms": span,
                    "start_ms_max": float(starts.max()),
                    "end_ms_pct": {p: float(np.percentile(ends, p)) for p in (10, 25, 50, 75, 90, 99, 100)},
                    "wave_ms_mean": float(dur.mean()), "slot_utilisation": util})
        print(json.dumps(out[-1]), flush=True)
        if dump and k == nsf - 1:
            hw = np.zeros(2 * W, np.uint32)
            lib.kl_wave_hw.argtypes = [ctypes.c_void_p, ctypes.c_int]
            lib.kl_wave_hw(hw.ctypes.data, 2 * W)
            np.savez(dump, start=starts, end=ends, hwid=hw[0::2], xcc=hw[1::2])
    eng.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(int(a[0]) if a else 262144, int(a[1]) if len(a) > 1 else 6, a[2] if len(a) > 2 else None)
