#!/usr/bin/env python3
"""Diagnostics: per-wave durations of the lane analysis launch against the
wave's place in the lane order (its content: the order runs from the lightest
pitch classes to the heaviest) and against its placement (HW_ID / XCC_ID:
which SIMD it shares with which waves), from tools/wave_times.py's npz dump.

  python tools/wave_place.py gpurun_out/r06m/wt_262k.npz
"""
import sys

import numpy as np


def main(path):
    d = np.load(path)
    st, en, hw, xcc = d["start"], d["end"], d["hwid"], d["xcc"]
    W = len(en)
    dur = en - st
    simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 0xF, (hw >> 13) & 7
    x = (xcc & 0xF).astype(np.int64)
    print("waves %d, span %.2f ms, mean wave %.2f ms" % (W, en.max(), dur.mean()))
    print("XCC of waves 0..15:", " ".join(str(v) for v in x[:16]))
    nch = 32
    ch = dur[: W // nch * nch].reshape(nch, -1)
    print("wave duration by 1/%d of the lane order (light -> heavy classes), ms:" % nch)
    print("  mean:", " ".join("%.1f" % v for v in ch.mean(1)))
    print("  max: ", " ".join("%.1f" % v for v in ch.max(1)))
    sid = (x * 8 + se) * 64 + cu * 4 + simd
    u, inv, cnt = np.unique(sid, return_inverse=True, return_counts=True)
    print("SIMDs %d, waves per SIMD %s" % (len(u), dict(zip(*[a.tolist() for a in np.unique(cnt, return_counts=True)]))))
    mx = np.zeros(len(u))
    mn = np.full(len(u), 1e30)
    np.maximum.at(mx, inv, en)
    np.minimum.at(mn, inv, en)
    q = (4 * np.arange(W)) // W
    qs = np.zeros((len(u), 4), np.int64)
    np.add.at(qs, (inv, q), 1)
    print("SIMD's last wave end, percentiles 0/10/50/90/100: %s ms" %
          " ".join("%.2f" % v for v in np.percentile(mx, [0, 10, 50, 90, 100])))
    print("spread of end times inside a SIMD, p10/p50/p90: %s ms" %
          " ".join("%.2f" % v for v in np.percentile(mx - mn, [10, 50, 90])))
    print("SIMDs holding one wave of each quarter of the order: %d of %d" % (int((qs == 1).all(1).sum()), len(u)))


if __name__ == "__main__":
    main(sys.argv[1])
