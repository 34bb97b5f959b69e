#!/usr/bin/env python3
"""Lane vs four-wave analysis crossover (engine.hip ana_launch's live-count
threshold, melpe_engine_set_mw_live_max): a 65,536-channel engine under a
random activity mask with L live channels, the analysis launch timed with
each mapping forced (set_ana_waves 1 / 4), L in --live.  Each point is a
fresh engine: superframes 0..W-1 untimed, then K timed (HIP events on the
caller's stream around encode_ana_dev).  Prints one JSON line per point and
a summary line with the measured crossover.

  python tools/mw_crossover.py [--channels 65536] [--live 8192,16384,...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def point(C, live, waves, K, W, seed=7):
    import torch
    from pairphone_amd import MelpeEngine
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    eng = MelpeEngine(C)
    eng.set_ana_waves(waves)
    eng.synth_seed(2026)
    rng = np.random.default_rng(seed)
    m = np.zeros(C, np.uint8)
    m[rng.choice(C, live, replace=False)] = 1
    mask = torch.from_numpy(m).to(dev)
    pcm = torch.empty((W + K, C, 540), dtype=torch.int16, device=dev)
    bits = torch.empty((W + K, C, 11), dtype=torch.uint8, device=dev)
    for k in range(W + K):
        eng.synth_dev(pcm[k].data_ptr(), 540, s.cuda_stream)
    ms = []
    for k in range(W + K):
        eng.encode_npp_dev(pcm[k].data_ptr(), mask.data_ptr(), s.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.encode_ana_dev(bits[k].data_ptr(), pcm[k].data_ptr(), mask.data_ptr(), s.cuda_stream)
        b.record(s)
        ms.append((a, b))
    torch.cuda.synchronize(dev)
    t = [a.elapsed_time(b) for a, b in ms[W:]]
    ran = eng.last_ana_waves()
    eng.close()
    del pcm, bits
    torch.cuda.empty_cache()
    return float(np.mean(t)), ran


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=65536)
    ap.add_argument("--live", default="8192,16384,24576,32768,40960,49152")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    res = []
    for L in [int(x) for x in a.live.split(",")]:
        for w in (1, 4):
            ms, ran = point(a.channels, L, w, a.steps, a.warmup)
            r = {"channels": a.channels, "live": L, "waves": w, "ran": ran, "analysis_ms": ms}
            res.append(r)
            print(json.dumps(r), flush=True)
    # the largest live count at which the four-wave kernel is not slower
    best = max([r["live"] for r in res if r["waves"] == 4 and
                r["analysis_ms"] <= next(x["analysis_ms"] for x in res
                                         if x["waves"] == 1 and x["live"] == r["live"])] or [0])
    print(json.dumps({"crossover_live_max": best}), flush=True)


if __name__ == "__main__":
    main()
