#!/usr/bin/env python3
"""Diagnostics: the encode step serialised (melpe_encode_npp_dev then
melpe_encode_ana_dev, the bench's encode leg) against the pipelined form
(melpe_encode_pipe_dev: superframe k's analysis beside superframe k+1's NPP
on the engine's second stream), same channels and input, wall-clock per
step; and whether the bits agree.

  python tools/pipe_exp.py [channels] [steps] [warmup]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(C=262144, K=10, W=2):
    import torch
    import bench
    from pairphone_amd import MelpeEngine
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    bits = {}
    for mode in ("serial", "pipe", "serial2", "pipe2"):
        eng = MelpeEngine(C)
        n = W + K
        pcm = torch.empty((n, C, 540), dtype=torch.int16, device=dev)
        b = torch.zeros((n, C, 11), dtype=torch.uint8, device=dev)
        eng.synth_seed(bench.RUN_SEED)
        for k in range(n):
            eng.synth_dev(pcm[k].data_ptr(), 540, s)
        torch.cuda.synchronize(dev)

        def serial(k):
            eng.encode_npp_dev(pcm[k].data_ptr(), None, s)
            eng.encode_ana_dev(b[k].data_ptr(), pcm[k].data_ptr(), None, s)
        if mode.startswith("serial"):
            for k in range(W):
                serial(k)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for k in range(W, n):
                serial(k)
            torch.cuda.synchronize(dev)
        else:
            for k in range(W):
                serial(k)
            torch.cuda.synchronize(dev)
            # the timed region holds the same K NPPs and K analyses
            t0 = time.perf_counter()
            eng.encode_npp_dev(pcm[W].data_ptr(), None, s)
            for k in range(W, n):
                nxt = pcm[k + 1].data_ptr() if k + 1 < n else None
                eng.encode_pipe_dev(b[k].data_ptr(), pcm[k].data_ptr(), nxt, stream=s)
            torch.cuda.synchronize(dev)
        res[mode] = 1e3 * (time.perf_counter() - t0) / K
        bits[mode] = b.cpu()
        eng.close()
        del pcm, b
    res["bits_equal"] = bool(torch.equal(bits["serial"], bits["pipe"]))
    res["channels"] = C
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*(int(x) for x in a))
