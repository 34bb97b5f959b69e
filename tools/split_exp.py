#!/usr/bin/env python3
"""Diagnostic: the encode step of C channels as S engines of C/S channels,
each on its own HIP stream, launched interleaved, so the NPP kernel of one
engine can share the GPU with the analysis kernels of another (the two are
bound by different things: VALU/SALU/LDS vs scratch latency).

  python tools/split_exp.py [C] [S...]      e.g. 262144 1 2 4
Prints ms per step for each S (same input: the bench's synthetic PCM).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(C, S, K=8, W=2):
    import torch
    import bench
    from pairphone_amd import MelpeEngine
    dev = torch.device("cuda", 0)
    n = C // S
    engs = [MelpeEngine(n) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    pcm = torch.empty((W + K, C, 540), dtype=torch.int16, device=dev)
    bits = torch.zeros((W + K, C, 11), dtype=torch.uint8, device=dev)
    s0 = torch.cuda.current_stream(dev).cuda_stream
    for i, e in enumerate(engs):
        e.synth_seed(bench.RUN_SEED, first_channel=i * n)
        for k in range(W + K):
            e.synth_dev(pcm[k, i * n:(i + 1) * n].data_ptr(), 540, s0)
    torch.cuda.synchronize(dev)

    def step(k):
        for i, (e, st) in enumerate(zip(engs, streams)):
            e.encode_npp_dev(pcm[k, i * n:(i + 1) * n].data_ptr(), None, st.cuda_stream)
            e.encode_ana_dev(bits[k, i * n:(i + 1) * n].data_ptr(), pcm[k, i * n:(i + 1) * n].data_ptr(),
                             None, st.cuda_stream)
    for k in range(W):
        step(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(W, W + K):
        step(k)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / K
    out = bits[W:].cpu().numpy()
    for e in engs:
        e.close()
    return dt * 1e3, out


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    Ss = [int(a) for a in sys.argv[2:]] or [1, 2]
    ref = None
    for S in Ss:
        ms, b = run(C, S)
        same = "" if ref is None else (" bits %s" % ("same" if (b == ref).all() else "DIFFER"))
        ref = b if ref is None else ref
        print("C %d  S %d: %.2f ms/step  %.0f channel-s/s%s" % (C, S, ms, C * 0.0675 / (ms / 1e3), same),
              flush=True)


if __name__ == "__main__":
    main()
