"""Lane-divergence bound (diagnostics): k_enc_ana / k_decode time when every
channel carries the same signal (no divergence within a wave) against the
default per-channel signals, with the pitch-class lane order on and off.

    python tools/diverge_exp.py [channels] [steps]

"same:<c>" broadcasts synthetic channel c to every channel.  Prints one JSON
line of mean analysis / decode kernel ms over the steps after the first.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairphone_amd import MelpeEngine  # noqa: E402

SF, NB = 540, 11


def run(C, K, src, order):
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    eng = MelpeEngine(C, device=0)
    eng.set_lane_order(order)
    pcm = torch.empty((K, C, SF), dtype=torch.int16, device=dev)
    eng.synth_seed(2026, first_channel=0 if src is None else src)
    for k in range(K):
        eng.synth_dev(pcm[k].data_ptr(), SF, s)
    if src is not None:
        pcm[:] = pcm[:, :1, :]
    bits = torch.zeros((K, C, NB), dtype=torch.uint8, device=dev)
    out = torch.empty_like(pcm)
    ta, td = [], []
    for k in range(K):
        e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        eng.encode_npp_dev(pcm[k].data_ptr(), None, s)
        e0.record()
        eng.encode_ana_dev(bits[k].data_ptr(), pcm[k].data_ptr(), None, s)
        e1.record()
        e2.record()
        eng.decode_dev(out[k].data_ptr(), bits[k].data_ptr(), None, s)
        e3.record()
        torch.cuda.synchronize()
        ta.append(e0.elapsed_time(e1))
        td.append(e2.elapsed_time(e3))
    eng.close()
    return sum(ta[1:]) / (K - 1), sum(td[1:]) / (K - 1)


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    torch.cuda.set_device(0)
    res = {"channels": C, "steps": K}
    for order in (False, True):
        for src in (None, 0, 1, 2, 3):
            a, d = run(C, K, src, order)
            key = "%s/%s" % ("random" if src is None else "same:%d" % src, "order" if order else "ident")
            res[key] = {"ana_ms": round(a, 2), "dec_ms": round(d, 2)}
            print(key, res[key], file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
