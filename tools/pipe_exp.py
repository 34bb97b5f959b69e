"""Superframe pipeline experiment (diagnostics): NPP of superframe s+1 on a
second stream beside the analysis of superframe s, against the sequential
NPP -> analysis step, on the product library (or MELPE_AMD_LIB).

    python tools/pipe_exp.py [channels] [steps]

Prints one JSON line: sequential and pipelined ms per superframe step, and
whether the pipelined bitstreams equal the sequential ones.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairphone_amd import MelpeEngine  # noqa: E402

SF, NB = 540, 11


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev)
    out = {"channels": C, "steps": K}
    bits = {}
    for mode in ("seq", "pipe"):
        eng = MelpeEngine(C, device=0)
        pcm = torch.empty((K + 1, C, SF), dtype=torch.int16, device=dev)
        b = torch.zeros((K + 1, C, NB), dtype=torch.uint8, device=dev)
        eng.synth_seed(2026, first_channel=0)
        for s in range(K + 1):
            eng.synth_dev(pcm[s].data_ptr(), SF, s1.cuda_stream)
        # superframe 0 outside the timed region
        eng.encode_npp_dev(pcm[0].data_ptr(), None, s1.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "seq":
            for s in range(K):
                eng.encode_ana_dev(b[s].data_ptr(), pcm[s].data_ptr(), None, s1.cuda_stream)
                eng.encode_npp_dev(pcm[s + 1].data_ptr(), None, s1.cuda_stream)
        else:
            ev = [torch.cuda.Event() for _ in range(K + 1)]
            ev[0].record(s1)
            s2.wait_event(ev[0])
            for s in range(K):
                eng.encode_npp_dev(pcm[s + 1].data_ptr(), None, s2.cuda_stream)
                ev[s + 1].record(s2)
                eng.encode_ana_dev(b[s].data_ptr(), pcm[s].data_ptr(), None, s1.cuda_stream)
                s1.wait_event(ev[s + 1])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[mode + "_ms_per_step"] = 1e3 * dt / K
        bits[mode] = b[:K].cpu()
        eng.close()
        del pcm, b
        torch.cuda.empty_cache()
    out["bit_exact"] = bool(torch.equal(bits["seq"], bits["pipe"]))
    out["lib"] = os.environ.get("MELPE_AMD_LIB", "product")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
