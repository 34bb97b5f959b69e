#!/usr/bin/env python3
"""Config-3 round trip with the decode of superframe k - 1 beside the encode
of superframe k (experiment).  Modes:
  one: one engine, pipelined encode then decode per step (bench.py round_trip)
  two: an encoder engine and a decoder engine, each on its own stream
       (melpe_engine_set_own_stream); caller stream A runs the pipelined
       encode of k, stream B the decode of k - 1 once A recorded its bits
Prints one JSON line per mode: ms per step over K timed steps, and whether
bits and PCM equal mode `one`'s.
  python tools/rt_overlap_exp.py [channels] [K] [W]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pairphone_amd import MelpeEngine  # noqa: E402

SF_SAMPLES, SF_BYTES, RUN_SEED = 540, 11, 2026


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    N = W + K + 1
    ref = None
    for mode in sys.argv[4:] or ["one", "two", "one", "two"]:
        enc = MelpeEngine(C, device=0)
        dec = enc if mode == "one" else MelpeEngine(C, device=0)
        if mode != "one":
            enc.set_own_stream(True)
            dec.set_own_stream(True)
        pcm = torch.empty((N, C, SF_SAMPLES), dtype=torch.int16, device=dev)
        out = torch.empty((N, C, SF_SAMPLES), dtype=torch.int16, device=dev)
        bits = torch.zeros((N, C, SF_BYTES), dtype=torch.uint8, device=dev)
        sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        enc.synth_seed(RUN_SEED, first_channel=0)
        for s in range(N):
            enc.synth_dev(pcm[s].data_ptr(), SF_SAMPLES, sa.cuda_stream)
        torch.cuda.synchronize()
        evs = [torch.cuda.Event() for _ in range(N)]

        def step(s, nxt):
            enc.encode_pipe_dev(bits[s].data_ptr(), pcm[s].data_ptr(),
                                None if nxt is None else pcm[nxt].data_ptr(), stream=sa.cuda_stream)
            if mode == "one":
                dec.decode_dev(out[s].data_ptr(), bits[s].data_ptr(), None, sa.cuda_stream)
                return
            evs[s].record(sa)
            if s > 0:
                sb.wait_event(evs[s - 1])
                dec.decode_dev(out[s - 1].data_ptr(), bits[s - 1].data_ptr(), None, sb.cuda_stream)

        enc.encode_npp_dev(pcm[0].data_ptr(), None, sa.cuda_stream)
        for s in range(W):
            step(s, s + 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(W, W + K):
            step(s, s + 1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if mode != "one":	# the last superframe's decode, outside the timing
            sb.wait_event(evs[W + K - 1])
            dec.decode_dev(out[W + K - 1].data_ptr(), bits[W + K - 1].data_ptr(), None, sb.cuda_stream)
            torch.cuda.synchronize()
        b, o = bits[:W + K].cpu(), out[:W + K].cpu()
        if ref is None and mode == "one":
            ref = (b, o)
        same = None if ref is None else bool(torch.equal(ref[0], b) and torch.equal(ref[1], o))
        print(json.dumps({"mode": mode, "channels": C, "steps": K, "ms_per_step": 1e3 * dt / K,
                          "channel_s_per_s": C * K * 0.0675 / dt, "equal_to_one": same}), flush=True)
        enc.close()
        if dec is not enc:
            dec.close()
        del pcm, out, bits
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
