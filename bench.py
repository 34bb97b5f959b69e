#!/usr/bin/env python3
"""Benchmark: MELPe-1200 channel-seconds encoded per second on MI355X.

Workload (BASELINE.json config 4 at N=1): 262,144 independent 8 kHz channels
per GPU, each step = one melpe_a superframe (540 samples -> 81 bits) of every
channel, i.e. 262,144 x 67.5 ms = 17,694 channel-seconds of audio per GPU per
step.  Channels are sharded statically across ranks (rank r owns channels
[r*C, (r+1)*C)) with no collective on the data path: weak scaling.

Inputs: the integer speech-like generator (pairphone_amd/csrc/synth.h) run on
the device before the timed region, so every step's PCM is resident in HBM;
bitstreams stay on the device.  The decode leg (melpe_s of the bits just
produced) is timed the same way and reported beside the headline.

A step is two kernels on one stream: k_enc_npp (noise pre-processor, one
wavefront per channel) then k_enc_ana (analysis + packing, one lane per
channel); both are timed with HIP events around each launch.

Roofline: the codec is bit-exact saturating int16/int32 arithmetic with
serial recursions per channel, so it is bounded by INT VALU issue, not HBM
and not MFMA.  For the dominant kernel (k_enc_ana) achieved =
W_ana (the reference's basic ops per channel-superframe of the analysis,
profiles/opcount.json, counted by tools/opcount.py on this same input) x
channels / its average launch duration; peak = 256 CUs x 4 SIMDs x 32
lanes/clk x 2.4 GHz = 78.6 T lane-ops/s.  traffic = HBM bytes per launch
from the committed rocprofv3 --pmc passes at this channel count.

cpu_baseline: the reference codec itself (oracle/_ref/ref_tool, compiled
from /root/reference by oracle/Makefile), one process per core on a bounded
sample of the same channels; its bitstreams double as a parity spot check of
the timed GPU output.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RUN_SEED = 2026
SF_SAMPLES = 540
SF_BYTES = 11
SF_SECONDS = SF_SAMPLES / 8000.0
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12     # INT32 lane-ops/s, T
# Keccak-f[1600] per voice packet, 64-bit ops counted as two 32-bit lane-ops:
# per round theta 55 (25 xor parity, 5 rot + 5 xor D, 25 xor apply), rho+pi
# 24 rot, chi 75 (not, and, xor per lane), iota 1 = 155 64-bit ops; x 24 rounds
VC_OPS_PER_PACKET = 2 * 155 * 24
REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_tool")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--channels", type=int, default=262144, help="channels per GPU")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-channels", type=int, default=128)
    ap.add_argument("--cpu-jobs", type=int, default=0, help="0 = min(16, usable cores)")
    return ap.parse_args()


def opcount():
    p = os.path.join(ROOT, "profiles", "opcount.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p))


def pmc_traffic(kernel, channels):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc
    passes (profiles/pmc_latest.json, written by tools/prof_summary.py), if
    they were taken at this channel count; else None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p))
    if d.get("channels") != channels:
        return None
    k = d.get("kernels", {}).get(kernel)
    return None if k is None else k["bytes_per_launch"]


def cpu_baseline(args, gpu_bits):
    """Reference codec, one process per core, on channels 0..S-1 of the same
    synthetic input.  Returns (baseline dict, parity dict)."""
    if args.no_cpu_baseline or not os.path.exists(REF_TOOL):
        return None, None
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    jobs = args.cpu_jobs or min(16, usable)
    S = args.cpu_sample_channels
    nsf = max(149, gpu_bits.shape[0])
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "b.bits")
        t0 = time.perf_counter()
        subprocess.run([REF_TOOL, "jobs", str(jobs), "encgen", str(RUN_SEED), "0", str(S),
                        str(nsf), out], check=True)
        dt = time.perf_counter() - t0
        ref = np.fromfile(out, dtype=np.uint8).reshape(S, nsf * SF_BYTES)
    base = {"value": S * nsf * SF_SECONDS / dt, "unit": "channel-s/s", "cores": jobs,
            "kind": "reference",
            "sample": "%d channels x %d superframes (%.1f s of audio each), melpe_a, "
                      "one forked reference process per channel, %d at a time, %.1f s wall"
                      % (S, nsf, nsf * SF_SECONDS, jobs, dt)}
    n = min(S, gpu_bits.shape[1])
    k = gpu_bits.shape[0]
    g = np.ascontiguousarray(gpu_bits[:, :n, :].transpose(1, 0, 2)).reshape(n, k * SF_BYTES)
    same = bool(np.array_equal(g, ref[:n, :k * SF_BYTES]))
    parity = {"channels": n, "superframes": k, "bit_exact_vs_reference": same}
    return base, parity


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    if not torch.cuda.is_available():
        sys.exit("bench.py needs a HIP device (MI355X)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from pairphone_amd import MelpeEngine
    C, K, W = args.channels, args.steps, args.warmup
    eng = MelpeEngine(C, device=local)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    # every step's PCM generated on the device before the timed region
    pcm = torch.empty((W + K, C, SF_SAMPLES), dtype=torch.int16, device=dev)
    bits = torch.zeros((W + K, C, SF_BYTES), dtype=torch.uint8, device=dev)
    eng.synth_seed(RUN_SEED, first_channel=rank * C)
    for s in range(W + K):
        eng.synth_dev(pcm[s].data_ptr(), SF_SAMPLES, sptr)
    torch.cuda.synchronize(dev)
    log("rank %d: %d channels x %d superframes of input resident" % (rank, C, W + K))

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(fns):
        """W untimed steps, then K timed steps bracketed by barrier + sync;
        each step runs the launches in `fns` (callables of the step index)
        in order on `stream`, with a HIP event around each launch.  Returns
        (wall seconds for K steps, max over ranks; mean ms per launch)."""
        for s in range(W):
            for fn in fns:
                fn(s)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(fns) + 1)]
              for _ in range(K)]
        t0 = time.perf_counter()
        for i in range(K):
            ev[i][0].record(stream)
            for j, fn in enumerate(fns):
                fn(W + i)
                ev[i][j + 1].record(stream)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        kms = [float(np.mean([ev[i][j].elapsed_time(ev[i][j + 1]) for i in range(K)]))
               for j in range(len(fns))]
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, kms

    # one step = melpe_a on every channel = k_enc_npp then k_enc_ana
    # (melpe_encode_npp_dev + melpe_encode_ana_dev == melpe_encode_dev)
    enc_s, (npp_kms, ana_kms) = timed([
        lambda s: eng.encode_npp_dev(pcm[s].data_ptr(), None, sptr),
        lambda s: eng.encode_ana_dev(bits[s].data_ptr(), pcm[s].data_ptr(), None, sptr)])
    enc_kms = npp_kms + ana_kms
    log("encode: %.1f ms/step (k_enc_npp %.1f ms + k_enc_ana %.1f ms)"
        % (1e3 * enc_s / K, npp_kms, ana_kms))
    # end-of-run bitstream gather (the only collective, outside the timed
    # region): every rank's K x C x 11 bytes to every rank, rank 0 keeps them
    from pairphone_amd.shard import gather_bitstreams
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    allbits = gather_bitstreams(bits[W:], world * C)
    torch.cuda.synchronize(dev)
    gather_ms = 1e3 * (time.perf_counter() - t0)
    gathered = {"bytes": int(allbits.numel()), "ms": gather_ms,
                "collective": "all_gather" if world > 1 else "none (1 rank)"}
    dec = None
    if not args.no_decode:
        out = torch.empty((W + K, C, SF_SAMPLES), dtype=torch.int16, device=dev)
        dec_s, (dec_kms,) = timed([lambda s: eng.decode_dev(out[s].data_ptr(), bits[s].data_ptr(),
                                                            None, sptr)])
        dec = {"value": world * C * K * SF_SECONDS / dec_s, "unit": "channel-s/s decoded",
               "ms_per_step": 1e3 * dec_s / K, "kernel_ms": dec_kms}
        log("decode: %.1f ms/step (kernel %.1f ms)" % (1e3 * dec_s / K, dec_kms))

    # voice-frame crypt (VoiceEnc, crp.c:986-1000) of each superframe's
    # packets, the TX step after melpe_a: one packet per channel per launch
    lib = eng.lib
    g = torch.Generator().manual_seed(RUN_SEED + rank)
    keys = torch.randint(0, 256, (C, 16), dtype=torch.uint8, generator=g).to(dev)
    ctrs = torch.randint(0, 2**31, (C,), dtype=torch.int32, generator=g).to(dev)
    cbits = bits.clone()

    def crypt(s):
        if lib.melpe_voice_crypt_dev(cbits[s].data_ptr(), ctrs.data_ptr(), keys.data_ptr(),
                                     None, C, 1, 0, sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    crypt_s, (crypt_kms,) = timed([crypt])
    crypt_ach = VC_OPS_PER_PACKET * C / (crypt_kms / 1e3) / 1e12
    vcrypt = {"kernel": "k_voice_crypt", "value": world * C * K / crypt_s, "unit": "packets/s",
              "kernel_ms": crypt_kms, "packets_per_launch": C,
              "roofline": {"bound": "valu", "ops_per_packet": VC_OPS_PER_PACKET,
                           "achieved": crypt_ach, "peak": PEAK_VALU_TOPS,
                           "unit": "T INT32 VALU lane-ops/s", "frac": crypt_ach / PEAK_VALU_TOPS,
                           "algorithmic_hbm_bytes_per_launch": C * (2 * SF_BYTES + 16 + 4)}}
    log("voice crypt: kernel %.3f ms per %d packets" % (crypt_kms, C))
    # TX voice-activity gate (vad2 x6 per superframe, tx.c:234-239) on the
    # same PCM, one superframe per channel per launch, state resident
    vst = torch.zeros(C * lib.melpe_vad_state_bytes(), dtype=torch.uint8, device=dev)
    votes = torch.zeros((W + K, C), dtype=torch.uint8, device=dev)
    if lib.melpe_vad_reset_dev(vst.data_ptr(), C, None, sptr):
        raise RuntimeError(lib.melpe_last_error().decode())

    def vad(s):
        if lib.melpe_vad_dev(vst.data_ptr(), pcm[s].data_ptr(), votes[s].data_ptr(), C, None,
                             sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    vad_s, (vad_kms,) = timed([vad])
    vgate = {"kernel": "k_vad", "value": world * C * K * SF_SECONDS / vad_s,
             "unit": "channel-s/s gated", "kernel_ms": vad_kms,
             "silent_fraction": float((votes[W:] == 0).float().mean().item())}
    log("vad: kernel %.3f ms per %d channel-superframes" % (vad_kms, C))

    if rank != 0:
        return
    value = world * C * K * SF_SECONDS / enc_s
    oc = opcount()
    roof = None
    if oc:
        def kroof(kernel, W_sf, kms, in_b, out_b):
            ach = W_sf * C / (kms / 1e3) / 1e12
            return {"kernel": kernel, "kernel_ms": kms, "W_per_channel_superframe": W_sf,
                    "achieved": ach, "frac": ach / PEAK_VALU_TOPS,
                    "algorithmic_hbm_bytes_per_launch": C * (in_b + out_b),
                    "traffic": pmc_traffic(kernel, C)}
        # the dominant kernel of the step (analysis) carries the headline
        # roofline; the NPP kernel and the whole step are listed beside it
        ana = kroof("k_enc_ana", oc["W_enc_ana_per_sf"], ana_kms, 2 * SF_SAMPLES, SF_BYTES)
        npp = kroof("k_enc_npp", oc["W_enc_npp_per_sf"], npp_kms, 2 * SF_SAMPLES, 2 * SF_SAMPLES)
        step_ach = oc["W_enc_per_sf"] * C / (enc_kms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": ana["achieved"], "peak": PEAK_VALU_TOPS,
                "unit": "T basic-ops/s (INT32 VALU lane-ops)", "frac": ana["frac"],
                "traffic": ana["traffic"], "kernel": "k_enc_ana", "kernel_ms": ana_kms,
                "W_per_channel_superframe": ana["W_per_channel_superframe"],
                "algorithmic_hbm_bytes_per_launch": ana["algorithmic_hbm_bytes_per_launch"],
                "kernels": [ana, npp],
                "encode_step": {"W_per_channel_superframe": oc["W_enc_per_sf"],
                                "kernel_ms": enc_kms, "achieved": step_ach,
                                "frac": step_ach / PEAK_VALU_TOPS}}
        if dec:
            dec["roofline_frac"] = oc["W_dec_per_sf"] * C / (dec["kernel_ms"] / 1e3) / 1e12 / PEAK_VALU_TOPS
            dec["W_per_channel_superframe"] = oc["W_dec_per_sf"]
            dec["traffic"] = pmc_traffic("k_decode", C)
    if oc and oc.get("W_vad_per_sf"):
        vach = oc["W_vad_per_sf"] * C / (vgate["kernel_ms"] / 1e3) / 1e12
        vgate["roofline"] = {"bound": "valu", "W_per_channel_superframe": oc["W_vad_per_sf"],
                             "achieved": vach, "peak": PEAK_VALU_TOPS,
                             "unit": "T basic-ops/s (INT32 VALU lane-ops)",
                             "frac": vach / PEAK_VALU_TOPS}
    base, parity = (None, None)
    if world == 1:
        base, parity = cpu_baseline(args, bits[:W + K, :args.cpu_sample_channels].cpu().numpy())
    line = {
        "metric": "MELPe-1200 channel-seconds encoded/sec (node)",
        "value": value, "unit": "channel-s/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": 1e3 * enc_s / K, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int16/int32 saturating fixed point",
        "data": "synthetic (integer speech-like generator csrc/synth.h, run seed %d)" % RUN_SEED,
        "config": {"workload": "config 4: %d channels per GPU, melpe_a per superframe "
                               "(NPP x3 + MELPe-1200 analysis + 81-bit packing)" % C,
                   "channels_per_gpu": C, "channels_total": world * C,
                   "parallelism": "channel shards, %d GPU(s), no collective" % world},
        "realtime_factor": value / (world * C),
        "roofline": roof, "cpu_baseline": base, "decode": dec, "parity_spot_check": parity,
        "bitstream_gather": gathered, "voice_crypt": vcrypt, "vad": vgate,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
