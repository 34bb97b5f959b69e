#!/usr/bin/env python3
"""Benchmark: MELPe-1200 channel-seconds encoded per second on MI355X.

Headline (BASELINE.json metric, config 4 at N=1): every step is one melpe_a
superframe (540 samples -> 81 bits) of each of C channels per GPU (default
262,144 = 17,694 channel-seconds of audio per GPU per step); channels are
sharded statically across ranks (rank r owns channels [r*C, (r+1)*C)) with no
collective on the data path: "scaling": "weak".  Beside it, the strong-
scaling leg of config 4 as BASELINE states it: --total-channels (262,144)
split across the N ranks with channel_range (32,768 per GPU at N=8).

Inputs: the integer speech-like generator (pairphone_amd/csrc/synth.h) run on
the device before the timed region, so every step's PCM is resident in HBM;
bitstreams stay on the device until one all_gather after the timed region.
The decode leg (melpe_s of the bits just produced), the TX front end (VAD
gate + melpe_a on ragged streams, config 5), the voice-frame crypt and the
VAD alone are timed the same way and reported beside the headline.

A step is two launches on one stream: k_enc_npp (noise pre-processor, one
wavefront per channel) then the analysis (k_enc_ana, lane per channel, up to
the Fourier magnitudes; k_enc_harm, their FFTs with a wavefront per channel;
k_enc_tail, the packing -- or k_enc_ana_mw at up to 32,768 channels); each
launch is bracketed by HIP events on that stream.

Roofline: the codec is bit-exact saturating int16/int32 arithmetic with
serial recursions per channel, so it is bounded by INT VALU issue, not HBM
and not MFMA.  For the dominant launch (the analysis, reported as
"k_enc_ana") achieved = W_ana x channels / its average duration, W_ana = the
reference's basic
ops per channel-superframe of the analysis averaged over exactly the
superframes this run times (profiles/opcount.json W_enc_ana_by_sf, counted by
tools/opcount.py on this same input); peak = 256 CUs x 4 SIMDs x 32
lanes/clk x 2.4 GHz = 78.6 T lane-ops/s.  traffic = HBM bytes per launch from
the committed rocprofv3 --pmc passes at this channel count
(profiles/pmc_latest.json, which names its source file).

cpu_baseline: the reference codec itself (oracle/_ref/ref_tool, compiled from
/root/reference by oracle/Makefile), one single-channel process per host
core on a bounded sample of the same channels, measured at 16, 64 and all
usable cores (the value is the curve's best point: past the cgroup's CPU
quota more processes only time-share the same cores); its bitstreams double
as a parity spot check of the timed GPU output.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C]
                  [--total-channels T]
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
rank processes itself (before touching the GPU); under torch.distributed.run
it is one of them.
"""
import argparse
import json
import os
import socket
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
# the kernels of one analysis launch (encode_ana_dev): the lane-per-channel
# analysis split around the wave-per-channel Fourier magnitudes (k_harm.hip),
# or the multi-wave kernel at the channel counts the engine runs it
# (engine.hip ana_launch: the two launch orders never run together, so a
# PMC set's traffic is summed over the order the engine runs at that
# channel count only)
ANALYSIS_LANE = ("k_enc_ana<1>", "k_enc_harm", "k_enc_tail")
ANALYSIS_MW = ("k_enc_ana_mw<4>",)
MW_MAX_CHANNELS = 32768
DEC2_MAX_CHANNELS = 65536    # engine.hip: the two-wave decoder up to here


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--channels", type=int, default=262144, help="channels per GPU (weak)")
    ap.add_argument("--total-channels", type=int, default=262144,
                    help="config 4 strong-scaling leg: channels split across the ranks "
                         "(0 = skip)")
    ap.add_argument("--tx-channels", type=int, default=65536,
                    help="config 5 TX front end leg, channels per GPU (0 = skip)")
    ap.add_argument("--rt-channels", type=int, default=65536,
                    help="config 3 round-trip leg (encode + decode per superframe), channels per "
                         "GPU (0 = skip)")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-side-legs", action="store_true", help="skip crypt and VAD legs")
    ap.add_argument("--no-duplex", action="store_true",
                    help="skip the duplex leg (encoder + decoder engines, shared vs own streams)")
    ap.add_argument("--no-host-leg", action="store_true",
                    help="skip the host-fed (pinned host buffers, PCIe-inclusive) encode leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-channels", type=int, default=128)
    ap.add_argument("--cpu-jobs", type=int, default=0,
                    help="one point at this many processes (0 = the curve 16, 64, all cores)")
    return ap.parse_args(argv)


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- launch --

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(argv, n):
    """--gpus N without a launcher: start N rank processes (one GPU each) and
    wait.  Runs before this process touches the GPU."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


# ----------------------------------------------------------- device rigs --

class GpuRig:
    """torch device, the stream every engine call is enqueued on, HIP events
    on that stream, barrier + max over ranks"""

    def __init__(self, local, world):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.world = torch, dist, world
        if not torch.cuda.is_available():
            sys.exit("bench.py needs a HIP device (MI355X)")
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.stream = torch.cuda.current_stream(self.dev)
        self.sptr = self.stream.cuda_stream

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)

    def record(self, ev):
        ev.record(self.stream)

    @staticmethod
    def elapsed_ms(a, b):
        return a.elapsed_time(b)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def timed(rig, fns, K, W):
    """W untimed steps, then K timed steps bracketed by barrier + sync; each
    step runs the launches in `fns` (callables of the step index) in order,
    with an event recorded around each launch.  Returns (wall seconds for K
    steps, max over ranks; mean ms per launch of each fn)."""
    for s in range(W):
        for fn in fns:
            fn(s)
    rig.sync()
    rig.barrier()
    rig.sync()
    ev = [[rig.event() for _ in range(len(fns) + 1)] for _ in range(K)]
    t0 = time.perf_counter()
    for i in range(K):
        rig.record(ev[i][0])
        for j, fn in enumerate(fns):
            fn(W + i)
            rig.record(ev[i][j + 1])
    rig.sync()
    rig.barrier()
    rig.sync()
    dt = time.perf_counter() - t0
    kms = [float(np.mean([rig.elapsed_ms(ev[i][j], ev[i][j + 1]) for i in range(K)]))
           for j in range(len(fns))]
    return rig.max_over_ranks(dt), kms


# -------------------------------------------------------------- workload --

class EngineWorkload:
    """C channels (global ids first..first+C-1) on one engine; PCM of every
    step generated on the device up front; bits stay on the device."""

    def __init__(self, rig, C, first, steps):
        import torch
        from pairphone_amd import MelpeEngine
        self.rig, self.C, self.first, self.steps = rig, C, first, steps
        self.eng = MelpeEngine(C, device=rig.dev.index)
        self.lib = self.eng.lib
        self.pcm = torch.empty((steps, C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
        self.bits = torch.zeros((steps, C, SF_BYTES), dtype=torch.uint8, device=rig.dev)
        self.out = None
        self.regen_pcm()

    def regen_pcm(self):
        """the raw synthetic PCM of every step (melpe_a overwrites it in place
        with the NPP output, melpe/melpe.c:94-96)"""
        self.eng.synth_seed(RUN_SEED, first_channel=self.first)
        for s in range(self.steps):
            self.eng.synth_dev(self.pcm[s].data_ptr(), SF_SAMPLES, self.rig.sptr)
        self.rig.sync()

    def npp(self, s):
        self.eng.encode_npp_dev(self.pcm[s].data_ptr(), None, self.rig.sptr)

    def ana(self, s):
        self.eng.encode_ana_dev(self.bits[s].data_ptr(), self.pcm[s].data_ptr(), None,
                                self.rig.sptr)

    def pipe(self, s, nxt):
        """superframe s's analysis beside superframe nxt's NPP (None: none)"""
        self.eng.encode_pipe_dev(self.bits[s].data_ptr(), self.pcm[s].data_ptr(),
                                 None if nxt is None else self.pcm[nxt].data_ptr(), stream=self.rig.sptr)

    def duplex(self, s, nxt, d):
        """pipe(s, nxt) plus the decode of superframe d (None: none) on the
        engine's decoder stream, beside it (melpe_duplex_pipe_dev)"""
        if self.out is None:
            self.out = self.rig.torch.empty_like(self.pcm)
        self.eng.duplex_pipe_dev(self.bits[s].data_ptr(), self.pcm[s].data_ptr(),
                                 None if nxt is None else self.pcm[nxt].data_ptr(),
                                 None if d is None else self.out[d].data_ptr(),
                                 None if d is None else self.bits[d].data_ptr(), stream=self.rig.sptr)

    def restart(self):
        """fresh-process state and the raw input again (melpe_engine_reset)"""
        self.eng.reset()
        self.regen_pcm()

    def dec(self, s):
        if self.out is None:
            self.out = self.rig.torch.empty_like(self.pcm)
        self.eng.decode_dev(self.out[s].data_ptr(), self.bits[s].data_ptr(), None,
                            self.rig.sptr)

    def close(self):
        self.eng.close()
        self.pcm = self.bits = self.out = None


# ------------------------------------------------------------ roofline W --

def opcount():
    p = os.path.join(ROOT, "profiles", "opcount.json")
    return json.load(open(p)) if os.path.exists(p) else None


def w_over(oc, key, lo, hi):
    """mean W per channel-superframe over superframe indices [lo, hi) (the
    ones this run times); the 149-superframe mean where the census does not
    reach that far"""
    by = oc.get(key + "_by_sf")
    if by and hi <= len(by):
        return float(np.mean(by[lo:hi])), "superframes %d..%d (the timed ones)" % (lo, hi - 1)
    return oc[key + "_per_sf"], "149-superframe mean (timed range not in the census)"


def pmc_traffic(kernel, channels):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc
    passes (profiles/pmc_latest.json, written by tools/prof_summary.py: one
    set per channel count), if a set was taken at this channel count; else
    None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(p):
        return None, None
    d = json.load(open(p))
    sets = d.get("sets", [d])
    d = next((x for x in sets if x.get("channels") == channels), None)
    if d is None:
        return None, None
    ks = d.get("kernels", {})
    if kernel == "k_enc_ana":
        names = ANALYSIS_MW if channels <= MW_MAX_CHANNELS else ANALYSIS_LANE
    else:
        names = (kernel,)
    got = [ks[n]["bytes_per_launch"] for n in names if n in ks]
    return (sum(got) if got else None), d.get("source")


def kroof(kernel, W_sf, C, kms, in_b, out_b, traffic_key=None):
    ach = W_sf * C / (kms / 1e3) / 1e12
    traffic, src = pmc_traffic(traffic_key or kernel, C)
    return {"kernel": kernel, "kernel_ms": kms, "W_per_channel_superframe": W_sf,
            "achieved": ach, "frac": ach / PEAK_VALU_TOPS,
            "algorithmic_hbm_bytes_per_launch": C * (in_b + out_b),
            "traffic": traffic, "traffic_source": src}


# ----------------------------------------------------------- CPU baseline --

def usable_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """cores' worth of CPU time the job's cgroup grants (cpu.max), or None"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _ref_encode_rate(jobs, S, nsf, first=0):
    """the reference encoding S channels x nsf superframes, `jobs` single-
    channel processes at a time: (channel-s/s, wall s, bits [S, nsf*11])"""
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "b.bits")
        t0 = time.perf_counter()
        subprocess.run([REF_TOOL, "jobs", str(jobs), "encgen", str(RUN_SEED), str(first), str(S),
                        str(nsf), out], check=True)
        dt = time.perf_counter() - t0
        bits = np.fromfile(out, dtype=np.uint8).reshape(S, nsf * SF_BYTES)
    return S * nsf * SF_SECONDS / dt, dt, bits


def cpu_baseline(args, gpu_bits):
    """The reference codec, one single-channel process per host core
    (north_star), on a bounded sample of the same channels: a curve over 16,
    64 and all usable cores, each point 2 channels per process x 10 s of
    audio; the line's value is the curve's best point.  The first point's
    bitstreams double as a parity spot check of the timed GPU output.
    Returns (baseline dict, parity dict)."""
    if args.no_cpu_baseline or not os.path.exists(REF_TOOL):
        return None, None
    usable = usable_cores()
    nsf = max(149, gpu_bits.shape[0])
    points = sorted(set([args.cpu_jobs] if args.cpu_jobs else
                        [n for n in (16, 64) if n < usable] + [usable]))
    curve, ref = [], None
    for jobs in points:
        S = max(args.cpu_sample_channels, 2 * jobs)
        value, dt, bits = _ref_encode_rate(jobs, S, nsf)
        if ref is None:
            ref = bits
        curve.append({"processes": jobs, "channels": S, "value": value, "wall_s": dt,
                      "per_process": value / jobs})
        log("cpu baseline: %d processes, %d channels: %.0f channel-s/s (%.1f s)"
            % (jobs, S, value, dt))
    # the value is the best point of the curve: past the cgroup's CPU quota
    # the extra processes only time-share the same cores (the oversubscribed
    # points stay in the curve)
    top = max(curve, key=lambda p: p["value"])
    quota = cgroup_cpu_quota()
    # cores = the CPU the processes actually had: the process count, capped
    # by the cgroup's quota where one is set (more processes than the quota
    # only time-share those cores)
    cores = top["processes"] if quota is None else min(top["processes"], int(round(quota)))
    base = {"value": top["value"], "unit": "channel-s/s", "cores": cores,
            "processes": top["processes"],
            "kind": "reference", "host_cores_visible": usable, "cgroup_cpu_quota_cores": quota,
            "curve": curve,
            "sample": "channels 0..S-1 x %d superframes (%.1f s of audio each), melpe_a, one "
                      "forked single-channel reference process per channel, `processes` at a "
                      "time; value = the best point of the curve (%d processes, %d channels, "
                      "%.1f s wall)"
                      % (nsf, nsf * SF_SECONDS, top["processes"], top["channels"], top["wall_s"])}
    n = min(ref.shape[0], gpu_bits.shape[1])
    k = gpu_bits.shape[0]
    g = np.ascontiguousarray(gpu_bits[:, :n, :].transpose(1, 0, 2)).reshape(n, k * SF_BYTES)
    same = bool(np.array_equal(g, ref[:n, :k * SF_BYTES]))
    parity = {"channels": n, "superframes": k, "bit_exact_vs_reference": same}
    return base, parity


# ------------------------------------------------------------------ legs --

def encode_leg(rig, wl, K, W):
    return timed(rig, [wl.npp, wl.ana], K, W)


def pipe_warmup(wl, W, dec=False):
    """W warm-up steps in the pipelined form (the engine makes and warms its
    side stream at the first pipelined call, outside the timed region):
    npp(0), pipe(0, 1), ..., pipe(W-1, none) -- superframe W is left for
    the timed region's first NPP"""
    if W <= 0:
        return
    wl.npp(0)
    for s in range(W):
        wl.pipe(s, s + 1 if s + 1 < W else None)
        if dec:
            wl.dec(s)


def pipe_leg(rig, wl, K, W):
    """The headline step pipelined (melpe_encode_pipe_dev): superframe k's
    analysis on the engine stream beside superframe k + 1's NPP on the
    engine's second stream, whose waves take the SIMD slots the analysis'
    waves free as they finish (the launch's tail: profiles/
    r06_i_wave_times.jsonl).  W warm-up steps pipelined, then a timed
    region holding exactly K NPPs and K analyses: the NPP of superframe W,
    then K pipelined steps, the last without a next NPP.  HIP events on the
    caller's stream bracket each step.  Returns (wall seconds, max over
    ranks; mean ms per step by events)."""
    pipe_warmup(wl, W)
    rig.sync()
    rig.barrier()
    rig.sync()
    ev = [rig.event() for _ in range(K + 1)]
    t0 = time.perf_counter()
    wl.npp(W)
    rig.record(ev[0])
    for i in range(K):
        wl.pipe(W + i, W + i + 1 if i + 1 < K else None)
        rig.record(ev[i + 1])
    rig.sync()
    rig.barrier()
    rig.sync()
    dt = time.perf_counter() - t0
    ems = float(np.mean([rig.elapsed_ms(ev[i], ev[i + 1]) for i in range(K)]))
    return rig.max_over_ranks(dt), ems


def host_leg(rig, C, first, K, W, dev_bits, world):
    """The host-fed form of the headline (melpe/melpe.c:91-99's contract:
    the caller hands host buffers): the same channels and synthetic input,
    in pinned host memory, through melpe_encode_host_async -- per superframe
    the PCM over PCIe to the device, melpe_a, the NPP output (in place, as
    melpe_a) and the bits back, double-buffered so the copies of superframes
    k - 1 and k + 1 overlap the kernels of k.  A fresh engine, so its bits
    must equal the device-resident run's bit for bit."""
    import torch
    from pairphone_amd import MelpeEngine
    eng = MelpeEngine(C, device=rig.dev.index)
    eng.synth_seed(RUN_SEED, first_channel=first)
    tmp = torch.empty((C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
    t0 = time.perf_counter()
    pcm_h = torch.empty((W + K, C, SF_SAMPLES), dtype=torch.int16, pin_memory=True)
    bits_h = torch.zeros((W + K, C, SF_BYTES), dtype=torch.uint8, pin_memory=True)
    for s in range(W + K):
        eng.synth_dev(tmp.data_ptr(), SF_SAMPLES, rig.sptr)
        pcm_h[s].copy_(tmp)
    rig.sync()
    log("host leg: %.1f GB of pinned input made in %.1f s" % (pcm_h.numel() * 2 / 1e9,
                                                               time.perf_counter() - t0))
    del tmp

    def step(s):
        eng.encode_host_async(bits_h[s].data_ptr(), pcm_h[s].data_ptr())
    for s in range(W):
        step(s)
    eng.encode_host_wait()
    rig.sync()
    rig.barrier()
    t0 = time.perf_counter()
    for s in range(W, W + K):
        step(s)
    eng.encode_host_wait()
    dt = rig.max_over_ranks(time.perf_counter() - t0)
    same = bool(torch.equal(bits_h[W:], dev_bits[W:].cpu()))
    eng.close()
    del pcm_h, bits_h
    return {"value": world * C * K * SF_SECONDS / dt, "unit": "channel-s/s (host buffers in and out)",
            "ms_per_step": 1e3 * dt / K, "steps": K, "warmup": W,
            "pcie_bytes_per_step": C * (2 * SF_SAMPLES * 2 + SF_BYTES),
            "bits_equal_device_resident": same,
            "how": "melpe_encode_host_async: pinned host PCM [C, 540] in, NPP output and bits "
                   "out per superframe, two device slots, H2D / kernels / D2H on three streams"}


def duplex_leg(rig, wl, C, K, W):
    """A duplex link's two directions on one GPU: an encoder engine and a
    decoder engine of C channels, superframe k encoded on one caller stream
    while superframe k - 1's bits are decoded on another.  Timed with fresh
    engines each time: with both engines on the device's shared engine
    stream (the default: one hardware queue, the kernels serialise), with
    each on a stream of its own (melpe_engine_set_own_stream: the kernels
    may overlap), and with one engine doing both directions
    (melpe_duplex_pipe_dev: the analysis, the next NPP and the decode on the
    engine's three streams).  ms per duplex step each way, and whether the
    runs' bits agree."""
    import torch
    from pairphone_amd import MelpeEngine
    out = {}
    ref_bits = None
    for mode in ("shared", "own"):
        wl.regen_pcm()
        enc, dec = MelpeEngine(C, device=rig.dev.index), MelpeEngine(C, device=rig.dev.index)
        if mode == "own":
            enc.set_own_stream(True)
            dec.set_own_stream(True)
        sa, sb = torch.cuda.Stream(rig.dev), torch.cuda.Stream(rig.dev)
        bits = torch.zeros((W + K, C, SF_BYTES), dtype=torch.uint8, device=rig.dev)
        pcm = torch.empty((C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
        evs = [torch.cuda.Event() for _ in range(W + K)]

        def step(s):
            enc.encode_dev(bits[s].data_ptr(), wl.pcm[s].data_ptr(), None, sa.cuda_stream)
            evs[s].record(sa)
            if s > 0:
                sb.wait_event(evs[s - 1])
                dec.decode_dev(pcm.data_ptr(), bits[s - 1].data_ptr(), None, sb.cuda_stream)
        for s in range(W):
            step(s)
        rig.sync()
        t0 = time.perf_counter()
        for s in range(W, W + K):
            step(s)
        rig.sync()
        out[mode] = 1e3 * (time.perf_counter() - t0) / K
        if ref_bits is None:
            ref_bits = bits.cpu()
        else:
            out["bits_equal"] = bool(torch.equal(ref_bits, bits.cpu()))
        enc.close()
        dec.close()
        del bits, pcm
    # one engine, both directions: melpe_duplex_pipe_dev (superframe k's
    # analysis, k+1's NPP, the decode of k-1 on the engine's three streams)
    wl.regen_pcm()
    eng = MelpeEngine(C, device=rig.dev.index)
    bits = torch.zeros((W + K, C, SF_BYTES), dtype=torch.uint8, device=rig.dev)
    pcm = torch.empty((C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
    s0 = rig.sptr

    def dstep(s):
        nx = s + 1 < W + K
        eng.duplex_pipe_dev(bits[s].data_ptr(), wl.pcm[s].data_ptr(), wl.pcm[s + 1].data_ptr() if nx else None,
                            pcm.data_ptr() if s > 0 else None, bits[s - 1].data_ptr() if s > 0 else None,
                            stream=s0)
    eng.encode_npp_dev(wl.pcm[0].data_ptr(), None, s0)
    for s in range(W):
        dstep(s)
    rig.sync()
    t0 = time.perf_counter()
    for s in range(W, W + K):
        dstep(s)
    rig.sync()
    out["pipe"] = 1e3 * (time.perf_counter() - t0) / K
    out["pipe_bits_equal"] = bool(torch.equal(ref_bits, bits.cpu()))
    eng.close()
    del bits, pcm
    res = {"ms_per_step_shared_stream": out["shared"], "ms_per_step_own_streams": out["own"],
           "ms_per_step_one_engine_duplex_pipe": out["pipe"],
           "bits_equal": out["bits_equal"] and out["pipe_bits_equal"], "channels": C,
           "step": "encode superframe k (caller stream A) + decode superframe k - 1 (caller stream B)"}
    log("duplex: %.1f ms/step on the shared engine stream, %.1f ms/step on own streams, "
        "%.1f ms/step on one engine (melpe_duplex_pipe_dev)" % (out["shared"], out["own"], out["pipe"]))
    return res


def round_trip_leg(rig, args, rank, world):
    """BASELINE config 3: the encode + decode round trip (melpe_a then melpe_s
    with the postfilter, melpe/melpe.c:91-107) of --rt-channels channels per
    GPU on one engine; one step = k_enc_npp + the analysis + k_decode of one
    superframe of every channel.  Timed serialised (each launch alone, HIP
    events), then from fresh state as the engine runs it: superframe k's
    analysis, k+1's NPP and the decode of k-1's bits on three queues
    (melpe_duplex_pipe_dev), whose bits and PCM must equal the serialised
    run's.  After the timed region the bits and the decoded PCM of sampled channels are checked
    against the reference (oracle/_ref/ref_tool encgen + decgen on the same
    synthetic channels), on rank 0."""
    C, K, W = args.rt_channels, args.steps, args.warmup
    wl = EngineWorkload(rig, C, rank * C, W + K)
    # serialised, each launch timed alone; then from fresh state the same
    # work on the engine's three queues
    ser, (npp_kms, ana_kms, dec_kms) = timed(rig, [wl.npp, wl.ana, wl.dec], K, W)
    ser_bits, ser_out = wl.bits.clone(), wl.out.clone()
    wl.restart()
    # warm-up in the same form (the engine makes and warms its side streams
    # at the first call): npp(0), duplex(0, 1, -), duplex(1, 2, 0), ...,
    # duplex(W-1, -, W-2); the timed region then holds exactly K NPPs, K
    # analyses and K decodes: npp(W), duplex(W+i, W+i+1, W+i-1) for i < K
    # (the decode of W+K-1 follows it)
    if W > 0:
        wl.npp(0)
        for s in range(W):
            wl.duplex(s, s + 1 if s + 1 < W else None, s - 1 if s > 0 else None)
    rig.sync()
    rig.barrier()
    rig.sync()
    t0 = time.perf_counter()
    wl.npp(W)
    for i in range(K):
        s = W + i
        wl.duplex(s, s + 1 if i + 1 < K else None, s - 1 if s > 0 else None)
    rig.sync()
    rig.barrier()
    rig.sync()
    dt = rig.max_over_ranks(time.perf_counter() - t0)
    wl.dec(W + K - 1)
    rig.sync()
    same = bool((ser_bits == wl.bits).all()) and bool((ser_out == wl.out).all())
    del ser_bits, ser_out
    res = {"workload": "config 3: %d channels per GPU, melpe_a + melpe_s (with postfilter) "
                       "per superframe on one engine" % C,
           "channels_per_gpu": C, "value": world * C * K * SF_SECONDS / dt,
           "unit": "channel-s/s (encoded and decoded)", "ms_per_step": 1e3 * dt / K,
           "step": "melpe_duplex_pipe_dev: superframe k's analysis, k+1's NPP and the decode of "
                   "k-1's bits on three queues of one engine",
           "ms_per_step_serialised": 1e3 * ser / K, "bits_pcm_equal_serialised": same,
           "kernels_ms": {"k_enc_npp": npp_kms, "k_enc_ana": ana_kms, "k_decode": dec_kms}}
    oc = opcount()
    if oc:
        w_ana, _ = w_over(oc, "W_enc_ana", W, W + K)
        w_npp, _ = w_over(oc, "W_enc_npp", W, W + K)
        w_dec, _ = w_over(oc, "W_dec", W, W + K)
        res["roofline_frac"] = {
            k: w * C / (ms / 1e3) / 1e12 / PEAK_VALU_TOPS
            for k, w, ms in (("k_enc_npp", w_npp, npp_kms), ("k_enc_ana", w_ana, ana_kms),
                             ("k_decode", w_dec, dec_kms))}
        res["roofline_frac"]["step"] = ((w_ana + w_npp + w_dec) * C / dt * K / 1e12
                                        / PEAK_VALU_TOPS)
    if rank == 0 and not args.no_cpu_baseline and os.path.exists(REF_TOOL):
        n = W + K
        chans = sorted(set([0, C - 1] + [int(c) for c in np.linspace(1, C - 2, 14)]))
        gb = wl.bits[:, chans].cpu().numpy()
        go = wl.out[:, chans].cpu().numpy()
        ok_b = ok_p = True
        with tempfile.TemporaryDirectory() as tmp:
            for i, c in enumerate(chans):
                bp, pp = os.path.join(tmp, "%d.bits" % c), os.path.join(tmp, "%d.pcm" % c)
                subprocess.run([REF_TOOL, "encgen", str(RUN_SEED), str(c), "1", str(n), bp],
                               check=True)
                subprocess.run([REF_TOOL, "decgen", bp, "1", str(n), pp], check=True)
                rb = np.fromfile(bp, dtype=np.uint8).reshape(n, SF_BYTES)
                rp = np.fromfile(pp, dtype=np.int16).reshape(n, SF_SAMPLES)
                ok_b &= bool(np.array_equal(gb[:, i], rb))
                ok_p &= bool(np.array_equal(go[:, i], rp))
        res["parity_spot_check"] = {"channels": chans, "superframes": n,
                                    "bits_equal_reference": ok_b, "pcm_equal_reference": ok_p}
    wl.close()
    log("round trip (config 3, %d channels): %.2f ms/step (npp %.2f, analysis %.2f, "
        "decode %.2f ms)" % (C, res["ms_per_step"], npp_kms, ana_kms, dec_kms))
    return res


def tx_leg(rig, args, rank, world):
    """BASELINE config 5: the TX front end (tx.c:232-246: VAD gate, then
    melpe_a on the superframes it opens) on ragged streams, per-channel
    lengths uniform in [1 s, 20 s] (seeded), world x --tx-channels streams
    in all.  Ranks own contiguous ranges balanced by total superframes
    (shard.superframe_range), so a rank's step count follows its longest
    stream.  One step = one superframe of every channel whose stream is
    still running; the job is done when the longest stream ends.  Whole-job
    throughput = channel-seconds of all streams / wall time (max over
    ranks)."""
    import torch
    from pairphone_amd import MelpeEngine
    from pairphone_amd.shard import superframe_range
    g = np.random.default_rng(RUN_SEED + 5)
    lengths_all = g.integers(15, 297, size=world * args.tx_channels)     # 1 s .. 20 s
    lo, hi = superframe_range(rank, world, lengths_all)
    lengths = lengths_all[lo:hi]
    C = hi - lo
    nsf = int(lengths.max())
    eng = MelpeEngine(C, device=rig.dev.index)
    lib = eng.lib
    pcm = torch.empty((nsf, C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
    eng.synth_seed(RUN_SEED, first_channel=lo)
    for s in range(nsf):
        eng.synth_dev(pcm[s].data_ptr(), SF_SAMPLES, rig.sptr)
    act = (torch.arange(nsf, device=rig.dev)[:, None] <
           torch.from_numpy(lengths).to(rig.dev)[None, :]).to(torch.uint8).contiguous()
    bits = torch.zeros((nsf, C, SF_BYTES), dtype=torch.uint8, device=rig.dev)
    votes = torch.zeros((nsf, C), dtype=torch.uint8, device=rig.dev)
    gate = torch.zeros((nsf, C), dtype=torch.uint8, device=rig.dev)
    vst = torch.zeros(C * lib.melpe_vad_state_bytes(), dtype=torch.uint8, device=rig.dev)

    def fresh():
        """fresh codec and VAD state, the raw input again"""
        eng.reset()
        eng.synth_seed(RUN_SEED, first_channel=lo)
        for s in range(nsf):
            eng.synth_dev(pcm[s].data_ptr(), SF_SAMPLES, rig.sptr)
        if lib.melpe_vad_reset_dev(vst.data_ptr(), C, None, rig.sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
        for t in (bits, votes, gate):
            t.zero_()
        rig.sync()

    def step(s):
        if s < nsf:
            eng.tx_dev(vst.data_ptr(), bits[s].data_ptr(), pcm[s].data_ptr(), votes[s].data_ptr(),
                       gate[s].data_ptr(), act[s].data_ptr(), rig.sptr)

    def pstep(s):
        """the pipelined form: superframe s's analysis beside s+1's VAD and NPP"""
        if s == 0:
            eng.tx_npp_dev(vst.data_ptr(), pcm[0].data_ptr(), votes[0].data_ptr(), gate[0].data_ptr(),
                           act[0].data_ptr(), rig.sptr)
        if s < nsf:
            nx = s + 1 < nsf
            eng.tx_pipe_dev(vst.data_ptr(), bits[s].data_ptr(), pcm[s].data_ptr(), gate[s].data_ptr(),
                            pcm[s + 1].data_ptr() if nx else None, votes[s + 1].data_ptr() if nx else None,
                            gate[s + 1].data_ptr() if nx else None, act[s + 1].data_ptr() if nx else None,
                            stream=rig.sptr)
    # every rank runs the job's step count (its own streams may end sooner)
    steps = int(rig.max_over_ranks(float(nsf)))
    fresh()
    ser_dt, (ser_kms,) = timed(rig, [step], steps, 0)
    ser = (bits.clone(), votes.clone(), gate.clone())
    fresh()
    # the engine makes and warms its side stream at its first pipelined call:
    # one call with every mask zero (no channel's state moves) before timing
    z = torch.zeros((2, C), dtype=torch.uint8, device=rig.dev)
    zp = torch.zeros((2, C, SF_SAMPLES), dtype=torch.int16, device=rig.dev)
    zb = torch.zeros((C, SF_BYTES), dtype=torch.uint8, device=rig.dev)
    eng.tx_pipe_dev(vst.data_ptr(), zb.data_ptr(), zp[0].data_ptr(), z[0].data_ptr(), zp[1].data_ptr(),
                    zb.data_ptr(), z[1].data_ptr(), z[0].data_ptr(), stream=rig.sptr)
    rig.sync()
    del z, zp, zb
    dt, (kms,) = timed(rig, [pstep], steps, 0)
    same = all(bool(torch.equal(a, b)) for a, b in zip(ser, (bits, votes, gate)))
    del ser
    chs = float(lengths_all.sum()) * SF_SECONDS
    res = {"workload": "config 5: %d streams (%d per GPU on average), ragged lengths uniform in "
                       "[1 s, 20 s] (seed %d), VAD2 gate + melpe_a on the opened superframes"
                       % (len(lengths_all), args.tx_channels, RUN_SEED + 5),
           "value": chs / dt, "unit": "channel-s/s (whole streams)",
           "wall_s": dt, "steps": steps, "mean_step_ms": kms,
           "step": "melpe_tx_pipe_dev: superframe k's analysis beside k+1's VAD gate and NPP",
           "value_serialised": chs / ser_dt, "mean_step_ms_serialised": ser_kms,
           "bits_votes_gates_equal_serialised": same,
           "channel_seconds": chs,
           "gated_open_fraction": float(gate.float().sum().item() / act.float().sum().item()),
           "sharding": "shard.superframe_range: contiguous channel ranges balanced by total "
                       "superframes (rank 0: channels %d..%d)" % (lo, hi - 1)}
    eng.close()
    return res


def run(args, rank, world, local, backend="nccl", rig_cls=None, workload_cls=None):
    """one rank of the benchmark; returns the JSON line on rank 0.  rig_cls /
    workload_cls replace the device plumbing in the CPU tests (gloo ranks,
    tests/test_shard.py); the timing, sharding, gather and reporting code is
    this one."""
    import torch.distributed as dist
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend)
    rig = (rig_cls or GpuRig)(local, world)
    Workload = workload_cls or EngineWorkload
    C, K, W = args.channels, args.steps, args.warmup

    wl = Workload(rig, C, rank * C, W + K)
    log("rank %d: %d channels x %d superframes of input resident" % (rank, C, W + K))
    # one step = melpe_a on every channel = k_enc_npp then k_enc_ana
    # the serialised step: each launch alone, HIP events around each (the
    # kernels' own durations, for the roofline)
    ser_s, (npp_kms, ana_kms) = encode_leg(rig, wl, K, W)
    enc_kms = npp_kms + ana_kms
    log("encode, serialised: %.1f ms/step (k_enc_npp %.1f ms + k_enc_ana %.1f ms)"
        % (1e3 * ser_s / K, npp_kms, ana_kms))
    # the headline step: the same work pipelined, from fresh state on the
    # same input; its bits must equal the serialised run's
    ser_bits = wl.bits.clone()
    wl.restart()
    enc_s, pipe_ems = pipe_leg(rig, wl, K, W)
    pipe_equal = bool((ser_bits == wl.bits).all())
    del ser_bits
    log("encode, pipelined: %.1f ms/step, bits equal to the serialised run: %s"
        % (1e3 * enc_s / K, pipe_equal))
    hostfed = None
    if not args.no_host_leg and workload_cls is None:
        hostfed = host_leg(rig, C, rank * C, K, W, wl.bits, world)
        # against the serialised device-resident step: the host-fed call is
        # melpe_a's NPP + analysis of one superframe, not the pipelined pair
        hostfed["frac_of_device_resident"] = hostfed["value"] / (world * C * K * SF_SECONDS / ser_s)
        log("host-fed encode: %.1f ms/step (%.0f%% of device-resident), bits equal: %s"
            % (hostfed["ms_per_step"], 100 * hostfed["frac_of_device_resident"],
               hostfed["bits_equal_device_resident"]))
    # end-of-run bitstream gather (the only collective, outside the timed
    # region): every rank's K x C x 11 bytes to every rank, rank 0 keeps them
    from pairphone_amd.shard import gather_bitstreams, channel_range
    rig.sync()
    t0 = time.perf_counter()
    allbits = gather_bitstreams(wl.bits[W:], world * C)
    rig.sync()
    gathered = {"bytes": int(allbits.numel()), "ms": 1e3 * (time.perf_counter() - t0),
                "collective": "all_gather" if world > 1 else "none (1 rank)"}
    del allbits
    dec = None
    if not args.no_decode:
        dec_s, (dec_kms,) = timed(rig, [wl.dec], K, W)
        dec = {"value": world * C * K * SF_SECONDS / dec_s, "unit": "channel-s/s decoded",
               "ms_per_step": 1e3 * dec_s / K, "kernel_ms": dec_kms}
        log("decode: %.1f ms/step (kernel %.1f ms)" % (1e3 * dec_s / K, dec_kms))
    cpu_bits = wl.bits[:W + K, :args.cpu_sample_channels].cpu().numpy() if rank == 0 else None
    duplex = None
    if not args.no_duplex and workload_cls is None:
        duplex = duplex_leg(rig, wl, C, K, W)

    side = {}
    if not args.no_side_legs:
        side = side_legs(rig, wl, C, K, W, rank, world)
    wl.close()

    strong = None
    if args.total_channels:
        lo, hi = channel_range(rank, world, args.total_channels)
        if hi - lo == C:
            strong = {"ms_per_step": 1e3 * enc_s / K, "kernel_ms": enc_kms,
                      "ms_per_step_serialised": 1e3 * ser_s / K}
        else:
            sw = Workload(rig, hi - lo, lo, W + K)
            sser_s, (snpp, sana) = encode_leg(rig, sw, K, W)
            sw.restart()
            st_s, _ = pipe_leg(rig, sw, K, W)
            sw.close()
            strong = {"ms_per_step": 1e3 * st_s / K, "kernel_ms": snpp + sana,
                      "k_enc_npp_ms": snpp, "k_enc_ana_ms": sana,
                      "ms_per_step_serialised": 1e3 * sser_s / K}
        strong.update({"total_channels": args.total_channels,
                       "channels_per_gpu_max": -(-args.total_channels // world),
                       "value": args.total_channels * K * SF_SECONDS / (strong["ms_per_step"] / 1e3 * K),
                       "unit": "channel-s/s", "scaling": "strong",
                       "sharding": "shard.channel_range: contiguous, balanced"})
        log("strong (%d total): %.1f ms/step" % (args.total_channels, strong["ms_per_step"]))

    rt = None
    if args.rt_channels and workload_cls is None:
        rt = round_trip_leg(rig, args, rank, world)

    tx = None
    if args.tx_channels:
        tx = tx_leg(rig, args, rank, world)
        log("tx front end: %.0f channel-s/s over %d steps" % (tx["value"], tx["steps"]))

    if rank != 0:
        return None
    value = world * C * K * SF_SECONDS / enc_s
    oc = opcount()
    roof = None
    if oc:
        w_ana, w_src = w_over(oc, "W_enc_ana", W, W + K)
        w_npp, _ = w_over(oc, "W_enc_npp", W, W + K)
        # the dominant kernel of the step (analysis) carries the headline
        # roofline; the NPP kernel and the whole step are listed beside it
        ana = kroof("k_enc_ana", w_ana, C, ana_kms, 2 * SF_SAMPLES, SF_BYTES)
        npp = kroof("k_enc_npp", w_npp, C, npp_kms, 2 * SF_SAMPLES, 2 * SF_SAMPLES)
        step_ach = (w_ana + w_npp) * C / (enc_kms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": ana["achieved"], "peak": PEAK_VALU_TOPS,
                "unit": "T basic-ops/s (INT32 VALU lane-ops)", "frac": ana["frac"],
                "traffic": ana["traffic"], "traffic_source": ana["traffic_source"],
                "kernel": "k_enc_ana", "kernel_ms": ana_kms,
                "kernel_note": "the analysis launch: k_enc_ana + k_enc_harm + k_enc_tail (lane / "
                               "wave / lane per channel), or k_enc_ana_mw up to 32,768 channels",
                "W_per_channel_superframe": w_ana, "W_source": w_src,
                "algorithmic_hbm_bytes_per_launch": ana["algorithmic_hbm_bytes_per_launch"],
                "kernels": [ana, npp],
                "encode_step": {"W_per_channel_superframe": w_ana + w_npp,
                                "kernel_ms": enc_kms, "achieved": step_ach,
                                "frac": step_ach / PEAK_VALU_TOPS}}
        if dec:
            w_dec, _ = w_over(oc, "W_dec", W, W + K)
            dec["W_per_channel_superframe"] = w_dec
            dec["roofline_frac"] = w_dec * C / (dec["kernel_ms"] / 1e3) / 1e12 / PEAK_VALU_TOPS
            # the engine runs the two-wave decoder up to DEC2_MAX_CHANNELS
            dec["kernel"] = "k_decode2" if C <= DEC2_MAX_CHANNELS else "k_decode"
            dec["traffic"], _ = pmc_traffic(dec["kernel"], C)
        if side.get("vad") and oc.get("W_vad_per_sf"):
            v = side["vad"]
            vach = oc["W_vad_per_sf"] * C / (v["kernel_ms"] / 1e3) / 1e12
            v["roofline"] = {"bound": "valu", "W_per_channel_superframe": oc["W_vad_per_sf"],
                             "achieved": vach, "peak": PEAK_VALU_TOPS,
                             "unit": "T basic-ops/s (INT32 VALU lane-ops)",
                             "frac": vach / PEAK_VALU_TOPS}
    base, parity = (None, None)
    if world == 1:
        base, parity = cpu_baseline(args, cpu_bits)
    return {
        "metric": "MELPe-1200 channel-seconds encoded/sec (node)",
        "value": value, "unit": "channel-s/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": 1e3 * enc_s / K, "higher_is_better": True, "scaling": "weak",
        "step": {"form": "pipelined: superframe k's analysis beside superframe k+1's NPP "
                         "(melpe_encode_pipe_dev); the timed region holds K NPPs and K analyses",
                 "ms_per_step_events": pipe_ems,
                 "ms_per_step_serialised": 1e3 * ser_s / K,
                 "bits_equal_serialised": pipe_equal},
        "vs_baseline": None, "dtype": "int16/int32 saturating fixed point",
        "data": "synthetic (integer speech-like generator csrc/synth.h, run seed %d)" % RUN_SEED,
        "config": {"workload": "config 4: %d channels per GPU, melpe_a per superframe "
                               "(NPP x3 + MELPe-1200 analysis + 81-bit packing)" % C,
                   "channels_per_gpu": C, "channels_total": world * C,
                   "parallelism": "channel shards, %d GPU(s), no collective" % world},
        "realtime_factor": value / (world * C),
        "roofline": roof, "cpu_baseline": base, "decode": dec, "parity_spot_check": parity,
        "strong_scaling": strong, "round_trip": rt, "tx_front_end": tx, "host_fed": hostfed, "duplex": duplex,
        "bitstream_gather": gathered, "voice_crypt": side.get("crypt"), "vad": side.get("vad"),
        "modem": side.get("modem"),
    }


def side_legs(rig, wl, C, K, W, rank, world):
    """voice-frame crypt of each superframe's packets (VoiceEnc, crp.c:986,
    the TX step after melpe_a) and the VAD gate alone (vad2 x6 per
    superframe, tx.c:234-239) on the raw PCM"""
    import torch
    lib = wl.lib
    g = torch.Generator().manual_seed(RUN_SEED + rank)
    keys = torch.randint(0, 256, (C, 16), dtype=torch.uint8, generator=g).to(rig.dev)
    ctrs = torch.randint(0, 2**31, (C,), dtype=torch.int32, generator=g).to(rig.dev)
    cbits = wl.bits.clone()

    def crypt(s):
        if lib.melpe_voice_crypt_dev(cbits[s].data_ptr(), ctrs.data_ptr(), keys.data_ptr(),
                                     None, C, 1, 0, rig.sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    crypt_s, (crypt_kms,) = timed(rig, [crypt], K, W)
    del cbits
    ach = VC_OPS_PER_PACKET * C / (crypt_kms / 1e3) / 1e12
    vcrypt = {"kernel": "k_voice_crypt", "value": world * C * K / crypt_s, "unit": "packets/s",
              "kernel_ms": crypt_kms, "packets_per_launch": C,
              "roofline": {"bound": "valu", "ops_per_packet": VC_OPS_PER_PACKET,
                           "achieved": ach, "peak": PEAK_VALU_TOPS,
                           "unit": "T INT32 VALU lane-ops/s", "frac": ach / PEAK_VALU_TOPS,
                           "algorithmic_hbm_bytes_per_launch": C * (2 * SF_BYTES + 16 + 4)}}
    log("voice crypt: kernel %.3f ms per %d packets" % (crypt_kms, C))
    # the encode leg overwrote the PCM with the NPP output: regenerate the raw
    # input, which is what tx.c's vad2 sees
    wl.regen_pcm()
    vst = torch.zeros(C * lib.melpe_vad_state_bytes(), dtype=torch.uint8, device=rig.dev)
    votes = torch.zeros((W + K, C), dtype=torch.uint8, device=rig.dev)
    if lib.melpe_vad_reset_dev(vst.data_ptr(), C, None, rig.sptr):
        raise RuntimeError(lib.melpe_last_error().decode())

    def vad(s):
        if lib.melpe_vad_dev(vst.data_ptr(), wl.pcm[s].data_ptr(), votes[s].data_ptr(), C, None,
                             rig.sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    vad_s, (vad_kms,) = timed(rig, [vad], K, W)
    vgate = {"kernel": "k_vad", "value": world * C * K * SF_SECONDS / vad_s,
             "unit": "channel-s/s gated", "kernel_ms": vad_kms,
             "silent_fraction": float((votes[W:] == 0).float().mean().item()),
             "input": "raw synthetic PCM (before NPP)"}
    log("vad: kernel %.3f ms per %d channel-superframes" % (vad_kms, C))
    del vst, votes
    return {"crypt": vcrypt, "vad": vgate, "modem": modem_leg(rig, wl, C, K, W, world)}


MODEM_PKT = 3240          # 48 kHz samples per 81-bit packet (modem/modem.c:136)
MODEM_CALLS = 15          # Demodulate calls per packet time (216 samples each)


def modem_leg(rig, wl, C, K, W, world):
    """PairPhone's pseudo-voice modem on the encoded packets: Modulate (tx.c:271)
    one packet per channel per step, and Demodulate (rx.c:294) the 15 calls
    of one packet time per channel per step on the modulated streams.  Both
    are byte-moving kernels: roofline = HBM bytes / launch time."""
    import torch
    lib = wl.lib
    sb = lib.melpe_modem_state_bytes()
    st = torch.zeros(C * sb, dtype=torch.uint8, device=rig.dev)
    if lib.melpe_modem_reset_dev(st.data_ptr(), C, None, rig.sptr):
        raise RuntimeError(lib.melpe_last_error().decode())
    out = torch.empty((C, MODEM_PKT), dtype=torch.int16, device=rig.dev)

    def mod(s):
        if lib.melpe_modulate_dev(st.data_ptr(), wl.bits[s].data_ptr(), out.data_ptr(), C, 1, None,
                                  rig.sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    mod_s, (mod_kms,) = timed(rig, [mod], K, W)
    del out
    # the receive side: every channel's modulated stream of all W + K
    # packets, made before the timed region
    steps = W + K
    stride = steps * MODEM_PKT + 2048
    stream = torch.zeros((C, stride), dtype=torch.int16, device=rig.dev)
    pk = wl.bits.transpose(0, 1).contiguous()            # C x steps x 11
    if lib.melpe_modem_reset_dev(st.data_ptr(), C, None, rig.sptr):
        raise RuntimeError(lib.melpe_last_error().decode())
    if lib.melpe_modulate_dev(st.data_ptr(), pk.data_ptr(), stream.data_ptr(), C, steps, None,
                              rig.sptr):
        raise RuntimeError(lib.melpe_last_error().decode())
    # modulate wrote C x steps x 3240 contiguously; spread rows to the stride
    flat = stream.view(-1)[:C * steps * MODEM_PKT].view(C, steps * MODEM_PKT).clone()
    stream.zero_()
    stream[:, :steps * MODEM_PKT] = flat
    del flat, pk
    if lib.melpe_modem_reset_dev(st.data_ptr(), C, None, rig.sptr):
        raise RuntimeError(lib.melpe_last_error().decode())
    pos = torch.zeros(C, dtype=torch.int32, device=rig.dev)
    data = torch.zeros((C, 12), dtype=torch.uint8, device=rig.dev)

    def demod(s):
        if lib.melpe_demodulate_dev(st.data_ptr(), stream.data_ptr(), stride, pos.data_ptr(),
                                    data.data_ptr(), None, None, C, MODEM_CALLS, None, rig.sptr):
            raise RuntimeError(lib.melpe_last_error().decode())
    dem_s, (dem_kms,) = timed(rig, [demod], K, W)
    locked = float(((data[:, 11] & 0x40) > 0).float().mean().item())
    del stream
    mod_bytes = C * (SF_BYTES + 2 * MODEM_PKT)
    dem_bytes = C * MODEM_CALLS * (2 * 216 + 12) + 2 * C * sb
    res = {"modulate": {"kernel": "k_modulate", "kernel_ms": mod_kms,
                        "value": world * C * K / mod_s, "unit": "packets/s",
                        "roofline": {"bound": "hbm", "achieved": mod_bytes / (mod_kms / 1e3) / 1e9,
                                     "peak": 8000.0, "unit": "GB/s",
                                     "frac": mod_bytes / (mod_kms / 1e3) / 1e9 / 8000.0,
                                     "bytes_per_launch": mod_bytes}},
           "demodulate": {"kernel": "k_demodulate", "kernel_ms": dem_kms,
                          "value": world * C * K / dem_s, "unit": "packet times/s",
                          "calls_per_launch": MODEM_CALLS, "block_locked_fraction": locked,
                          "roofline": {"bound": "hbm", "achieved": dem_bytes / (dem_kms / 1e3) / 1e9,
                                       "peak": 8000.0, "unit": "GB/s",
                                       "frac": dem_bytes / (dem_kms / 1e3) / 1e9 / 8000.0,
                                       "bytes_per_launch": dem_bytes,
                                       "bytes_note": "unique samples + 12-byte outputs + state "
                                                     "read and write"}}}
    log("modem: modulate %.3f ms, demodulate %.3f ms per %d channels" % (mod_kms, dem_kms, C))
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(argv, args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("WORLD_SIZE %d overrides --gpus %d" % (world, args.gpus))
    line = run(args, rank, world, local)
    if line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
