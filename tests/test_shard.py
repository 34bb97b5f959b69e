"""Multi-GPU path on CPU: static channel shards and the end-of-run bitstream
gather (pairphone_amd/shard.py), world size 2 over gloo, plus the bench's
max-over-ranks timing line with --gpus 2 semantics."""
import os
import queue
import socket
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pairphone_amd.shard import channel_range, superframe_range, gather_bitstreams


def test_channel_range_partitions():
    for C in (0, 1, 7, 1024, 262144, 262147):
        for W in (1, 2, 3, 4, 8):
            got = [channel_range(r, W, C) for r in range(W)]
            assert got[0][0] == 0 and got[-1][1] == C
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


def test_superframe_range_balances_ragged():
    import numpy as np
    lengths = np.random.default_rng(5).integers(15, 297, 1000)
    W = 4
    got = [superframe_range(r, W, lengths) for r in range(W)]
    assert got[0][0] == 0 and got[-1][1] == len(lengths)
    loads = [int(lengths[a:b].sum()) for a, b in got]
    assert max(loads) - min(loads) <= 2 * int(lengths.max())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, C, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = channel_range(rank, world, C)
    # each rank "encodes" its own channels: byte = f(step, global channel)
    g = torch.arange(lo, hi, dtype=torch.int64)
    bits = torch.stack([((g[:, None] * 31 + s * 7 + torch.arange(11)) % 251).to(torch.uint8)
                        for s in range(steps)])
    allbits = gather_bitstreams(bits, C)
    # max-over-ranks timing, as bench.py does
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((allbits.numpy().copy(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("C", [10, 11])
def test_gather_world2_gloo(C):
    steps, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, C, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.arange(C, dtype=torch.int64)
    want = torch.stack([((g[:, None] * 31 + s * 7 + torch.arange(11)) % 251).to(torch.uint8)
                        for s in range(steps)]).numpy()
    assert (got == want).all()
    assert tmax == 2.0


class CpuRig:
    """bench.GpuRig's interface on the CPU (perf_counter events, gloo)"""

    def __init__(self, local, world):
        import torch
        self.torch, self.dist, self.world = torch, dist, world
        self.dev = torch.device("cpu")

    def sync(self):
        pass

    def event(self):
        return [0.0]

    def record(self, ev):
        import time
        ev[0] = time.perf_counter()

    @staticmethod
    def elapsed_ms(a, b):
        return 1e3 * (b[0] - a[0])

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def max_over_ranks(self, x):
        t = torch.tensor([x], dtype=torch.float64)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


class FakeWorkload:
    """stands in for the engine where there is no GPU: 'encodes' a channel's
    superframe s into bytes that depend only on (global channel, s)"""

    def __init__(self, rig, C, first, steps):
        self.C, self.first, self.steps = C, first, steps
        self.bits = torch.zeros((steps, C, 11), dtype=torch.uint8)
        self.calls = []

    def npp(self, s):
        self.calls.append(("npp", s))

    def ana(self, s):
        g = torch.arange(self.first, self.first + self.C, dtype=torch.int64)
        self.bits[s] = ((g[:, None] * 31 + s * 7 + torch.arange(11)) % 251).to(torch.uint8)

    def pipe(self, s, nxt):
        self.ana(s)
        if nxt is not None:
            self.npp(nxt)

    def restart(self):
        self.bits.zero_()

    def dec(self, s):
        pass

    def close(self):
        pass


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import pairphone_amd.shard as shard
    got = {}
    real = shard.gather_bitstreams

    def spy(bits, total):
        out = real(bits, total)
        got["all"] = out.clone()
        return out
    shard.gather_bitstreams = spy
    args = bench.parse(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--channels", "5",
                        "--total-channels", "13", "--tx-channels", "0", "--no-side-legs",
                        "--no-cpu-baseline"])
    line = bench.run(args, rank, world, rank, rig_cls=CpuRig, workload_cls=FakeWorkload)
    if rank == 0:
        q.put((line, got["all"].numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_run_world2_gloo():
    """bench.run itself on two gloo ranks (engine stubbed on the CPU): the
    JSON line has n_gpus 2, the weak value counts both ranks' channels, the
    strong leg splits --total-channels with channel_range, and the gathered
    bitstreams are every rank's channels in global order"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    line, allbits = _collect(procs, q, 180)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["channels_total"] == 10
    assert abs(line["value"] - 10 * 3 * 0.0675 / (line["ms_per_step"] * 3 / 1e3)) < 1e-6 * line["value"]
    st = line["strong_scaling"]
    assert st["total_channels"] == 13 and st["channels_per_gpu_max"] == 7
    assert line["bitstream_gather"]["collective"] == "all_gather"
    g = torch.arange(10, dtype=torch.int64)
    want = torch.stack([((g[:, None] * 31 + s * 7 + torch.arange(11)) % 251).to(torch.uint8)
                        for s in range(1, 4)]).numpy()
    assert allbits.shape == (3, 10, 11) and (allbits == want).all()


def _gpu_bench_worker(rank, world, port, C, q):
    """one rank of bench.run with the real engine; every rank on GPU 0 (the
    one-GPU box), collectives over gloo"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import pairphone_amd.shard as shard

    class SharedGpuRig(bench.GpuRig):
        def __init__(self, local, world):
            super().__init__(0, world)

        def max_over_ranks(self, x):
            t = torch.tensor([x], dtype=torch.float64)
            if self.world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
    got = {}
    real = shard.gather_bitstreams

    def spy(bits, total):
        out = real(bits, total)
        got["all"] = out.cpu().clone()
        return out
    shard.gather_bitstreams = spy
    args = bench.parse(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--channels", str(C),
                        "--total-channels", "0", "--tx-channels", "0", "--no-side-legs",
                        "--no-cpu-baseline", "--no-decode"])
    line = bench.run(args, rank, world, rank, backend="gloo", rig_cls=SharedGpuRig)
    if rank == 0:
        q.put((line, got["all"].numpy().copy()))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _collect(procs, q, limit):
    """rank 0's result from q; fails at once (instead of waiting out the
    limit) when a rank exits without one"""
    t0 = time.monotonic()
    while True:
        try:
            res = q.get(timeout=2)
            break
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, "a rank exited with %s before rank 0's result" % dead
            assert time.monotonic() - t0 < limit, "no result within %d s" % limit
            print("[test_shard] waiting for the ranks (%.0f s)" % (time.monotonic() - t0),
                  file=sys.stderr, flush=True)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _spawn_bench(world, C):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_bench_worker, args=(r, world, port, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    return _collect(procs, q, 240)


@pytest.mark.gpu
def test_bench_run_world2_real_engine():
    """bench.run on two processes with the real engine (one engine per
    process, both on GPU 0 of the box, gloo in place of RCCL): the line
    counts both ranks, and the gathered bitstreams of 2 x 2,048 channels are
    the bits a one-rank run of the same 4,096 channels produces."""
    line2, bits2 = _spawn_bench(2, 2048)
    line1, bits1 = _spawn_bench(1, 4096)
    assert line2["n_gpus"] == 2 and line2["config"]["channels_total"] == 4096
    assert line2["bitstream_gather"]["collective"] == "all_gather"
    assert bits2.shape == bits1.shape == (3, 4096, 11)
    assert (bits2 == bits1).all()
    assert bits1.any()
