"""Multi-GPU path on CPU: static channel shards and the end-of-run bitstream
gather (pairphone_amd/shard.py), world size 2 over gloo, plus the bench's
max-over-ranks timing line with --gpus 2 semantics."""
import os
import socket

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
