"""Static channel sharding across GPUs and the end-of-run bitstream gather.

SURVEY.md §8(e): channels are independent and a channel's superframes are
sequential, so rank r of W owns the contiguous channel range
channel_range(r, W, C).  Nothing is exchanged while encoding; after the
timed region each rank's bitstreams (steps x channels x 11 bytes) are
gathered to every rank (rank 0 writes them) with one all_gather over the
process group (RCCL over xGMI on GPUs, gloo on CPU).  Ragged shards (the
last rank holding fewer channels) are padded to the largest shard for the
collective and trimmed after it.
"""
import torch
import torch.distributed as dist

SF_BYTES = 11


def channel_range(rank, world, channels):
    """[lo, hi) of the channels rank `rank` of `world` owns (balanced,
    contiguous; the first channels % world ranks get one more)."""
    if world <= 0 or not 0 <= rank < world or channels < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(channels, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def superframe_range(rank, world, lengths):
    """Ragged streams (BASELINE config 5): channels with `lengths[c]`
    superframes each, split into contiguous ranges of roughly equal total
    superframes.  Returns [lo, hi) for `rank`."""
    total = int(sum(lengths))
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad shard request")
    bounds, acc, c = [0], 0, 0
    for r in range(1, world):
        target = (total * r) // world
        while c < len(lengths) and acc + lengths[c] <= target:
            acc += lengths[c]
            c += 1
        bounds.append(c)
    bounds.append(len(lengths))
    return bounds[rank], bounds[rank + 1]


def gather_bitstreams(bits, channels_total):
    """bits: uint8 tensor [steps, local_channels, 11] of this rank, in rank
    order of channel_range.  Returns the [steps, channels_total, 11] tensor of
    all ranks (on every rank), on bits.device."""
    if bits.dim() != 3 or bits.shape[2] != SF_BYTES or bits.dtype != torch.uint8:
        raise ValueError("bits must be uint8 [steps, channels, 11]")
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        if bits.shape[1] != channels_total:
            raise ValueError("single rank must hold every channel")
        return bits
    world = dist.get_world_size()
    steps = bits.shape[0]
    sizes = [channel_range(r, world, channels_total) for r in range(world)]
    width = max(hi - lo for lo, hi in sizes)
    mine = sizes[dist.get_rank()]
    if bits.shape[1] != mine[1] - mine[0]:
        raise ValueError("local shard has %d channels, expected %d"
                         % (bits.shape[1], mine[1] - mine[0]))
    # RCCL gathers device tensors over xGMI; gloo (CPU ranks, or ranks that
    # share one GPU in the tests) gathers host tensors
    on = bits.device if dist.get_backend() != "gloo" else torch.device("cpu")
    pad = torch.zeros((steps, width, SF_BYTES), dtype=torch.uint8, device=on)
    pad[:, :bits.shape[1]] = bits.to(on)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:, :hi - lo] for p, (lo, hi) in zip(parts, sizes)], dim=1).to(bits.device)
