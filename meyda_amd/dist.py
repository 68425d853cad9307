"""Multi-GPU sharding of the frame stream: one process per GPU (torch.distributed).

Frames are independent (the reference keeps no cross-buffer state,
src/meyda.js:69-91), so a batch of F frames is cut into contiguous per-rank
shards and each rank runs the fused extraction on its own shard with no data
exchange (weak scaling). The only collective is the optional gather of the
per-frame feature vectors (SoA) to one rank, for consumers that want the whole
batch in one place; on MI355X it runs over RCCL/xGMI
(backend "nccl"), and on CPU over gloo (the tests).
"""
import os

import torch
import torch.distributed as dist


def env_rank_world():
    """(rank, local_rank, world_size) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_range(total, world, rank):
    """Contiguous shard [start, start + count) of `total` frames for `rank`; the first
    `total % world` ranks get one extra frame, so shards differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d out of range for world size %d" % (rank, world))
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def init(backend=None):
    """Initialise the default process group from the environment (MASTER_ADDR=127.0.0.1
    is the caller's job). Returns (rank, local_rank, world); a no-op for world 1."""
    rank, local, world = env_rank_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, local, world


def gather_features(outs, counts, dst=0, group=None):
    """Gather each rank's SoA feature tensors to rank `dst`.

    outs:   {name: tensor[count_r, ...]} on this rank (same names and trailing shapes
            on every rank, as produced by Plan.alloc_outputs for one feature list).
    counts: frames per rank (shard_range counts), identical on every rank.
    Returns {name: tensor[sum(counts), ...]} on `dst` (frames in rank order), None elsewhere.
    Shards may be ragged; they are padded to max(counts) for the collective.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world:
        raise ValueError("counts has %d entries for world size %d" % (len(counts), world))
    cmax = max(counts)
    result = {} if rank == dst else None
    for name in sorted(outs):
        t = outs[name]
        if t.shape[0] != counts[rank]:
            raise ValueError("%s has %d frames, shard has %d" % (name, t.shape[0], counts[rank]))
        if t.shape[0] < cmax:
            pad = torch.zeros((cmax - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            t = torch.cat([t, pad])
        t = t.contiguous()
        bufs = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, bufs, dst=dst, group=group)
        if rank == dst:
            result[name] = torch.cat([b[:c] for b, c in zip(bufs, counts)])
    return result
