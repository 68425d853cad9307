"""Process topology of a multi-GPU run: one process per GPU (torchrun), torch.distributed
(gloo) as the control plane only.

Frames are independent (the reference keeps no cross-buffer state, src/meyda.js:69-91),
so a batch of F frames is cut into contiguous per-rank shards and each rank runs the fused
extraction on its own shard. The one data exchange -- the gather of the per-frame feature
records to rank 0 over RCCL/xGMI -- is the library's own (include/meyda_gpu.h
"Multi-device groups", meyda_amd/csrc/group.cpp, capi.Group); this module only reads the
launcher's environment and starts the control-plane process group (the RCCL unique id
broadcast, barriers, the max-over-ranks timing).
"""
import os

import torch.distributed as dist


def env_rank_world(env=None):
    """(rank, local_rank, world_size) from the torchrun environment (1 process if unset)."""
    env = os.environ if env is None else env
    return (int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0")), int(env.get("WORLD_SIZE", "1")))


def shard_range(total, world, rank):
    """Contiguous shard [start, start + count) of `total` frames for `rank`; the first
    `total % world` ranks get one extra frame, so shards differ by at most one (the Python
    statement of mgx_shard_range, checked against it in tests/test_group_host.py)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d out of range for world size %d" % (rank, world))
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def init_control_plane():
    """The gloo process group of a torchrun launch (MASTER_ADDR=127.0.0.1 is the caller's
    job). Returns (rank, local_rank, world); a no-op for world 1."""
    rank, local, world = env_rank_world()
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo")
    return rank, local, world
