"""Multi-process tests of the frame sharding and the feature gather (CPU, gloo, world 2).

The GPU extraction itself cannot run here; each rank computes its shard's features
with the CPU oracle as the stand-in producer, and rank 0 checks that the gathered
SoA record equals one single-process extraction of the whole batch. This is the
same code path bench.py / the GPU job use (meyda_amd.dist), minus the device.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_covers_exactly():
    from meyda_amd.dist import shard_range
    for total in (0, 1, 7, 64, 262144, 2097152 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _worker(rank, world, port, total, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    try:
        from meyda_amd import SEED
        from meyda_amd.dist import gather_features, init, shard_range
        from oracle import oracle
        r, _, w = init(backend="gloo")
        assert (r, w) == (rank, world)
        start, count = shard_range(total, world, rank)
        x = oracle.synth_frames(SEED, start, count, n)  # this rank's shard of the global stream
        ref = oracle.extract(x)
        outs = {"scalars": torch.from_numpy(np.ascontiguousarray(ref["scalars"])),
                "mfcc": torch.from_numpy(np.ascontiguousarray(ref["mfcc"])),
                "loudness.specific": torch.from_numpy(np.ascontiguousarray(ref["loudness_specific"]))}
        counts = [shard_range(total, world, i)[1] for i in range(world)]
        got = gather_features(outs, counts, dst=0)
        if rank == 0:
            whole = oracle.extract(oracle.synth_frames(SEED, 0, total, n))
            ok = (np.array_equal(got["scalars"].numpy(), whole["scalars"], equal_nan=True)
                  and np.array_equal(got["mfcc"].numpy(), whole["mfcc"], equal_nan=True)
                  and np.array_equal(got["loudness.specific"].numpy(), whole["loudness_specific"], equal_nan=True)
                  and got["scalars"].shape[0] == total)
            q.put(("ok" if ok else "mismatch", rank))
        else:
            q.put(("ok" if got is None else "unexpected result", rank))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put(("error: %r" % (e,), rank))


@pytest.mark.parametrize("total", [64, 67])  # even and ragged shards
def test_gather_world2_matches_single_process(total):
    world, n = 2, 512
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res, key=lambda t: t[1]) == [("ok", 0), ("ok", 1)], res
