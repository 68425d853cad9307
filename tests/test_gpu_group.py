"""Multi-device groups on the GPU (include/meyda_gpu.h "Multi-device groups"): a one-rank
group, single-process (mgx_group_create) and per-process (mgx_group_create_rank), run
through the chunked extraction path and must be byte-identical to one plan's extraction;
with two or more devices visible, the RCCL gather of a real multi-device group too.
Frame independence (src/meyda.js:69-91) makes every chunking and sharding legal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6D657964
FEATS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
         "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness",
         "perceptualSpread", "perceptualSharpness", "mfcc", "amplitudeSpectrum", "powerSpectrum",
         "complexSpectrum"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def _frames(capi, F, n, first=0):
    import torch
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, SEED, first_frame=first)
    return x


@pytest.mark.parametrize("mode", ["devices", "rank"])
@pytest.mark.parametrize("nch", [1, 3, 8])
def test_one_rank_group_equals_plan(capi, mode, nch):
    import torch
    n, F = 1024, 5000
    x = _frames(capi, F, n)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    want = plan.extract_torch(x, FEATS)
    if mode == "devices":
        g = capi.Group(buffer_size=n, devices=[0], scalar_f64=True)
        assert g.comm_info() == (-1, -1, -1)  # one rank: no communicator
    else:
        g = capi.Group(buffer_size=n, rank=0, nranks=1, device=0, scalar_f64=True)
    assert (g.nranks, g.first_local, g.num_local) == (1, 0, 1)
    got, o = plan.alloc_outputs(F, FEATS)
    for v in got.values():
        v.fill_(float("nan"))
    stream = torch.cuda.current_stream().cuda_stream
    g.extract_device([x.data_ptr()], [F], o, capi.output_mask(o), num_chunks=nch, streams=[stream])
    torch.cuda.synchronize()
    for k in want:
        assert torch.equal(got[k].view(torch.int32) if got[k].dtype == torch.float32 else got[k].view(torch.int64),
                           want[k].view(torch.int32) if want[k].dtype == torch.float32 else want[k].view(torch.int64)), k
    g.close()


def test_group_host_batch_equals_plan(capi):
    n, F = 512, 3001
    x = _frames(capi, F, n).cpu().numpy()
    feats = ["rms", "zcr", "spectralCentroid", "loudness", "mfcc", "amplitudeSpectrum"]
    want = capi.Plan(buffer_size=n).extract(x, feats)
    g = capi.Group(buffer_size=n, devices=[0])
    got = g.extract(x, feats)
    for k in want:
        assert np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32)), k


def test_group_argument_errors(capi):
    with pytest.raises(capi.MgxError):
        capi.Group(buffer_size=512, devices=[0, 0])  # a device twice
    with pytest.raises(capi.MgxError):
        capi.Group(buffer_size=512, rank=1, nranks=1)
    g = capi.Group(buffer_size=512, devices=[0])
    with pytest.raises(capi.MgxError):  # the root's outputs must hold every masked field
        g.extract_device([0], [0], capi.Outputs(), capi.OUT_MFCC)


@pytest.mark.parametrize("n,F", [(1024, 40000), (2048, 40003)])
def test_multi_device_gather(capi, n, F):
    """Every visible device in one process: ragged shards, 8-chunk RCCL gather to device 0 of
    every output bench.py gathers (13 scalars + loudness.specific + MFCC; at N = 2048 config
    C5's), byte-identical to one plan's extraction of the whole batch."""
    import torch
    ndev = capi.device_count()
    if ndev < 2:
        pytest.skip("one device visible: the RCCL gather needs two (covered on the multi-GPU node)")
    devs = list(range(ndev))
    g = capi.Group(buffer_size=n, devices=devs, scalar_f64=True)
    assert (g.nranks, g.first_local, g.num_local) == (len(devs), 0, len(devs))
    assert g.comm_info() == (len(devs), 0, 0)
    counts = [capi.shard_range(F, len(devs), r)[1] for r in range(len(devs))]
    starts = [capi.shard_range(F, len(devs), r)[0] for r in range(len(devs))]
    xs = []
    for d, s, c in zip(devs, starts, counts):
        with torch.cuda.device(d):
            xs.append(_frames(capi, c, n, first=s))
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    feats = capi.ALL_FEATURES
    got, o = plan.alloc_outputs(F, feats)
    for v in got.values():
        v.fill_(float("nan"))
    for dd in devs:
        torch.cuda.synchronize(dd)
    g.extract_device([t.data_ptr() for t in xs], counts, o, capi.output_mask(o), num_chunks=8)
    for dd in devs:
        torch.cuda.synchronize(dd)
    want = plan.extract_torch(_frames(capi, F, n), feats)
    torch.cuda.synchronize()
    for k in want:
        assert torch.equal(got[k].view(torch.int64) if got[k].dtype == torch.float64 else got[k].view(torch.int32),
                           want[k].view(torch.int64) if want[k].dtype == torch.float64 else want[k].view(torch.int32)), k
    g.close()


@pytest.mark.parametrize("ranks,nch", [(2, 1), (3, 8), (4, 3)])
def test_loopback_group_gather(capi, ranks, nch):
    """The gather path of a multi-rank group on one device (mgx_group_create_loopback: chunk
    transfers as device copies): ragged shards, chunks cycling through the two transfer
    slots and both compute streams, the root's unpack of every output field. Two calls on
    different frames: the second's record must not hold anything of the first's."""
    import torch
    n, F = 1024, 40001
    g = capi.Group(buffer_size=n, loopback=ranks, scalar_f64=True)
    assert (g.nranks, g.first_local, g.num_local) == (ranks, 0, ranks)
    counts = [capi.shard_range(F, ranks, r)[1] for r in range(ranks)]
    starts = [capi.shard_range(F, ranks, r)[0] for r in range(ranks)]
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    got, o = plan.alloc_outputs(F, FEATS)
    stream = torch.cuda.current_stream().cuda_stream
    for seed_shift in (0, 7919):
        xs = [_frames(capi, c, n, first=s + seed_shift) for s, c in zip(starts, counts)]
        for v in got.values():
            v.fill_(float("nan"))
        g.extract_device([t.data_ptr() for t in xs], counts, o, capi.output_mask(o), num_chunks=nch,
                         streams=[stream] * ranks)
        torch.cuda.synchronize()
        want = plan.extract_torch(_frames(capi, F, n, first=seed_shift), FEATS)
        torch.cuda.synchronize()
        for k in want:
            a = got[k].view(torch.int32) if got[k].dtype == torch.float32 else got[k].view(torch.int64)
            b = want[k].view(torch.int32) if want[k].dtype == torch.float32 else want[k].view(torch.int64)
            assert torch.equal(a, b), (k, seed_shift)
    g.close()


@pytest.mark.parametrize("ranks,nch,n", [(2, 1, 1024), (3, 8, 1024), (4, 3, 2048)])
def test_rccl_transport_group_gather(capi, ranks, nch, n):
    """The RCCL transport on one GPU (mgx_group_create_loopback_rccl): every peer chunk crosses
    as ncclSend / ncclRecv on a one-rank communicator (to and from itself) through group.cpp's
    chunk loop, transfer slots and root unpack. The gathered record must be byte-identical to
    one plan's extraction, for two calls on different frames, and the communicator must
    report itself (one rank, rank 0, this device)."""
    import torch
    F = 40001 if n == 1024 else 20011
    g = capi.Group(buffer_size=n, loopback=ranks, transport="rccl", scalar_f64=True)
    assert (g.nranks, g.first_local, g.num_local) == (ranks, 0, ranks)
    assert g.comm_info() == (1, 0, torch.cuda.current_device())
    counts = [capi.shard_range(F, ranks, r)[1] for r in range(ranks)]
    starts = [capi.shard_range(F, ranks, r)[0] for r in range(ranks)]
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    got, o = plan.alloc_outputs(F, FEATS)
    stream = torch.cuda.current_stream().cuda_stream
    for seed_shift in (0, 7919):
        xs = [_frames(capi, c, n, first=s + seed_shift) for s, c in zip(starts, counts)]
        for v in got.values():
            v.fill_(float("nan"))
        g.extract_device([t.data_ptr() for t in xs], counts, o, capi.output_mask(o), num_chunks=nch,
                         streams=[stream] * ranks)
        torch.cuda.synchronize()
        want = plan.extract_torch(_frames(capi, F, n, first=seed_shift), FEATS)
        torch.cuda.synchronize()
        for k in want:
            a = got[k].view(torch.int32) if got[k].dtype == torch.float32 else got[k].view(torch.int64)
            b = want[k].view(torch.int32) if want[k].dtype == torch.float32 else want[k].view(torch.int64)
            assert torch.equal(a, b), (k, seed_shift)
    g.close()


def test_rccl_transport_pipelined_steps(capi):
    """bench.py's multi-rank step shape on the RCCL transport: consecutive group calls
    alternating between two streams and two output sets, no host wait between them."""
    import torch
    n, F, ranks = 1024, 65536 + 7, 3
    g = capi.Group(buffer_size=n, loopback=ranks, transport="rccl")
    counts = [capi.shard_range(F, ranks, r)[1] for r in range(ranks)]
    starts = [capi.shard_range(F, ranks, r)[0] for r in range(ranks)]
    plan = capi.Plan(buffer_size=n)
    feats = capi.ALL_FEATURES
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    calls = []
    for shift in (0, 104729, 7919, 31):
        got, o = plan.alloc_outputs(F, feats)
        calls.append((shift, got, o, [_frames(capi, c, n, first=s + shift) for s, c in zip(starts, counts)]))
    torch.cuda.synchronize()
    for i, (_, _, o, xs) in enumerate(calls):
        st = streams[i & 1].cuda_stream
        g.extract_device([t.data_ptr() for t in xs], counts, o, capi.output_mask(o), num_chunks=8, streams=[st] * ranks)
    torch.cuda.synchronize()
    for shift, got, _, _ in calls:
        want = plan.extract_torch(_frames(capi, F, n, first=shift), feats)
        torch.cuda.synchronize()
        for k in want:
            assert torch.equal(got[k].view(torch.int32), want[k].view(torch.int32)), (k, shift)
    g.close()


@pytest.mark.parametrize("ranks,nch", [(2, 8), (3, 3)])
def test_loopback_group_calls_overlap_on_two_streams(capi, ranks, nch):
    """Consecutive group calls on two different streams (as bench.py pipelines its steps): the
    second call's first chunks reuse the transfer slots of the first call's last ones, so they
    must wait for those sends; both records must match one plan's extraction byte for byte."""
    import torch
    n, F = 1024, 30011
    g = capi.Group(buffer_size=n, loopback=ranks, scalar_f64=True)
    counts = [capi.shard_range(F, ranks, r)[1] for r in range(ranks)]
    starts = [capi.shard_range(F, ranks, r)[0] for r in range(ranks)]
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    shifts = (0, 7919, 104729)
    calls = []
    for shift in shifts:
        got, o = plan.alloc_outputs(F, FEATS)
        for v in got.values():
            v.fill_(float("nan"))
        calls.append((shift, got, o, [_frames(capi, c, n, first=s + shift) for s, c in zip(starts, counts)]))
    torch.cuda.synchronize()
    for i, (shift, got, o, xs) in enumerate(calls):  # issued back to back, no host wait between
        st = streams[i & 1].cuda_stream
        g.extract_device([t.data_ptr() for t in xs], counts, o, capi.output_mask(o), num_chunks=nch,
                         streams=[st] * ranks)
    torch.cuda.synchronize()
    outs = [(shift, got) for shift, got, _, _ in calls]
    for shift, got in outs:
        want = plan.extract_torch(_frames(capi, F, n, first=shift), FEATS)
        torch.cuda.synchronize()
        for k in want:
            a = got[k].view(torch.int32) if got[k].dtype == torch.float32 else got[k].view(torch.int64)
            b = want[k].view(torch.int32) if want[k].dtype == torch.float32 else want[k].view(torch.int64)
            assert torch.equal(a, b), (k, shift)
    g.close()


@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_plan_launches_pipelined_on_two_streams(capi, n):
    """One plan, consecutive launches alternating between two streams with their own outputs
    (bench.py's pipelined steps): the launches run concurrently and each record
    equals the same batch extracted alone, bit for bit."""
    import torch
    F = 65536 + 37
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    calls = []
    for i in range(4):
        got, o = plan.alloc_outputs(F, FEATS)
        calls.append((got, o, _frames(capi, F, n, first=i * 1009)))
    torch.cuda.synchronize()
    ev = torch.cuda.Event()
    ev.record(streams[0])
    streams[1].wait_event(ev)
    for i, (_, o, x) in enumerate(calls):  # issued back to back
        plan.extract_device(x.data_ptr(), F, o, streams[i & 1].cuda_stream)
    torch.cuda.synchronize()
    for i, (got, _, x) in enumerate(calls):
        want = plan.extract_torch(x, FEATS)
        torch.cuda.synchronize()
        for k in want:
            a = got[k].view(torch.int32) if got[k].dtype == torch.float32 else got[k].view(torch.int64)
            b = want[k].view(torch.int32) if want[k].dtype == torch.float32 else want[k].view(torch.int64)
            assert torch.equal(a, b), (k, i)


def _ipc_rank(rank, nranks, uid, n, calls, q):
    """One process of the cross-process rehearsal (MGX_GROUP_TRANSPORT=ipc, every rank on device 0):
    its shard of each call's frames through mgx_group_create_rank's group; the root compares the
    gathered record with one plan's extraction of the whole batch, byte for byte."""
    import os
    os.environ["MGX_GROUP_TRANSPORT"] = "ipc"
    os.environ["MGX_IPC_TIMEOUT_S"] = "60"
    try:
        import torch
        from meyda_amd import capi
        g = capi.Group(buffer_size=n, rank=rank, nranks=nranks, unique_id=uid, device=0, scalar_f64=True)
        assert (g.nranks, g.first_local, g.num_local) == (nranks, rank, 1)
        assert g.comm_info() == (nranks, rank, 0), g.comm_info()
        plan = capi.Plan(buffer_size=n, scalar_f64=True)
        feats = FEATS
        bad = []
        for F, first, nch in calls:
            counts = [capi.shard_range(F, nranks, r)[1] for r in range(nranks)]
            s0 = capi.shard_range(F, nranks, rank)[0]
            x = torch.empty(counts[rank], n, dtype=torch.float32, device="cuda")
            capi.synth_frames_device(x, SEED, first_frame=first + s0)
            got, o = plan.alloc_outputs(F if rank == 0 else 1, feats)
            for v in got.values():
                v.fill_(float("nan"))
            torch.cuda.synchronize()
            g.extract_device([x.data_ptr()], counts, o if rank == 0 else None, capi.output_mask(o), num_chunks=nch)
            torch.cuda.synchronize()
            if rank == 0:
                xa = torch.empty(F, n, dtype=torch.float32, device="cuda")
                capi.synth_frames_device(xa, SEED, first_frame=first)
                want = plan.extract_torch(xa, feats)
                torch.cuda.synchronize()
                for k in want:
                    a = got[k].view(torch.int64) if got[k].dtype == torch.float64 else got[k].view(torch.int32)
                    b = want[k].view(torch.int64) if want[k].dtype == torch.float64 else want[k].view(torch.int32)
                    if not torch.equal(a, b):
                        bad.append((F, nch, k))
        g.close()
        q.put((rank, "ok" if not bad else "mismatch %s" % bad[:5]))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, "error %r" % (e,)))


@pytest.mark.parametrize("n", [1024, 2048])
def test_ipc_transport_two_processes(capi, n):
    """The cross-process gather rehearsed on one GPU: two processes, each with its own plan and
    mgx_group_create_rank group, the chunks moving through hipIpcGetMemHandle / hipIpcOpenMemHandle
    and a shared-memory mailbox in place of ncclSend / ncclRecv (MGX_GROUP_TRANSPORT=ipc). This is
    the code a multi-GPU torchrun job runs -- per-rank group creation, ragged shards, the chunk
    loop over two transfer slots on two compute streams, slot reuse across calls, the root's
    unpack -- across a process boundary. Three calls: 8 chunks, then fewer frames (slot reuse),
    then more (the peer reallocates and republishes its transfer buffer); byte-identical to one
    plan's extraction every time."""
    import multiprocessing as mp
    import os
    os.environ["MGX_GROUP_TRANSPORT"] = "ipc"
    try:
        uid = capi.comm_unique_id()
    finally:
        del os.environ["MGX_GROUP_TRANSPORT"]
    assert uid.startswith(b"mgx-ipc:")
    calls = [(40003, 0, 8), (9001, 50000, 3), (70001, 100000, 8)] if n == 1024 else [(20003, 0, 8), (5001, 30000, 2), (36001, 40000, 8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ipc_rank, args=(r, 2, uid, n, calls, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    try:
        for _ in ps:
            res.append(q.get(timeout=150))
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert sorted(res) == [(0, "ok"), (1, "ok")], res
