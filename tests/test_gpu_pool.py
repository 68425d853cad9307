"""The N = 2048 tail pool (kernels.hip: the last pool_pct percent of a launch's groups taken one
batch per ticket from a per-stream device counter) against the same plan with the pool off.

Every frame must be computed exactly once whatever the launch order -- the reference handles each
buffer on its own (src/meyda.js:69-91), so a batch that a ticket skipped would be a frame with no
features. The counter is reset on the device by the wave that draws a launch's last ticket, so
consecutive launches of different sizes on one stream, and a launch captured into a HIP graph and
replayed, must each give the pool-off plan's bytes. Outputs are pre-filled with NaN before every
launch / replay, so a batch that was not computed cannot pass as a stale copy of a previous one.
"""
import os

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6D657964
N = 2048
FEATS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
         "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness",
         "perceptualSpread", "perceptualSharpness", "mfcc"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def make_plan(capi, pct, **kw):
    old = os.environ.get("MGX_POOL_PCT")
    os.environ["MGX_POOL_PCT"] = str(pct)
    try:
        return capi.Plan(buffer_size=N, **kw)
    finally:
        if old is None:
            del os.environ["MGX_POOL_PCT"]
        else:
            os.environ["MGX_POOL_PCT"] = old


def run(plan, frames, F, feats, stream):
    import torch
    out, o = plan.alloc_outputs(F, feats, device=frames.device)
    for t in out.values():
        t.fill_(float("nan"))
    plan.extract_device(frames.data_ptr(), F, o, stream.cuda_stream)
    return out


def same(a, b):
    import torch
    for k in a:
        x, y = a[k], b[k]
        assert x.shape == y.shape, k
        # bit patterns: NaN never equals NaN, so an uncomputed entry fails here
        xb = x.view(torch.int64 if x.dtype == torch.float64 else torch.int32)
        yb = y.view(torch.int64 if y.dtype == torch.float64 else torch.int32)
        bad = (xb != yb).nonzero()
        assert bad.numel() == 0, (k, bad[:4].tolist(), int(bad.shape[0]))


@pytest.mark.parametrize("pct", [15, 50])
def test_pool_launch_sequence_one_stream(capi, pct):
    """Five launches of different frame counts back to back on one stream (counts not multiples of 4
    or 16; large ones defer their scalars to the per-wave windows, small ones do not), each
    byte-identical to the pool-off plan."""
    import torch
    Fmax = 200003
    frames = torch.empty(Fmax, N, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, SEED)
    off = make_plan(capi, 0)
    on = make_plan(capi, pct)
    s = torch.cuda.Stream()
    sizes = [200003, 4099, 131075, 65538, 1001, 200003]
    ref = {}
    for F in sorted(set(sizes)):
        ref[F] = run(off, frames, F, FEATS, s)
    got = [run(on, frames, F, FEATS, s) for F in sizes]  # queued back to back, no sync between
    torch.cuda.synchronize()
    for F, g in zip(sizes, got):
        same(g, ref[F])
    off.close()
    on.close()


def test_pool_graph_replay(capi):
    """One launch captured into a HIP graph and replayed four times: every replay computes every frame
    (the pool's tickets start from 0 each time), byte-identical to the pool-off plan."""
    import torch
    F = 150001
    frames = torch.empty(F, N, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, SEED, first_frame=7 * F)
    off = make_plan(capi, 0, scalar_f64=True)
    on = make_plan(capi, 15, scalar_f64=True)
    s = torch.cuda.Stream()
    ref = run(off, frames, F, FEATS + ["amplitudeSpectrum"], s)
    # the stream's scratch set comes from a first, uncaptured call (include/meyda_gpu.h)
    warm = run(on, frames, 64, FEATS, s)
    torch.cuda.synchronize()
    out, o = on.alloc_outputs(F, FEATS + ["amplitudeSpectrum"], device=frames.device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        on.extract_device(frames.data_ptr(), F, o, s.cuda_stream)
    torch.cuda.synchronize()
    for rep in range(4):
        for t in out.values():
            t.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        same(out, ref)
    del warm
    g.reset()
    off.close()
    on.close()
