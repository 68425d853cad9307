"""BASELINE config C5 on one GPU: the per-GPU shard of the 8-GPU job (262,144 frames of
bufferSize = 2048, every feature including MFCC), synthesised in HBM. (The RCCL gather of
the sharded records is tests/test_gpu_group.py::test_rccl_transport_group_gather.)

Reference path: lib/jsfft/fft.js:123-171 at N = 2048 (widths up to 1024), the extractors
src/extractors/*.js, and the per-buffer independence that makes frame sharding legal
(src/meyda.js:69-91). Sampled frames are checked against the CPU oracle (tests/tolerance.py
bars); the whole shard through size-independent properties and launch-to-launch
determinism.
"""
import numpy as np
import pytest

import tolerance

pytestmark = pytest.mark.gpu

SEED = 0x6D657964
FEATS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
         "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness",
         "perceptualSpread", "perceptualSharpness", "mfcc", "amplitudeSpectrum"]
SCALARS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
           "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis",
           "loudness.total", "perceptualSpread", "perceptualSharpness"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def test_c5_shard_2048_all_features(capi, oracle_mod):
    import torch
    n, F = 2048, 262144
    # rank 3 of 8: the shard starts at global frame 3 * 262,144 of the synthetic stream
    first = 3 * F
    frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, SEED, first_frame=first)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    out = plan.extract_torch(frames, FEATS)
    torch.cuda.synchronize()
    pick = np.array([0, 1, 2, 3, 63, 64, 1000, 32767, 131072, 199999, F - 2, F - 1])
    pt = torch.as_tensor(pick, device="cuda")
    xs = frames[pt].cpu().numpy()
    assert np.array_equal(xs[0].view(np.uint32), oracle_mod.synth_frames(SEED, first, 1, n)[0].view(np.uint32))
    ref = oracle_mod.extract(xs)
    got = {k: v[pt].cpu().numpy() for k, v in out.items()}
    bad, exact = tolerance.check_spectra(got["amplitudeSpectrum"], ref["amp"])
    assert not bad and exact == 1.0, (bad, exact)
    gs = np.stack([got[k].astype(np.float64) for k in SCALARS], 1)
    fails = tolerance.check_scalars(gs, ref["scalars"], ref["amp"], n)
    assert not fails, fails[:10]
    assert np.array_equal(got["zcr"], ref["scalars"][:, 2])
    assert not tolerance.check_vectors(got["mfcc"], ref["mfcc"])
    assert not tolerance.check_vectors(got["loudness.specific"], ref["loudness_specific"])
    # properties over the whole shard
    z = out["zcr"]
    assert torch.all((z >= 0) & (z <= n - 1))
    for k in ("mfcc", "loudness.specific", "spectralCentroid", "spectralKurtosis", "perceptualSharpness"):
        assert torch.all(torch.isfinite(out[k])), k
    rms = out["rms"]
    assert torch.allclose(rms * rms * n, out["energy"], rtol=1e-12)
    c = out["spectralCentroid"]
    assert torch.all((c > 0) & (c < n // 2))
    # a second launch is bitwise identical (deterministic: the N = 2048 tail pool takes its batches by
    # ticket, but each batch is computed once by one wave, whichever; tests/test_gpu_pool.py)
    out2 = plan.extract_torch(frames, ["amplitudeSpectrum", "mfcc", "spectralRolloff", "loudness"])
    torch.cuda.synchronize()
    for k in ("amplitudeSpectrum", "mfcc", "spectralRolloff", "loudness.specific"):
        assert torch.equal(out2[k], out[k]), k
