"""Non-temporal frame loads (plan.cpp KernelArgs::nt_frames, kernels.hip ld_frame): a batch larger than
the MALL reads its frames past the caches, a smaller one with plain loads. Both branches of every kernel
must compute the same bytes; MGX_NT_MIN_MB forces either on batches of any size.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALL = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff",
       "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness", "perceptualSpread",
       "perceptualSharpness", "mfcc", "amplitudeSpectrum"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def plan(capi, nt_min_mb, **kw):
    old = os.environ.get("MGX_NT_MIN_MB")
    os.environ["MGX_NT_MIN_MB"] = str(nt_min_mb)
    try:
        return capi.Plan(**kw)
    finally:
        if old is None:
            del os.environ["MGX_NT_MIN_MB"]
        else:
            os.environ["MGX_NT_MIN_MB"] = old


@pytest.mark.parametrize("n", [256, 512, 1024, 2048])
@pytest.mark.parametrize("kw", [{}, {"mfcc_reference": True}])
def test_nt_and_plain_frame_loads_agree(capi, n, kw):
    import torch
    F = 5000  # not a multiple of the 16-frame groups
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    x[7].fill_(float("nan"))
    x[9].zero_()
    always = plan(capi, 0, buffer_size=n, **kw)       # every batch past 0 MiB: non-temporal
    never = plan(capi, 1 << 20, buffer_size=n, **kw)  # no batch past 1 TiB: plain loads
    try:
        a = always.extract_torch(x, ALL)
        b = never.extract_torch(x, ALL)
        torch.cuda.synchronize()
        for k in a:
            u, v = a[k].cpu().numpy(), b[k].cpu().numpy()
            assert np.array_equal(u.view(np.uint8), v.view(np.uint8)), (n, kw, k)
    finally:
        always.close()
        never.close()
