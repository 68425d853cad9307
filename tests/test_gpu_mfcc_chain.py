"""MGX_FLAG_MFCC_REFERENCE at N <= 1024: the mel band sums as serial chains in the reference's
own order over the wave batch's power rows (kernels.hip mel_chains, plan.cpp chain_schedule),
the log in double, the DCT. Every coefficient must be bit-identical to the reference wherever
the amplitude spectrum is (mfcc.js:53-93 run as written), within 1e-5 per element with no norm
floor everywhere, on every instance that takes the flag (all features, subsets), on edge frames
(NaN / Inf / overflow / denormals: the non-finite frames keep the reference's bin-by-bin sums)
and for every mel band count."""
import numpy as np
import pytest

import golden_io
import tolerance
from test_gpu_edge import FEATS, compare, edge_frames
from test_gpu_parity import _mfcc_reference_checks

pytestmark = pytest.mark.gpu

CHAIN_SIZES = [256, 512, 1024, 2048]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def _frames(oracle_mod, n, count, seed):
    rng = np.random.default_rng(seed)
    x = oracle_mod.synth_frames(0x6D657964, seed, count, n).copy()
    t = np.arange(n) / 44100.0
    for i in range(0, count, 3):
        x[i] = (rng.uniform(0.01, 0.9) * np.sin(2 * np.pi * rng.uniform(30, 18000) * t)).astype(np.float32)
    return x


@pytest.mark.parametrize("n", CHAIN_SIZES)
def test_chain_all_features_vs_oracle(capi, oracle_mod, n):
    """The all-feature CHAIN kernel: every feature within the bars, the MFCC bit-exact wherever
    the spectrum is, non-finite frames as the reference."""
    x = np.concatenate([edge_frames(n), _frames(oracle_mod, n, 61, 11 + n)])
    ref = oracle_mod.extract(x)
    out = capi.Plan(buffer_size=n, scalar_f64=True, mfcc_reference=True).extract(x, FEATS)
    assert np.array_equal(out["zcr"], ref["scalars"][:, 2])
    compare(out, ref, n)
    fin = np.isfinite(ref["amp"]).all(1)
    frac, nexact = _mfcc_reference_checks(out["mfcc"][fin], out["amplitudeSpectrum"][fin], ref["mfcc"][fin], ref["amp"][fin])
    assert frac >= 0.95, frac
    print("N=%d: CHAIN all features, MFCC bit-exact on %.4f (%d frames with an exact spectrum)" % (n, frac, nexact))


@pytest.mark.parametrize("n", CHAIN_SIZES)
def test_chain_subsets_match_full_request(capi, n):
    """The subset CHAIN kernel (SUB) equals the all-feature CHAIN kernel bit for bit."""
    x = np.concatenate([edge_frames(n), np.random.default_rng(n).uniform(-1, 1, (40, n)).astype(np.float32)])
    plan = capi.Plan(buffer_size=n, scalar_f64=True, mfcc_reference=True)
    full = plan.extract(x, FEATS)
    for feats in (["mfcc"], ["mfcc", "powerSpectrum"], ["zcr", "mfcc"], ["mfcc", "spectralKurtosis", "loudness"],
                  ["rms", "spectralRolloff"]):
        out = plan.extract(x, feats)
        for k, v in out.items():
            if k not in full:
                continue
            a, b = np.asarray(v), np.asarray(full[k])
            same = (a.view(np.uint8) == b.view(np.uint8)).reshape(a.shape + (-1,)).all(-1) | (np.isnan(a) & np.isnan(b))
            assert same.all(), (feats, k, np.nonzero(~same)[0][:5])


@pytest.mark.parametrize("n", [512, 1024])
@pytest.mark.parametrize("nmel", [1, 7, 16, 17, 26, 33, 40, 64])
def test_chain_mel_band_counts(capi, oracle_mod, n, nmel):
    """1..64 bands: 1..4 chain phases, empty and one-bin segments at the low bands."""
    x = _frames(oracle_mod, n, 40, 300 + nmel)
    ref = oracle_mod.extract(x, num_mel=nmel)
    out = capi.Plan(buffer_size=n, num_mel_bands=nmel, mfcc_reference=True).extract(x, ["mfcc", "amplitudeSpectrum"])
    frac, _ = _mfcc_reference_checks(out["mfcc"], out["amplitudeSpectrum"], ref["mfcc"], ref["amp"])
    assert frac >= 0.95, (nmel, frac)


@pytest.mark.parametrize("n", CHAIN_SIZES)
def test_chain_golden(capi, n):
    """The reference's own outputs (tests/golden), 26 and 40 bands, all features requested."""
    if n == 256:
        pytest.skip("no golden fixtures at N = 256")
    g = golden_io.load(n)
    for bands, key in ((26, "mfcc"), (40, "mfcc40")):
        out = capi.Plan(buffer_size=n, num_mel_bands=bands, mfcc_reference=True).extract(g["input"], FEATS)
        frac, nexact = _mfcc_reference_checks(out["mfcc"], out["amplitudeSpectrum"], g[key], g["amp"])
        assert frac >= 0.95, (bands, frac)


def test_chain_large_batch_sample(capi, oracle_mod):
    """A 65,536-frame device batch (every workgroup's range, the batch tail), checked against
    the oracle on a spread sample of frames."""
    import torch
    n, F = 1024, 65536 + 13
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x5EED)
    plan = capi.Plan(buffer_size=n, mfcc_reference=True)
    out = plan.extract_torch(x, ["mfcc", "amplitudeSpectrum", "spectralCentroid"])
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(0, F, 517), np.arange(F - 40, F)]))
    xs = x[torch.from_numpy(idx).cuda()].cpu().numpy()
    ref = oracle_mod.extract(xs)
    frac, _ = _mfcc_reference_checks(out["mfcc"].cpu().numpy()[idx], out["amplitudeSpectrum"].cpu().numpy()[idx],
                                     ref["mfcc"], ref["amp"])
    assert frac >= 0.95, frac


@pytest.mark.parametrize("reference", [False, True])
def test_one_launch_equals_small_launches(capi, reference):
    """Frames are independent, so one launch over 40,963 frames -- waves of 3 batches each (with
    the reference order: a pair of batches whose chains run together, then a last batch finished
    alone after the loop), the last group of batches partial (its missing batches run on the
    clamped last frame and store nothing) -- equals the same frames extracted in launches of 997
    frames, every output bit for bit."""
    n, F, step = 1024, 40963, 997
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
    t = np.arange(n) / 44100.0
    for i in range(0, F, 5):
        x[i] = (rng.uniform(0.01, 0.9) * np.sin(2 * np.pi * rng.uniform(30, 18000) * t)).astype(np.float32)
    plan = capi.Plan(buffer_size=n, scalar_f64=True, mfcc_reference=reference)
    full = plan.extract(x, FEATS)
    parts = [plan.extract(x[i:i + step], FEATS) for i in range(0, F, step)]
    for k, v in full.items():
        joined = np.concatenate([p[k] for p in parts])
        assert np.array_equal(v.view(np.uint8), joined.view(np.uint8)), k


def test_chain_overflowing_band_then_next_chain(capi, oracle_mod):
    """A finite frame whose widest mel band overflows float32 (three loud tones inside band 25 of
    26 at N = 1024, bins 460 / 475 / 490, each bin's power finite): the reference's Float32Array
    sum is +inf there, so every coefficient is +-inf (the DCT column's signs), not NaN. On the packed
    tracks another band's chain follows band 25's on the same lanes; it must start from 0 (a
    select), not from inf x 0 = NaN, or the coefficients would turn NaN."""
    n = 1024
    t = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(11)
    x = []
    for a in (1.9e18, 2.0e18, 2.2e18):  # (jsfft scales by 2^-5 at N = 1024: peak |X| ~ 8 a)
        y = sum(a * np.sin(2 * np.pi * k * t / n + rng.uniform(0, 6.28)) for k in (460, 475, 490))
        x.append((y + rng.uniform(-1, 1, n)).astype(np.float32))
    x = np.stack(x)
    ref = oracle_mod.extract(x)
    assert np.isfinite(ref["amp"]).all()
    r = ref["mfcc"]
    assert np.isinf(r).all() and not np.isnan(r).any(), r[:, :4]
    out = capi.Plan(buffer_size=n, mfcc_reference=True).extract(x, ["mfcc", "amplitudeSpectrum"])
    # (these frames take the FFT's general path, whose last bits can differ from the reference's
    # on a few bins; band 25 overflows by a wide margin either way)
    g = out["mfcc"]
    assert not np.isnan(g).any(), g[:, :4]
    assert np.array_equal(g, r), (g[:, :4], r[:, :4])


@pytest.mark.parametrize("reference", [False, True])
@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_finite_amplitude_infinite_power(capi, oracle_mod, n, reference):
    """A loud tone whose amplitude bins stay finite but whose float32 power overflows (|X| above
    2^64, powerSpectrum.js a * a = +inf): the reference multiplies every bin by every band's weight
    (mfcc.js:56-61), so 0 x inf makes every band, and every coefficient, NaN. Both MFCC paths must
    send such a frame to the reference's own bin-by-bin sums, whatever the other features do."""
    t = np.arange(n, dtype=np.float64)
    x = []
    for a, k in ((1.2e20 / np.sqrt(n), n // 10), (2.0e20 / np.sqrt(n), n // 3)):  # peak |X| ~ a sqrt(n) / 4
        x.append((a * np.sin(2 * np.pi * k * t / n + 0.3) + np.random.default_rng(k).uniform(-1, 1, n)).astype(np.float32))
    x.append(np.random.default_rng(3).uniform(-1, 1, n).astype(np.float32))  # an ordinary frame beside them
    x = np.stack(x)
    ref = oracle_mod.extract(x)
    assert np.isfinite(ref["amp"][:2]).all() and (ref["amp"][:2].max(1) >= 2.0 ** 64).all()
    assert np.isnan(ref["mfcc"][:2]).all()
    plan = capi.Plan(buffer_size=n, scalar_f64=True, mfcc_reference=reference)
    out = plan.extract(x, FEATS)
    assert np.isnan(out["mfcc"][:2]).all(), out["mfcc"][:2, :4]
    assert not tolerance.check_vectors(out["mfcc"][2:], ref["mfcc"][2:])
    for feats in (["mfcc"], ["mfcc", "spectralCentroid"]):  # the light and the subset kernels
        sub = plan.extract(x, feats)
        assert np.isnan(sub["mfcc"][:2]).all(), (feats, sub["mfcc"][:2, :4])
    compare(out, ref, n)
