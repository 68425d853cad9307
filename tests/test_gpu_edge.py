"""GPU parity beyond the golden fixtures: non-finite and extreme inputs, other sample
rates, window and mel-band counts, N = 256, and a seeded randomized sweep of plan
configurations — every case against the CPU oracle (tests/tolerance.py bars; NaN/Inf
classes must match exactly)."""
import numpy as np
import pytest

import tolerance

pytestmark = pytest.mark.gpu

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


def compare(out, ref, n, sr=44100.0, spectra_exact_min=None):
    got_s = np.stack([out[k].astype(np.float64) for k in SCALARS], 1)
    fails = tolerance.check_scalars(got_s, ref["scalars"], ref["amp"], n, sr=sr)
    assert not fails, fails[:10]
    a, r = out["amplitudeSpectrum"].astype(np.float64), ref["amp"].astype(np.float64)
    # Frames where an infinity enters the FFT (an Inf sample, or overflow inside a stage):
    # the reference's full complex FFT forms 0 * Inf in its j = 0 twiddle product, which
    # turns the imaginary companion of the real DC / X[N/4] values into NaN; the
    # half-spectrum network never forms that product, so those two bins can be +-Inf where
    # the reference has NaN. Every other bin, and every feature (checked
    # above), matches in class.
    nonfin = ~np.isfinite(r).all(1)
    ex = np.zeros(a.shape, bool)
    ex[:, 0] = nonfin
    ex[:, a.shape[1] // 2] = nonfin
    assert np.array_equal(np.isnan(a) & ~ex, np.isnan(r) & ~ex)
    assert np.array_equal(np.isinf(a) & ~ex, np.isinf(r) & ~ex)
    assert np.all(~np.isfinite(a[ex]) | ~np.isfinite(r[ex]) | (a[ex] == r[ex]))
    fin = np.isfinite(r).all(1)
    bad, exact = tolerance.check_spectra(out["amplitudeSpectrum"][fin], ref["amp"][fin])
    assert not bad, bad
    if spectra_exact_min is not None:
        assert exact >= spectra_exact_min, exact
    # mfcc and specific loudness: exact policy on finite frames; on non-finite frames every
    # value the reference leaves finite must match (bands away from bins 0 and N/4), and
    # every NaN of the reference must be non-finite here.
    for key, rkey in (("mfcc", "mfcc"), ("loudness.specific", "loudness_specific")):
        g, rr = out[key], ref[rkey]
        assert not tolerance.check_vectors(g[~nonfin], rr[~nonfin]), key
        if nonfin.any():
            gn, rn = g[nonfin].astype(np.float64), rr[nonfin].astype(np.float64)
            fin = np.isfinite(rn)
            assert np.all(np.isfinite(gn[fin])), key
            with np.errstate(invalid="ignore"):
                assert np.all(np.abs(gn[fin] - rn[fin]) <= 1e-5 * np.abs(rn[fin]) + 1e-30), key
            assert np.all(~np.isfinite(gn[~fin])), key


def edge_frames(n):
    rng = np.random.default_rng(5)
    fr = []
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y = x.copy(); y[n // 3] = np.nan; fr.append(y)                    # one NaN sample
    y = x.copy(); y[7] = np.inf; fr.append(y)                         # one +Inf sample
    y = x.copy(); y[n - 1] = -np.inf; fr.append(y)                    # -Inf at the end
    fr.append(np.full(n, np.nan, np.float32))                         # all NaN
    fr.append(np.full(n, 3.0e38, np.float32))                         # energy overflows
    fr.append((x * 1e-39).astype(np.float32))                         # denormal samples
    fr.append(np.where(np.arange(n) % 2 == 0, 1.0, -1.0).astype(np.float32))  # Nyquist
    y = np.zeros(n, np.float32); y[0] = -0.0; y[1] = 0.0; fr.append(y)          # signed zeros
    fr.append(np.full(n, 1e-45, np.float32))                          # smallest denormal, DC
    y = x.copy(); y[: n // 2] = 0; fr.append(y)                       # half silence
    # tiny spectra on both sides of the amplitude fast path's range (|X| ~ 2^-40), down to
    # power spectra at the bottom of the normal float32 range; at 1e-24 the powers are 0.
    # (Between those, denormal powers leave the reference's own mel sums a few significant
    # bits: no parity target.)
    for scale in (1e-9, 1e-13, 1e-16, 1e-24):
        fr.append((x * np.float32(scale)).astype(np.float32))
    return np.stack(fr)


@pytest.mark.parametrize("n", [256, 512, 1024, 2048])
def test_nonfinite_and_extreme_frames(capi, oracle_mod, n):
    x = edge_frames(n)
    ref = oracle_mod.extract(x)
    out = capi.Plan(buffer_size=n, scalar_f64=True).extract(x, FEATS)
    assert np.array_equal(out["zcr"], ref["scalars"][:, 2])
    compare(out, ref, n)


@pytest.mark.parametrize("n", [256, 512, 1024, 2048])
def test_subsets_match_full_request_on_edge_frames(capi, n):
    """A feature subset runs the SUB kernel, which skips what the request does not read (zcr
    ballots, the energy sum, moments, the prefix row and, without both, the amplitude total:
    the non-finite test then comes from the amplitudes' bits). Its outputs must equal the
    all-feature kernel's bit for bit, on the NaN / Inf / overflow / denormal frames too."""
    x = np.concatenate([edge_frames(n), np.random.default_rng(n).uniform(-1, 1, (40, n)).astype(np.float32)])
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    full = plan.extract(x, FEATS)
    for feats in (["mfcc"], ["amplitudeSpectrum", "spectralCentroid"], ["mfcc", "powerSpectrum"],
                  ["spectralKurtosis", "loudness"], ["zcr", "mfcc"], ["rms", "spectralRolloff"]):
        out = plan.extract(x, feats)
        for k, v in out.items():
            if k not in full:
                continue
            a, b = np.asarray(v), np.asarray(full[k])
            same = (a.view(np.uint8) == b.view(np.uint8)).reshape(a.shape + (-1,)).all(-1) | (np.isnan(a) & np.isnan(b))
            assert same.all(), (feats, k, np.nonzero(~same)[0][:5])


@pytest.mark.parametrize("sr", [8000.0, 22050.0, 48000.0, 96000.0])
def test_sample_rates(capi, oracle_mod, sr):
    n = 1024
    x = oracle_mod.synth_frames(0x6D657964, 77, 48, n)
    t = np.arange(n) / sr
    x[::4] = (0.5 * np.sin(2 * np.pi * 1000.0 * t)).astype(np.float32)
    ref = oracle_mod.extract(x, sample_rate=sr)
    out = capi.Plan(buffer_size=n, sample_rate=sr, scalar_f64=True).extract(x, FEATS)
    compare(out, ref, n, sr=sr)


@pytest.mark.parametrize("nmel", [1, 7, 16, 17, 26, 33, 40, 64])
def test_mel_band_counts(capi, oracle_mod, nmel):
    n = 1024
    x = oracle_mod.synth_frames(0x6D657964, 300, 40, n)
    ref = oracle_mod.extract(x, num_mel=nmel)
    out = capi.Plan(buffer_size=n, num_mel_bands=nmel, scalar_f64=True).extract(x, ["mfcc", "amplitudeSpectrum"])
    assert not tolerance.check_vectors(out["mfcc"], ref["mfcc"]), nmel


@pytest.mark.parametrize("flags", [{}, {"dct_sequential": True}, {"mfcc_reference": True}])
def test_largest_lds_image(capi, oracle_mod, flags):
    """64 mel bands x 32 coefficients at N = 1024: the plan's LDS image (bark limits, twiddles, DCT table;
    kernels.hip lds_image_kernel) is larger than the prologue's first pass of 16-byte loads, so its tail
    (the DCT rows past 16 KB) takes the second loop. Every output but the MFCC equals the 13-coefficient
    plan's bit for bit (the twiddles came through), and each of the first 13 coefficients is that plan's
    DCT sum over 32 instead of 13 (mfcc.js:91; the reference fixes numCoeffs = 13, the engine allows 1..32)."""
    n = 1024
    x = oracle_mod.synth_frames(0x6D657964, 301, 40, n)
    a = capi.Plan(buffer_size=n, num_mel_bands=64, num_mfcc_coeffs=32, scalar_f64=True, **flags).extract(x, FEATS)
    b = capi.Plan(buffer_size=n, num_mel_bands=64, scalar_f64=True, **flags).extract(x, FEATS)
    for k in b:
        if k != "mfcc":
            assert np.array_equal(a[k], b[k], equal_nan=True), k
    v32 = a["mfcc"].reshape(len(x), 32)[:, :13].astype(np.float64) * 32
    v13 = b["mfcc"].reshape(len(x), 13).astype(np.float64) * 13
    scale = np.abs(v13).max(axis=1, keepdims=True)
    assert (np.abs(v32 - v13) <= 1e-6 * scale).all()


def test_n256_batch(capi, oracle_mod):
    n = 256
    x = oracle_mod.synth_frames(0x6D657964, 9, 200, n)
    ref = oracle_mod.extract(x)
    out = capi.Plan(buffer_size=n, scalar_f64=True).extract(x, FEATS)
    compare(out, ref, n, spectra_exact_min=0.999)


def test_randomized_plans(capi, oracle_mod):
    """A seeded sweep over (N, window, sample rate, mel bands, signal type, batch size)."""
    rng = np.random.default_rng(20261015)
    for case in range(24):
        n = int(rng.choice([256, 512, 1024, 2048]))
        window = str(rng.choice(["hanning", "hamming"]))
        sr = float(rng.choice([16000.0, 44100.0, 48000.0]))
        nmel = int(rng.integers(1, 65))
        F = int(rng.integers(1, 70))
        kind = case % 4
        t = np.arange(n) / sr
        if kind == 0:
            x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
        elif kind == 1:
            f = rng.uniform(20, sr / 2, (F, 1))
            x = (rng.uniform(0.01, 1, (F, 1)) * np.sin(2 * np.pi * f * t)).astype(np.float32)
        elif kind == 2:
            x = (rng.standard_normal((F, n)) * 10.0 ** rng.uniform(-8, 3, (F, 1))).astype(np.float32)
        else:
            x = np.round(rng.uniform(-1, 1, (F, n)) * 32768) / 32768  # int16-like PCM
            x = x.astype(np.float32)
        ref = oracle_mod.extract(x, sample_rate=sr, window=window, num_mel=nmel)
        out = capi.Plan(buffer_size=n, sample_rate=sr, window=window, num_mel_bands=nmel,
                        scalar_f64=True).extract(x, FEATS)
        try:
            compare(out, ref, n, sr=sr)
        except AssertionError as e:
            raise AssertionError("case %d: n=%d window=%s sr=%g nmel=%d F=%d kind=%d: %s"
                                 % (case, n, window, sr, nmel, F, kind, e))


SUBSETS = {
    "time_only": ["rms", "energy", "zcr"],
    "spectral": ["spectralCentroid", "spectralFlatness", "spectralKurtosis", "spectralRolloff"],
    "loudness": ["loudness", "perceptualSharpness"],
    "mfcc_only": ["mfcc"],
    "amp_centroid": ["amplitudeSpectrum", "spectralCentroid"],
    # the subset kernel's two flags one at a time (kernels.hip SUB: need_prefix, need_mom)
    "rolloff_only": ["spectralRolloff"],
    "flatness_slope_mfcc": ["spectralFlatness", "spectralSlope", "mfcc"],
}
SCALAR_INDEX = {k: i for i, k in enumerate(SCALARS)}


@pytest.mark.parametrize("n", [256, 512, 1024, 2048])
def test_feature_subsets_across_batches(capi, oracle_mod, n):
    """Each feature subset (the kernel skips the spectrum, the mel records or phase-2 parts
    per request) over a batch spanning several frame batches per wave, so every frame is
    fed by the next-frame load of the previous one (kernels.hip Geo::PF), mixing tame frames
    with huge finite ones (|x| ~ 1e30: the two-form block-start butterflies) and silence
    (the f64 amplitude path)."""
    rng = np.random.default_rng(n)
    # >= 2 groups of 16 frames per workgroup at every N (at most 6 x 256 workgroups), so
    # waves run several batches and cross batch boundaries with the next-frame load
    F = 1536 * 16 * 2 + 5
    x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
    x[5::7] *= np.float32(1e30)
    x[3::11] = 0.0
    ref = oracle_mod.extract(x)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    for name, feats in SUBSETS.items():
        out = plan.extract(x, feats)
        for k in feats:
            if k == "amplitudeSpectrum":
                bad, _ = tolerance.check_spectra(out[k], ref["amp"])
                assert not bad, (name, k, bad[:5])
            elif k == "mfcc":
                assert not tolerance.check_vectors(out[k], ref["mfcc"]), (name, k)
            elif k == "loudness":
                assert not tolerance.check_vectors(out["loudness.specific"], ref["loudness_specific"]), name
                i = SCALAR_INDEX["loudness.total"]
                got = np.asarray(out["loudness.total"], np.float64)[:, None]
                assert not tolerance.check_scalars(got, ref["scalars"][:, i:i + 1], ref["amp"], n,
                                                   names=["loudnessTotal"]), name
            else:
                i = SCALAR_INDEX[k]
                got = np.asarray(out[k], np.float64)[:, None]
                fails = tolerance.check_scalars(got, ref["scalars"][:, i:i + 1], ref["amp"], n,
                                                names=[tolerance.SCALAR_NAMES[i]])
                assert not fails, (name, k, fails[:5])
