"""GPU parity: libmeyda_gpu.so (through the C ABI) vs the reference golden vectors
and vs the CPU oracle. Tolerances: tests/tolerance.py (RTOL = 1e-5, zcr exact)."""
import numpy as np
import pytest

import golden_io
import tolerance

pytestmark = pytest.mark.gpu

SIZES = [512, 1024, 2048]
FEATS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
         "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness",
         "perceptualSpread", "perceptualSharpness", "mfcc", "amplitudeSpectrum", "powerSpectrum"]
GOLDEN_SCALARS = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
                  "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis",
                  "loudness.total", "perceptualSpread", "perceptualSharpness"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    if capi.device_count() == 0:
        pytest.fail("no GPU visible to libmeyda_gpu.so")
    return capi


def scalars_matrix(out):
    return np.stack([out[k].astype(np.float64) for k in GOLDEN_SCALARS], 1)


def check_all(n, g, out, frames_idx=None, mfcc_key="mfcc", scal_key="scalars", amp_key="amp"):
    idx = slice(None) if frames_idx is None else frames_idx
    ref_amp = g[amp_key][idx]
    bad, exact = tolerance.check_spectra(out["amplitudeSpectrum"], ref_amp)
    assert not bad, ("amplitude spectra outside tolerance", [g["labels"][i] for i in bad])
    fails = tolerance.check_scalars(scalars_matrix(out), g[scal_key][idx], ref_amp, n)
    assert not fails, fails[:10]
    if mfcc_key:
        vb = tolerance.check_vectors(out["mfcc"], g[mfcc_key][idx])
        assert not vb, ("mfcc", vb)
    return exact


@pytest.mark.parametrize("n", SIZES)
def test_golden_all_features(capi, n):
    g = golden_io.load(n)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    out = plan.extract(g["input"], FEATS)
    exact = check_all(n, g, out)
    # loudness.specific (Float32Array(24)) and the power spectrum
    lb = tolerance.check_vectors(out["loudness.specific"], g["loudness_specific"])
    assert not lb, lb
    pb, _ = tolerance.check_spectra(out["powerSpectrum"], g["power"])
    assert not pb
    # zcr exact; the broadband (noise) frames are bit-exact in the spectrum
    assert np.array_equal(out["zcr"], g["scalars"][:, 2])
    noise = golden_io.idx(g["labels"], "noise:")
    assert np.array_equal(out["amplitudeSpectrum"][noise].view(np.uint32), g["amp"][noise].view(np.uint32))
    assert exact > 0.995, exact
    print("N=%d amplitude bit-exact fraction %.6f" % (n, exact))


@pytest.mark.parametrize("n", SIZES)
def test_float32_scalar_outputs(capi, n):
    g = golden_io.load(n)
    plan = capi.Plan(buffer_size=n)  # float32 scalar arrays (the batch default)
    out = plan.extract(g["input"], ["spectralCentroid", "rms", "zcr", "amplitudeSpectrum"])
    assert out["rms"].dtype == np.float32
    ref = g["scalars"]
    with np.errstate(invalid="ignore"):
        for j, k in [(0, "rms"), (3, "spectralCentroid")]:
            r = ref[:, j]
            fin = np.isfinite(r)
            assert np.all(np.abs(out[k][fin] - r[fin]) <= 1e-6 * np.abs(r[fin]) + 1e-30)
            assert np.array_equal(np.isnan(out[k]), np.isnan(r))
    assert np.array_equal(out["zcr"], ref[:, 2].astype(np.float32))


@pytest.mark.parametrize("n", SIZES)
def test_complex_spectrum(capi, n):
    g = golden_io.load(n)
    c = g["complex_frames"]
    plan = capi.Plan(buffer_size=n)
    out = plan.extract(g["input"][:c], ["complexSpectrum"])
    for part, key in (("complexSpectrum.real", "complex_re"), ("complexSpectrum.imag", "complex_im")):
        bad, exact = tolerance.check_spectra(out[part], g[key])
        assert not bad
        assert exact > 0.99


@pytest.mark.parametrize("n", SIZES)
def test_mfcc_40_bands(capi, n):
    g = golden_io.load(n)
    plan = capi.Plan(buffer_size=n, num_mel_bands=40)
    out = plan.extract(g["input"], ["mfcc"])
    assert not tolerance.check_vectors(out["mfcc"], g["mfcc40"])


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("bands", [26, 40])
def test_dct_on_matrix_cores(capi, n, bands):
    """The default DCT (mfcc.js:85-93) runs on v_mfma_f64_4x4x4_4b_f64; MGX_FLAG_DCT_SEQUENTIAL
    keeps the reference's sequential VALU order. The products are the same exact f32 x f32
    products; only the f64 summation order differs, so the float32 coefficients of the two
    match on (nearly) every element, and both match the golden outputs within the MFCC bar."""
    g = golden_io.load(n)
    ref = g["mfcc"] if bands == 26 else g["mfcc40"]
    out = capi.Plan(buffer_size=n, num_mel_bands=bands).extract(g["input"], ["mfcc", "rms"])
    assert not tolerance.check_vectors(out["mfcc"], ref)
    base = capi.Plan(buffer_size=n, num_mel_bands=bands, dct_sequential=True).extract(g["input"], ["mfcc"])
    assert not tolerance.check_vectors(base["mfcc"], ref)
    same = np.mean(out["mfcc"].view(np.uint32) == base["mfcc"].view(np.uint32))
    assert same > 0.98, same
    print("N=%d bands=%d: DCT on MFMA equals the sequential VALU form on %.4f of the coefficients" % (n, bands, same))


def _mfcc_reference_checks(out_mfcc, out_amp, ref_mfcc, ref_amp):
    """MGX_FLAG_MFCC_REFERENCE: mfcc.js:53-93 in the reference's own order. Wherever the
    amplitude spectrum is bit-identical to the reference's, every coefficient must be too;
    everywhere, each finite coefficient within 1e-5 relative of the reference (no norm floor)
    and the NaN / +-Inf classes equal. Returns the bit-exact fraction of coefficients."""
    g, r = out_mfcc.astype(np.float64), ref_mfcc.astype(np.float64)
    assert np.array_equal(tolerance._cls(g), tolerance._cls(r))
    fin = np.isfinite(r)
    assert np.all(np.abs(g[fin] - r[fin]) <= tolerance.RTOL * np.abs(r[fin])), \
        np.max(np.abs(g[fin] - r[fin]) / np.maximum(np.abs(r[fin]), 1e-300))
    same = (out_mfcc.view(np.uint32) == ref_mfcc.view(np.uint32)) | (np.isnan(g) & np.isnan(r))
    amp_same = np.all(out_amp.view(np.uint32) == ref_amp.view(np.uint32), 1)
    assert np.all(same[amp_same]), np.nonzero(~same[amp_same].all(1))[0]
    return float(np.mean(same)), int(amp_same.sum())


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("bands", [26, 40])
def test_mfcc_reference_order(capi, n, bands):
    g = golden_io.load(n)
    ref = g["mfcc"] if bands == 26 else g["mfcc40"]
    plan = capi.Plan(buffer_size=n, num_mel_bands=bands, mfcc_reference=True)
    out = plan.extract(g["input"], ["mfcc", "amplitudeSpectrum"])
    frac, nexact = _mfcc_reference_checks(out["mfcc"], out["amplitudeSpectrum"], ref, g["amp"])
    # (the frames whose spectrum differs in a last ulp somewhere are ~16 % of the golden set at
    # N = 2048: their coefficients may differ by an ulp; 0.97 measured there with 40 bands)
    assert frac >= 0.95, frac
    # the default plan (segmented-scan mel, hardware log, matrix-core DCT) on the same frames
    base = capi.Plan(buffer_size=n, num_mel_bands=bands).extract(g["input"], ["mfcc"])["mfcc"]
    base_frac = float(np.mean(base.view(np.uint32) == ref.view(np.uint32)))
    print("N=%d bands=%d: reference-order MFCC bit-exact on %.4f of the coefficients (%d frames with a "
          "bit-exact spectrum all exact); default plan %.4f" % (n, bands, frac, nexact, base_frac))


@pytest.mark.parametrize("n", SIZES)
def test_mfcc_reference_order_vs_oracle(capi, oracle_mod, n):
    """Ragged seeded batch (noise + tones), hamming window too: the oracle restates the
    reference bit for bit, so the same bit-identity gate applies."""
    rng = np.random.default_rng(77 + n)
    F = 203
    x = oracle_mod.synth_frames(0x6D657964, 9000, F, n).copy()
    t = np.arange(n) / 44100.0
    for i in range(0, F, 2):
        x[i] = (rng.uniform(0.01, 0.9) * np.sin(2 * np.pi * rng.uniform(30, 18000) * t)).astype(np.float32)
    for window in ("hanning", "hamming"):
        ref = oracle_mod.extract(x, window=window)
        out = capi.Plan(buffer_size=n, window=window, mfcc_reference=True).extract(x, ["mfcc", "amplitudeSpectrum"])
        frac, _ = _mfcc_reference_checks(out["mfcc"], out["amplitudeSpectrum"], ref["mfcc"], ref["amp"])
        assert frac >= 0.95, (window, frac)  # (0.973 measured at N = 2048, where more spectra differ by an ulp)


@pytest.mark.parametrize("n", SIZES)
def test_hamming_window(capi, n):
    g = golden_io.load(n)
    idx = g["hamming_frames"]
    plan = capi.Plan(buffer_size=n, window="hamming", scalar_f64=True)
    out = plan.extract(g["input"][idx], FEATS)
    bad, _ = tolerance.check_spectra(out["amplitudeSpectrum"], g["hamming_amp"])
    assert not bad
    assert not tolerance.check_scalars(scalars_matrix(out), g["hamming_scalars"], g["hamming_amp"], n)
    assert not tolerance.check_vectors(out["mfcc"], g["hamming_mfcc"])


@pytest.mark.parametrize("n", SIZES)
def test_literal_snapshot_mode(capi, n):
    g = golden_io.load(n)
    idx = g["literal_frames"]
    plan = capi.Plan(buffer_size=n, mode="literal", scalar_f64=True)
    out = plan.extract(g["input"][idx], ["amplitudeSpectrum", "loudness"])
    assert np.array_equal(out["amplitudeSpectrum"].view(np.uint32), g["literal_amp"].view(np.uint32))
    assert not tolerance.check_vectors(out["loudness.specific"], g["literal_loudness_specific"])
    # specific loudness is within ~1 float32 ulp of Math.pow (kernels.hip pow023), so the
    # total is held to 1e-6 relative (north_star bar: 1e-5)
    assert np.allclose(out["loudness.total"], g["literal_loudness_total"], rtol=1e-6)


def test_config1_reference_numbers(capi):
    # get(['rms','spectralCentroid']) on frame 0 of sound1.wav, N=512
    g = golden_io.load(512)
    i = g["labels"].index("sound1:0")
    plan = capi.Plan(buffer_size=512, scalar_f64=True)
    out = plan.extract(g["input"][i:i + 1], ["rms", "spectralCentroid"])
    assert abs(out["rms"][0] - 0.0050815644) < 1e-10
    assert abs(out["spectralCentroid"][0] - 32.0121595) < 1e-6


@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_random_batch_vs_oracle(capi, oracle_mod, n):
    """Ragged batch (not a multiple of the workgroup batch) of seeded noise + tones."""
    rng = np.random.default_rng(1234 + n)
    F = 333
    x = oracle_mod.synth_frames(0x6D657964, 1000, F, n).copy()
    t = np.arange(n) / 44100.0
    for i in range(0, F, 3):
        x[i] = (0.7 * np.sin(2 * np.pi * rng.uniform(50, 15000) * t)).astype(np.float32)
    ref = oracle_mod.extract(x)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    out = plan.extract(x, FEATS)
    bad, exact = tolerance.check_spectra(out["amplitudeSpectrum"], ref["amp"])
    assert not bad
    fails = tolerance.check_scalars(scalars_matrix(out), ref["scalars"], ref["amp"], n)
    assert not fails, fails[:10]
    assert not tolerance.check_vectors(out["mfcc"], ref["mfcc"])
    assert not tolerance.check_vectors(out["loudness.specific"], ref["loudness_specific"])


def test_device_path_full_size_properties(capi, oracle_mod):
    """BASELINE config C3/C4 size (262,144 x 1024) on device: synth -> extract; a sample
    of frames is checked against the oracle and size-independent properties hold."""
    import torch
    n, F = 1024, 262144
    frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, 0x6D657964)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    out = plan.extract_torch(frames, FEATS)
    torch.cuda.synchronize()
    pick = np.array([0, 1, 17, 4095, 65536, 131071, 200001, F - 1])
    x = oracle_mod.synth_frames(0x6D657964, 0, 1, n)
    assert np.array_equal(frames[0].cpu().numpy().view(np.uint32), x[0].view(np.uint32))
    xs = frames[torch.as_tensor(pick, device="cuda")].cpu().numpy()
    ref = oracle_mod.extract(xs)
    got = {k: v[torch.as_tensor(pick, device="cuda")].cpu().numpy() for k, v in out.items()}
    bad, exact = tolerance.check_spectra(got["amplitudeSpectrum"], ref["amp"])
    assert not bad and exact == 1.0
    assert not tolerance.check_scalars(scalars_matrix(got), ref["scalars"], ref["amp"], n)
    assert not tolerance.check_vectors(got["mfcc"], ref["mfcc"])
    # properties over the full batch
    z = out["zcr"]
    assert torch.all((z >= 0) & (z <= n - 1))
    assert torch.all(torch.isfinite(out["mfcc"]))
    rms = out["rms"]
    assert torch.allclose(rms * rms * n, out["energy"], rtol=1e-12)
    # a second launch is bitwise identical (deterministic, no atomics)
    out2 = plan.extract_torch(frames, ["amplitudeSpectrum", "mfcc", "spectralKurtosis"])
    assert torch.equal(out2["amplitudeSpectrum"], out["amplitudeSpectrum"])
    assert torch.equal(out2["mfcc"], out["mfcc"])
    assert torch.equal(out2["spectralKurtosis"], out["spectralKurtosis"])


def test_fast_precision_noise_only(capi, oracle_mod):
    """precision='fast' (fp32 butterflies): spectra within the norm-wise bar on noise."""
    n = 1024
    x = oracle_mod.synth_frames(0x6D657964, 5000, 64, n)
    ref = oracle_mod.extract(x)
    plan = capi.Plan(buffer_size=n, precision="fast", scalar_f64=True)
    out = plan.extract(x, ["amplitudeSpectrum", "spectralCentroid", "spectralSpread", "rms"])
    bad, _ = tolerance.check_spectra(out["amplitudeSpectrum"], ref["amp"])
    assert not bad
    assert np.allclose(out["spectralCentroid"], ref["scalars"][:, 3], rtol=1e-5)
    assert np.allclose(out["spectralSpread"], ref["scalars"][:, 7], rtol=1e-5)


def test_errors_and_empty(capi):
    import ctypes
    plan = capi.Plan(buffer_size=512)
    o = capi.Outputs()
    assert capi.lib().mgx_extract_host(plan._h, None, 0, ctypes.byref(o)) == 0
    o.complex_real = 1234
    x = np.zeros((1, 512), np.float32)
    assert capi.lib().mgx_extract_host(plan._h, x.ctypes.data, 1, ctypes.byref(o)) == -1
    with pytest.raises(capi.MgxError):
        capi.Plan(buffer_size=128)  # below the GPU path's range: MGX_E_UNSUPPORTED


@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_small_host_batches_equal_staged_path(capi, n):
    """Host batches of up to 512 frames (the real-time get()/process() path) run one launch over
    plan-owned pinned host memory that the kernel reads and writes over PCIe (plan.cpp
    extract_host_small); larger ones stage through device memory. Both must give the device
    path's outputs bit for bit: 1 frame, a streaming batch, the threshold and one past it, with
    every output (the complex spectrum too) and with a two-feature request."""
    import os

    import torch
    rng = np.random.default_rng(n)
    os.environ["MGX_SMALL_BATCH_FRAMES"] = "0"
    try:
        staged = capi.Plan(buffer_size=n, scalar_f64=True)
    finally:
        del os.environ["MGX_SMALL_BATCH_FRAMES"]
    small = capi.Plan(buffer_size=n, scalar_f64=True)
    every = capi.ALL_FEATURES + ["amplitudeSpectrum", "powerSpectrum", "complexSpectrum"]
    for F, feats in ((1, ["rms", "spectralCentroid"]), (1, every), (64, every), (512, every), (513, every)):
        x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
        x[0, :7] = [np.nan, np.inf, -0.0, 1e-40, 3e38, -3e38, 0.0] if F > 1 else x[0, :7]
        a, b = small.extract(x, feats), staged.extract(x, feats)
        d = small.extract_torch(torch.from_numpy(x).cuda(), feats)
        torch.cuda.synchronize()
        for k in a:
            assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), (F, k)
            assert np.array_equal(a[k].view(np.uint8), d[k].cpu().numpy().view(np.uint8)), (F, k)
        # the pinned buffers are reused: a second call with other frames must not see the first's
        y = rng.uniform(-1, 1, (F, n)).astype(np.float32)
        a2, b2 = small.extract(y, feats), staged.extract(y, feats)
        for k in a2:
            assert np.array_equal(a2[k].view(np.uint8), b2[k].view(np.uint8)), (F, k, "second call")


@pytest.mark.parametrize("n", [256, 512, 1024])
def test_one_frame_calls_with_the_frame_in_the_kernel_arguments(capi, n):
    """A one-frame host call at N <= 1024 passes its frame inside the kernel arguments (KernelArgsInline;
    kernels.hip extract_kernel<..., INL>): each kernel kind that takes it -- every feature, a subset (SUB),
    a light subset (LIGHT: mfcc or a spectrum alone), every spectral feature without the time-domain ones
    (NOTIME) -- must give the device path's bits, for ordinary and for non-finite frames, call after call."""
    import torch
    rng = np.random.default_rng(n + 3)
    p = capi.Plan(buffer_size=n, scalar_f64=True)
    spectral = [f for f in capi.ALL_FEATURES if f not in ("rms", "energy", "zcr")]
    kinds = [capi.ALL_FEATURES, ["rms", "spectralCentroid"], ["zcr", "spectralRolloff", "loudness"], ["mfcc"],
             ["amplitudeSpectrum"], spectral]
    for i in range(12):
        x = rng.uniform(-1, 1, (1, n)).astype(np.float32)
        if i % 4 == 3:
            x[0, 5] = np.inf if i % 8 == 3 else np.nan
        feats = kinds[i % len(kinds)]
        a = p.extract(x, feats)
        d = p.extract_torch(torch.from_numpy(x).cuda(), feats)
        torch.cuda.synchronize()
        for k in a:
            assert np.array_equal(a[k].view(np.uint8), d[k].cpu().numpy().view(np.uint8)), (i, feats, k)
    p.close()


def test_one_frame_call_whose_outputs_equal_the_wait_preset(capi):
    """A one-frame host call without spectra waits on its output words, each preset to all ones (plan.cpp
    extract_host_small). A frame of all-ones NaN samples can produce outputs with exactly that bit pattern
    (the NaN payload propagates): the call must still end, through its spin limit and the stream, with the
    device path's bits -- with float32 and float64 scalars."""
    import torch
    for f64 in (False, True):
        p = capi.Plan(buffer_size=512, scalar_f64=f64)
        x = np.full((1, 512), 0xFFFFFFFF, np.uint32).view(np.float32)
        for feats in (["rms", "energy", "spectralCentroid"], capi.ALL_FEATURES):
            a = p.extract(x, feats)
            d = p.extract_torch(torch.from_numpy(x.copy()).cuda(), feats)
            torch.cuda.synchronize()
            for k in a:
                assert np.array_equal(a[k].view(np.uint8), d[k].cpu().numpy().view(np.uint8)), (f64, k)
        p.close()


def test_small_and_staged_calls_alternate_on_one_plan(capi):
    """One plan serving small host batches (its own compute stream, created by the small path) and
    staged ones (which create the copy stream beside it) in turn, then destroyed: the staged path must
    reuse the small path's stream rather than replace it (a replaced stream was never synchronised or
    destroyed), and every call gives the same bits as a fresh plan's."""
    n = 1024
    rng = np.random.default_rng(7)
    feats = capi.ALL_FEATURES
    ref = capi.Plan(buffer_size=n, scalar_f64=True)
    p = capi.Plan(buffer_size=n, scalar_f64=True)
    for F in (1, 600, 3, 2000, 64, 513, 1):
        x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
        a, b = p.extract(x, feats), ref.extract(x, feats)
        for k in a:
            assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), (F, k)
    p.close()
    ref.close()


def test_destroy_right_after_default_stream_launch(capi):
    """mgx_plan_destroy waits for every launch that used the plan (include/meyda_gpu.h), also a large
    batch launched on the default (NULL) stream before the plan had a stream of its own: its scratch
    completion event is recorded, and destroy waits on it before freeing the tables."""
    import torch
    n = 1024
    x = torch.empty(262144, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0xD35)
    torch.cuda.synchronize()
    outs = []
    for _ in range(3):
        p = capi.Plan(buffer_size=n)
        with torch.cuda.stream(torch.cuda.default_stream()):
            outs.append(p.extract_torch(x, capi.ALL_FEATURES))
        p.close()  # right away: the launch is still running
    torch.cuda.synchronize()
    for o in outs[1:]:
        for k in o:
            assert torch.equal(o[k], outs[0][k]), k
    assert torch.isfinite(outs[0]["spectralCentroid"]).all()


C3_SET = ["spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff", "spectralSpread",
          "spectralSkewness", "spectralKurtosis", "loudness", "perceptualSpread", "perceptualSharpness"]


@pytest.mark.parametrize("n", [256, 512, 1024, 2048])
def test_scalar_windows_equal_per_batch_form(capi, n):
    """A launch whose waves get 8 or more batches each computes the scalar features once per
    window of 16 batches, one lane per frame (kernels.hip scalar_pass); a smaller launch computes
    them per batch, one lane per (feature, frame). The same frames through both must give the same
    bits: a ragged 262,157-frame launch (partial batch, partial last windows) against chunks of
    16,384 frames, every feature, C3's subset, time features beside a spectrum-only request (the light
    kernels, whose records hold only those), float32 and float64 scalars, the reference-order MFCC,
    and non-finite, silent and loud frames among them (a NaN output may differ in its sign bit:
    the formulas are the same, the instructions that propagate the NaN are not)."""
    import torch
    F, chunk = 262144 + 13, 16384
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x5CA1AB1E)
    x[5, 3] = float("nan")
    x[70000, :] = 0.0
    x[140001, 9] = float("inf")
    x[200003, :] *= 1e19
    x[F - 1, 0] = float("-inf")
    for kw, feats in (({"scalar_f64": True}, capi.ALL_FEATURES), ({}, capi.ALL_FEATURES), ({}, C3_SET),
                      ({"scalar_f64": True, "mfcc_reference": True}, capi.ALL_FEATURES),
                      ({}, ["mfcc", "rms", "zcr"]), ({"scalar_f64": True}, ["amplitudeSpectrum", "energy"])):
        plan = capi.Plan(buffer_size=n, **kw)
        whole = plan.extract_torch(x, feats)
        parts = [plan.extract_torch(x[i:i + chunk].contiguous(), feats) for i in range(0, F, chunk)]
        torch.cuda.synchronize()
        for k, v in whole.items():
            w = torch.cat([p[k] for p in parts])
            # bit for bit, except that a NaN may differ in sign (the reference's NaN has none)
            nan = torch.isnan(v)
            assert torch.equal(nan, torch.isnan(w)), (n, kw, k)
            assert torch.equal(v[~nan].view(torch.uint8), w[~nan].view(torch.uint8)), (n, kw, k)
        plan.close()
