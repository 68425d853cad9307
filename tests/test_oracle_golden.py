"""Pin the CPU oracle (oracle/meyda_oracle.c) to the reference's own outputs.

The golden vectors were produced by running the reference modules under node
(tools/gen_golden.js). Spectra, loudness.specific and mfcc are compared bit for
bit; scalars to 1e-12 relative (glibc vs fdlibm transcendentals); host tables
bit for bit.
"""
import numpy as np
import pytest

import golden_io
import tolerance

SIZES = [512, 1024, 2048]


@pytest.fixture(scope="module", params=SIZES)
def case(request, oracle_mod):
    n = request.param
    g = golden_io.load(n)
    o = oracle_mod.extract(g["input"], want_complex=True)
    return n, g, o


@pytest.mark.parametrize("n", SIZES)
def test_tables_bit_exact(n, oracle_mod):
    g = golden_io.load(n)
    t = oracle_mod.tables(n)
    for k in ("hann", "hamming", "bark", "bblimits", "mel_bins", "mel_values", "mel_freq", "dct",
              "twiddle_seeds"):
        assert np.array_equal(t[k].view(np.uint8), g[k].view(np.uint8)), k
    t40 = oracle_mod.tables(n, num_mel=40)
    assert np.array_equal(t40["mel_bins"], g["mel40_bins"])
    assert np.array_equal(t40["dct"].view(np.uint32), g["dct40"].view(np.uint32))


def test_amplitude_bit_exact(case):
    n, g, o = case
    assert np.array_equal(o["amp"].view(np.uint32), g["amp"].view(np.uint32))


def test_complex_spectrum_bit_exact(case):
    n, g, o = case
    c = g["complex_frames"]
    assert np.array_equal(o["complex_re"][:c].view(np.uint32), g["complex_re"].view(np.uint32))
    assert np.array_equal(o["complex_im"][:c].view(np.uint32), g["complex_im"].view(np.uint32))


def test_scalars(case):
    n, g, o = case
    got, ref = o["scalars"], g["scalars"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = np.isfinite(ref)
    assert np.array_equal(got[~fin], ref[~fin], equal_nan=True)
    rel = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    assert rel.max() <= 1e-12
    assert not tolerance.check_scalars(got, ref, g["amp"], n)


def test_vectors_bit_exact(case):
    n, g, o = case
    assert np.array_equal(o["loudness_specific"].view(np.uint32), g["loudness_specific"].view(np.uint32))
    assert np.array_equal(o["mfcc"].view(np.uint32), g["mfcc"].view(np.uint32))


@pytest.mark.parametrize("n", SIZES)
def test_mfcc40_bit_exact(n, oracle_mod):
    g = golden_io.load(n)
    o = oracle_mod.extract(g["input"], num_mel=40)
    assert np.array_equal(o["mfcc"].view(np.uint32), g["mfcc40"].view(np.uint32))


@pytest.mark.parametrize("n", SIZES)
def test_hamming_window(n, oracle_mod):
    g = golden_io.load(n)
    x = g["input"][g["hamming_frames"]]
    o = oracle_mod.extract(x, window="hamming")
    assert np.array_equal(o["amp"].view(np.uint32), g["hamming_amp"].view(np.uint32))
    assert np.array_equal(o["mfcc"].view(np.uint32), g["hamming_mfcc"].view(np.uint32))
    assert not tolerance.check_scalars(o["scalars"], g["hamming_scalars"], g["hamming_amp"], n)


@pytest.mark.parametrize("n", SIZES)
def test_literal_snapshot_mode(n, oracle_mod):
    g = golden_io.load(n)
    x = g["input"][g["literal_frames"]]
    o = oracle_mod.extract(x, literal=True)
    assert np.array_equal(o["amp"].view(np.uint32), g["literal_amp"].view(np.uint32))
    assert np.array_equal(o["loudness_specific"].view(np.uint32),
                          g["literal_loudness_specific"].view(np.uint32))
    assert np.array_equal(o["scalars"][:, 10], g["literal_loudness_total"])


def test_config1_reference_numbers(oracle_mod):
    # frame 0 of sound1.wav at N=512 -> rms 0.0050815644, centroid 32.0121595
    g = golden_io.load(512)
    i = g["labels"].index("sound1:0")
    o = oracle_mod.extract(g["input"][i:i + 1])
    assert abs(o["scalars"][0, 0] - 0.0050815644) < 1e-10
    assert abs(o["scalars"][0, 3] - 32.0121595) < 1e-6


def test_synth_matches_golden_noise(oracle_mod):
    for n in SIZES:
        g = golden_io.load(n)
        noise = golden_io.idx(g["labels"], "noise:")
        x = oracle_mod.synth_frames(0x6D657964, 0, len(noise), n)
        assert np.array_equal(x.view(np.uint32), g["input"][noise].view(np.uint32))


def test_edge_semantics(oracle_mod):
    g = golden_io.load(512)
    lab = g["labels"]
    s = g["scalars"]
    z = lab.index("edge:zeros")
    # all-zero frame: NaN moments, +Inf sharpness, rolloff = L*sr/(2(L-1))
    assert np.isnan(s[z, 3]) and np.isinf(s[z, 12])
    assert s[z, 6] == 256 * 44100 / (2 * 255)
    sz = lab.index("edge:signedZeros")
    x = g["input"][sz]
    assert np.signbit(x[0]) and x[0] == 0
    o = oracle_mod.extract(g["input"][sz:sz + 1])
    assert o["scalars"][0, 2] == s[sz, 2]
