"""Parity tolerance policy, shared by the oracle and GPU tests.

* zcr: exact.
* spectra: per frame ||d||_inf <= RTOL * ||ref||_inf (and the bit-exact fraction is reported).
* scalars: |d| <= RTOL*|ref| + atol, atol = RTOL x the largest term of the formula for the
  features whose formula cancels (spectralSlope, spectralSkewness, spectralKurtosis).
* NaN / +-Inf: the class must match.
* spectralRolloff: exact, except a near-tie (|prefix - 0.99 total| < 1e-12 total) may move one bin.
* vectors (mfcc, loudness.specific): per element RTOL relative, with a floor of RTOL*||ref||_inf.
"""
import numpy as np

RTOL = 1e-5  # BASELINE.json north_star: "within 1e-5 relative float tolerance (zcr bit-exact)"

SCALAR_NAMES = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness",
                "spectralSlope", "spectralRolloff", "spectralSpread", "spectralSkewness",
                "spectralKurtosis", "loudnessTotal", "perceptualSpread", "perceptualSharpness"]


def _cls(v):
    return np.where(np.isnan(v), 0, np.where(np.isposinf(v), 1, np.where(np.isneginf(v), 2, 3)))


def term_scale(amp, n, sr):
    """Per-frame magnitude of the largest term in the cancelling formulas (reference amp)."""
    a = amp.astype(np.float64)
    L = n // 2
    k = np.arange(L, dtype=np.float64)
    den0 = a.sum(1)
    with np.errstate(all="ignore"):
        mus = [(a * k ** p).sum(1) / den0 for p in (1, 2, 3, 4)]
        m1, m2, m3, m4 = mus
        var = m2 - m1 * m1
        f = k * sr / n
        sf, sff, sfa = f.sum(), (f * f).sum(), (a * f).sum(1)
        slope = np.maximum(np.abs(L * sfa), np.abs(sf * den0)) / np.abs(den0 * (sff - sf * sf))
        skew = np.maximum.reduce([np.abs(2 * m1 ** 3), np.abs(3 * m1 * m2), np.abs(m3)]) / np.abs(var) ** 1.5
        kurt = np.maximum.reduce([np.abs(3 * m1 ** 4), np.abs(6 * m1 * m2), np.abs(4 * m1 * m3),
                                  np.abs(m4)]) / var ** 2
    return {"spectralSlope": slope, "spectralSkewness": skew, "spectralKurtosis": kurt}


def rolloff_near_tie(amp, sr):
    a = amp.astype(np.float64)
    total = a.sum(1)
    pref = np.concatenate([np.zeros((a.shape[0], 1)), np.cumsum(a, 1)], 1)
    thr = 0.99 * total
    return (np.abs(pref - thr[:, None]) <= 1e-12 * np.abs(total)[:, None] + 1e-300).any(1)


def check_scalars(got, ref, ref_amp, n, sr=44100.0, names=SCALAR_NAMES, rtol=RTOL):
    """Return a list of (frame, name, got, ref) failures."""
    fails = []
    ts = term_scale(ref_amp, n, sr)
    tie = rolloff_near_tie(ref_amp, sr)
    nyq = sr / (2.0 * (n // 2 - 1))
    for j, name in enumerate(names):
        g, r = got[:, j].astype(np.float64), ref[:, j].astype(np.float64)
        bad = _cls(g) != _cls(r)
        fin = np.isfinite(r) & np.isfinite(g)
        if name == "zcr":
            bad |= fin & (g != r)
        elif name == "spectralRolloff":
            d = np.abs(g - r)
            bad |= fin & (d > 0) & ~(tie & (d <= nyq * 1.0000001))
        else:
            atol = ts.get(name, np.zeros_like(r)) * rtol
            atol = np.where(np.isfinite(atol), atol, 0)
            with np.errstate(invalid="ignore"):
                bad |= fin & (np.abs(g - r) > rtol * np.abs(r) + atol)
        for f in np.nonzero(bad)[0]:
            fails.append((int(f), name, float(g[f]), float(r[f])))
    return fails


def check_vectors(got, ref, rtol=RTOL):
    """Per element rtol with a norm-wise floor; NaN classes must match. Returns bad frames."""
    g, r = got.astype(np.float64), ref.astype(np.float64)
    bad = (_cls(g) != _cls(r)).any(1)
    fin = np.isfinite(r) & np.isfinite(g)
    with np.errstate(invalid="ignore"):
        norm = np.max(np.where(np.isfinite(r), np.abs(r), 0), 1, keepdims=True)
        tol = np.maximum(rtol * np.abs(r), rtol * norm)
        bad |= (fin & (np.abs(g - r) > tol)).any(1)
    return np.nonzero(bad)[0].tolist()


def check_spectra(got, ref, rtol=RTOL):
    """Norm-wise per frame. Returns (bad_frames, bit_exact_fraction)."""
    g, r = got.astype(np.float64), ref.astype(np.float64)
    with np.errstate(invalid="ignore"):
        norm = np.max(np.abs(r), 1)
        err = np.max(np.abs(g - r), 1)
    bad = np.nonzero(~(err <= rtol * norm + 0.0) & ~((norm == 0) & (err == 0)))[0].tolist()
    exact = float(np.mean(got.view(np.uint32) == ref.view(np.uint32)))
    return bad, exact
