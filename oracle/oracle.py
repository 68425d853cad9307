"""ctypes front-end to the CPU oracle (liboracle.so built from meyda_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the meyda_amd product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
NUM_SCALARS = 13
NUM_BARK = 24
NUM_COEFFS = 13
SCALAR_NAMES = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness",
                "spectralSlope", "spectralRolloff", "spectralSpread", "spectralSkewness",
                "spectralKurtosis", "loudnessTotal", "perceptualSpread", "perceptualSharpness"]

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.oracle_extract.argtypes = [fp, ctypes.c_long, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, fp, fp, fp, dp, fp, fp]
        L.oracle_extract.restype = ctypes.c_int
        L.oracle_features_from_amp.argtypes = [fp, fp, ctypes.c_long, ctypes.c_int, ctypes.c_double,
                                               ctypes.c_int, dp, fp, fp]
        L.oracle_features_from_amp.restype = ctypes.c_int
        L.oracle_hanning.argtypes = [ctypes.c_int, fp]
        L.oracle_hamming.argtypes = [ctypes.c_int, fp]
        L.oracle_bark_scale.argtypes = [ctypes.c_int, ctypes.c_double, fp]
        L.oracle_bark_band_limits.argtypes = [fp, ctypes.c_int, ctypes.c_int, ip]
        L.oracle_mel_bins.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ip, fp, fp]
        L.oracle_dct.argtypes = [ctypes.c_int, fp]
        L.oracle_twiddle_seeds.argtypes = [ctypes.c_int, dp]
        L.oracle_jsfft.argtypes = [fp, fp, ctypes.c_int]
        L.oracle_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_long, fp]
        L.oracle_is_power_of_two.argtypes = [ctypes.c_double]
        L.oracle_is_power_of_two.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, ct=ctypes.c_float):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ct))


def extract(frames, sample_rate=44100.0, window="hanning", num_mel=26, literal=False,
            want_complex=False):
    """Run the oracle over frames (F x N float32). Returns a dict of numpy arrays."""
    frames = np.ascontiguousarray(frames, dtype=np.float32)
    F, N = frames.shape
    out = {
        "amp": np.empty((F, N // 2), np.float32),
        "scalars": np.empty((F, NUM_SCALARS), np.float64),
        "loudness_specific": np.empty((F, NUM_BARK), np.float32),
        "mfcc": np.empty((F, NUM_COEFFS), np.float32),
    }
    cre = cim = None
    if want_complex:
        cre = out["complex_re"] = np.empty((F, N), np.float32)
        cim = out["complex_im"] = np.empty((F, N), np.float32)
    rc = lib().oracle_extract(_p(frames), F, N, sample_rate, 1 if window == "hamming" else 0,
                              num_mel, 1 if literal else 0, _p(out["amp"]), _p(cre), _p(cim),
                              _p(out["scalars"], ctypes.c_double), _p(out["loudness_specific"]),
                              _p(out["mfcc"]))
    if rc != 0:
        raise ValueError("oracle_extract rejected the arguments (N=%d)" % N)
    return out


def features_from_amp(frames, amp, sample_rate=44100.0, num_mel=26):
    """Reference features of a given amplitude spectrum (rms/energy/zcr from frames)."""
    frames = np.ascontiguousarray(frames, dtype=np.float32)
    amp = np.ascontiguousarray(amp, dtype=np.float32)
    F, N = frames.shape
    out = {
        "scalars": np.empty((F, NUM_SCALARS), np.float64),
        "loudness_specific": np.empty((F, NUM_BARK), np.float32),
        "mfcc": np.empty((F, NUM_COEFFS), np.float32),
    }
    rc = lib().oracle_features_from_amp(_p(frames), _p(amp), F, N, sample_rate, num_mel,
                                        _p(out["scalars"], ctypes.c_double),
                                        _p(out["loudness_specific"]), _p(out["mfcc"]))
    if rc != 0:
        raise ValueError("oracle_features_from_amp rejected the arguments")
    return out


def synth(seed, first_index, count):
    out = np.empty(count, np.float32)
    lib().oracle_synth(seed, first_index, count, _p(out))
    return out


def synth_frames(seed, first_frame, nframes, n):
    return synth(seed, first_frame * n, nframes * n).reshape(nframes, n)


def tables(n, sample_rate=44100.0, num_mel=26):
    L = lib()
    t = {k: np.empty(n, np.float32) for k in ("hann", "hamming", "bark")}
    L.oracle_hanning(n, _p(t["hann"]))
    L.oracle_hamming(n, _p(t["hamming"]))
    L.oracle_bark_scale(n, sample_rate, _p(t["bark"]))
    t["bblimits"] = np.empty(NUM_BARK + 1, np.int32)
    L.oracle_bark_band_limits(_p(t["bark"]), n // 2, NUM_BARK, _p(t["bblimits"], ctypes.c_int32))
    t["mel_bins"] = np.empty(num_mel + 2, np.int32)
    t["mel_values"] = np.empty(num_mel + 2, np.float32)
    t["mel_freq"] = np.empty(num_mel + 2, np.float32)
    L.oracle_mel_bins(n, sample_rate, num_mel, _p(t["mel_bins"], ctypes.c_int32),
                      _p(t["mel_values"]), _p(t["mel_freq"]))
    t["dct"] = np.empty(NUM_COEFFS * num_mel, np.float32)
    L.oracle_dct(num_mel, _p(t["dct"]))
    nst = int(np.log2(n))
    t["twiddle_seeds"] = np.empty(2 * nst, np.float64)
    L.oracle_twiddle_seeds(n, _p(t["twiddle_seeds"], ctypes.c_double))
    return t
