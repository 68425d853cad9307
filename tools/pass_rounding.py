#!/usr/bin/env python3
"""Settles the per-pass-rounding lever on the CPU, before any GPU time.

jsfft rounds every FFT stage to float32 (lib/jsfft/fft.js:153-161, complex_array.js:7,31-32); the kernel
reproduces it at 2 conversions per value and stage. A precision that rounds only at the kernel's pass
boundaries (its LDS exchanges, R = N/128 slots per lane: stages s = RB, 2 RB, ... and the last) would drop
most of those conversions. This runs that schedule (tools/emu/pass_round.c) -- and, for scale, exact
double (rounded only at the end) -- through the oracle's feature code (oracle.features_from_amp) and the
parity policy of tests/tolerance.py, against:
  * the golden fixtures (tests/golden: the reference's own outputs; noise, sound1/2/3 slices, edge frames);
  * every full non-overlapping frame of the reference's audio/sound{1,2,3}.wav (read here as data; the
    faithful oracle, bit-exact to the reference on the goldens, supplies the expected values).
The faithful schedule (every stage rounded) is run too and must reproduce the oracle exactly.
usage: pass_rounding.py [N ...]   (writes the report to stdout)"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402
import tolerance  # noqa: E402
from oracle import oracle  # noqa: E402

LIB = "/tmp/libpass_round.so"
WAVS = "/root/reference/audio"


def lib():
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off",
                           os.path.join(ROOT, "tools", "emu", "pass_round.c"), "-lm", "-o", LIB])
    L = ctypes.CDLL(LIB)
    fp = ctypes.POINTER(ctypes.c_float)
    L.pr_amp.argtypes = [fp, ctypes.c_int, ctypes.c_uint32, fp]
    return L


def schedules(n):
    B = n.bit_length() - 1
    R = n // 128
    RB = R.bit_length() - 1
    per_pass = 0
    for s in range(B):
        if (s >= RB and s % RB == 0) or s == B - 1:
            per_pass |= 1 << s
    return {"faithful": (1 << B) - 1, "per_pass": per_pass, "exact_f64": 1 << (B - 1)}


def wav_frames(name, n):
    import wave
    with wave.open(os.path.join(WAVS, name), "rb") as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1
        pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")
    x = pcm.astype(np.float32) / np.float32(32768.0)  # decodeAudioData's scaling
    F = len(x) // n
    return x[:F * n].reshape(F, n)


def amps(L, frames, window, mask):
    xw = (frames * window[None, :]).astype(np.float32)
    out = np.empty((frames.shape[0], frames.shape[1] // 2), np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    for f in range(frames.shape[0]):
        row = np.ascontiguousarray(xw[f])
        L.pr_amp(row.ctypes.data_as(fp), frames.shape[1], mask, out[f].ctypes.data_as(fp))
    return out


def relerr(g, r):
    with np.errstate(all="ignore"):
        d = np.abs(g.astype(np.float64) - r.astype(np.float64)) / np.abs(r.astype(np.float64))
    d = d[np.isfinite(d)]
    return float(d.max()) if d.size else 0.0


def compare(n, frames, amp, ref):
    """Per-feature failures under tests/tolerance.py, plus the worst relative errors."""
    got = oracle.features_from_amp(frames, amp)
    res = {}
    fails = tolerance.check_scalars(got["scalars"], ref["scalars"], ref["amp"], n)
    for j, name in enumerate(tolerance.SCALAR_NAMES):
        nf = len([1 for f in fails if f[1] == name])
        res[name] = (nf, relerr(got["scalars"][:, j], ref["scalars"][:, j]))
    bad, exact = tolerance.check_spectra(amp, ref["amp"])
    res["amplitude"] = (len(bad), 1.0 - exact)
    res["loudness.specific"] = (len(tolerance.check_vectors(got["loudness_specific"], ref["loudness_specific"])),
                                relerr(got["loudness_specific"], ref["loudness_specific"]))
    res["mfcc"] = (len(tolerance.check_vectors(got["mfcc"], ref["mfcc"])), relerr(got["mfcc"], ref["mfcc"]))
    return res


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048]
    L = lib()
    print("# Per-pass rounding vs jsfft's per-stage rounding (tools/pass_rounding.py, tools/emu/pass_round.c).")
    print("# Each cell: frames failing the parity bar of tests/tolerance.py / worst relative error of the feature")
    print("# (amplitude: frames failing the norm-wise bar / fraction of bins not bit-exact).")
    print("# Expected values: the reference's own outputs (goldens) and the faithful oracle (whole wav files).")
    verdict = {}
    for n in sizes:
        tab = oracle.tables(n)
        window = np.asarray(tab["hann"], np.float32)
        sch = schedules(n)
        sets = []
        g = golden_io.load(n)
        ref_g = {"scalars": g["scalars"], "amp": g["amp"], "loudness_specific": g["loudness_specific"], "mfcc": g["mfcc"]}
        for cat in ("noise", "sound1", "sound2", "sound3", "edge"):
            ix = golden_io.idx(g["labels"], cat + ":")
            sets.append(("golden " + cat, g["input"][ix], {k: v[ix] for k, v in ref_g.items()}))
        if os.path.isdir(WAVS):
            for w in ("sound1.wav", "sound2.wav", "sound3.wav"):
                fr = wav_frames(w, n)
                ref = oracle.extract(fr)
                sets.append(("wav " + w.split(".")[0], fr, ref))
        print("\n## N = %d  (R = %d slots per lane; per-pass rounding after stages %s)" %
              (n, n // 128, [s for s in range(n.bit_length() - 1) if (sch["per_pass"] >> s) & 1]))
        for sname, mask in sch.items():
            print("\n### %s" % sname)
            header = None
            for label, fr, ref in sets:
                amp = amps(L, fr, window, mask)
                res = compare(n, fr, amp, ref)
                if header is None:
                    header = list(res)
                    print("%-16s %6s  " % ("set", "frames") + "  ".join("%-22s" % h for h in header))
                print("%-16s %6d  " % (label, fr.shape[0]) +
                      "  ".join("%-22s" % ("%d / %.2e" % res[h]) for h in header))
                real = label.startswith(("golden sound", "wav"))
                for h in header:
                    if h == "amplitude":
                        continue
                    key = (n, sname, h)
                    verdict.setdefault(key, [0, 0])
                    verdict[key][0 if real else 1] += res[h][0]
    print("\n## Verdict per schedule (frames failing, real audio / synthetic+edge, summed over sets)")
    for n in sizes:
        for sname in schedules(n):
            bad = {h: v for (nn, s, h), v in verdict.items() if nn == n and s == sname and (v[0] or v[1])}
            print("N=%d %-10s %s" % (n, sname, "PASS every feature" if not bad else
                                      "FAIL " + ", ".join("%s %d/%d" % (h, v[0], v[1]) for h, v in bad.items())))


if __name__ == "__main__":
    main()
