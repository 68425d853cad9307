#!/usr/bin/env python3
"""Max relative deviation of each GPU output from the CPU oracle on seeded noise and
structured frames (informational; the pass/fail bars live in tests/)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from meyda_amd import capi  # noqa: E402
from oracle import oracle  # noqa: E402

for n in [int(v) for v in (sys.argv[1:] or ["1024"])]:
    F = 2048
    x = oracle.synth_frames(0x6D657964, 0, F, n)
    t = np.arange(n)
    x[:64] = (np.sin(2 * np.pi * 440 * t / 44100) * 0.5).astype(np.float32)
    x[64:128] = (np.sin(2 * np.pi * 3000 * t / 44100) * 1e-3).astype(np.float32)
    ref = oracle.extract(x)
    plan = capi.Plan(buffer_size=n)
    got = plan.extract(x, capi.ALL_FEATURES + ["amplitudeSpectrum"])
    pairs = [("amplitudeSpectrum", ref["amp"]), ("loudness.specific", ref["loudness_specific"]),
             ("mfcc", ref["mfcc"])]
    pairs += [(nm, ref["scalars"][:, i]) for i, nm in enumerate(capi.SCALAR_NAMES)]
    for k, b in pairs:
        if k not in got:
            continue
        a, b = np.asarray(got[k], np.float64), np.asarray(b, np.float64)
        rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
        rel[~np.isfinite(rel)] = 0
        print("N=%d %-24s max rel %.3e  exact %.4f" % (n, k, rel.max(), np.mean(a == b)), flush=True)
