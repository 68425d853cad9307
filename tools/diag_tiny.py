"""Diagnostics for the tiny-spectrum edge frames: per frame, mfcc / amplitude / scalar
differences between the GPU library (MEYDA_AMD_LIB selects a build) and the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch  # noqa
from meyda_amd import capi
from oracle import oracle
from test_gpu_edge import edge_frames, FEATS
np.set_printoptions(precision=9, linewidth=150)
for n in (512, 1024):
    x = edge_frames(n)
    ref = oracle.extract(x)
    out = capi.Plan(buffer_size=n, scalar_f64=True).extract(x, FEATS)
    for f in range(len(x)):
        g, r = out["mfcc"][f].astype(np.float64), ref["mfcc"][f].astype(np.float64)
        a, ra = out["amplitudeSpectrum"][f].astype(np.float64), ref["amp"][f].astype(np.float64)
        with np.errstate(all="ignore"):
            md = np.nanmax(np.abs(g - r) / np.maximum(np.abs(r), 1e-300))
            ad = np.nanmax(np.abs(a - ra) / np.maximum(np.abs(ra), 1e-300))
        print("n=%d frame %d  amp[min,max]=%.3g,%.3g  amp max rel %.3g  mfcc max rel %.3g" %
              (n, f, np.nanmin(ra), np.nanmax(ra), ad, md))
        if f >= 10 and md > 1e-5:
            print("  gpu mfcc", g[:6]); print("  ref mfcc", r[:6])
            bad = np.nonzero(np.abs(a - ra) > 1e-5 * np.abs(ra))[0]
            print("  amp bad bins", bad[:10], a[bad[:5]], ra[bad[:5]])
