#!/usr/bin/env python3
"""Where a resident one-frame call's time goes (MGX_FLAG_RESIDENT): the median time of
mgx_extract_host on one frame per feature set, resident and launched per call, through the C ABI
(ctypes: its own overhead is the same in every row). Time-domain sets skip the FFT; the differences
between rows are the cost of the parts each set adds. resident_light: MGX_RESIDENT_POLL=light.
usage: resident_features.py [calls]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from meyda_amd import capi  # noqa: E402

SETS = [["zcr"], ["rms"], ["rms", "spectralCentroid"], ["amplitudeSpectrum"], ["spectralRolloff"], ["loudness"],
        ["mfcc"], ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff",
                   "spectralSpread", "spectralSkewness", "spectralKurtosis", "loudness", "perceptualSpread",
                   "perceptualSharpness", "mfcc"]]


def run(p, x, feats, calls):
    out, o = p._host_outputs(1, feats)
    L = capi.lib()
    for _ in range(200):
        capi.check(L.mgx_extract_host(p._h, x.ctypes.data, 1, ctypes.byref(o)))
    t = []
    for _ in range(calls):
        t0 = time.perf_counter_ns()
        L.mgx_extract_host(p._h, x.ctypes.data, 1, ctypes.byref(o))
        t.append((time.perf_counter_ns() - t0) / 1e3)
    t.sort()
    return t[len(t) // 2]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    for n in (512, 1024, 2048):
        x = np.random.default_rng(1).uniform(-1, 1, (1, n)).astype(np.float32)
        res = capi.Plan(buffer_size=n, scalar_f64=True, resident=True)
        os.environ["MGX_RESIDENT_POLL"] = "light"
        light = capi.Plan(buffer_size=n, scalar_f64=True, resident=True)
        del os.environ["MGX_RESIDENT_POLL"]
        lau = capi.Plan(buffer_size=n, scalar_f64=True)
        for feats in SETS:
            r = {"n": n, "features": feats if len(feats) < 5 else "all (%d)" % len(feats),
                 "resident_us": run(res, x, feats, calls), "resident_light_us": run(light, x, feats, calls),
                 "launched_us": run(lau, x, feats, calls)}
            print(json.dumps(r), flush=True)
        res.close()
        light.close()
        lau.close()


if __name__ == "__main__":
    main()
