#!/usr/bin/env python3
"""Latency of mgx_extract_host for small host batches (the real-time path under the JS facade's
get()/process()): the pinned zero-copy path (plan.cpp extract_host_small) against the staged DMA
path (MGX_SMALL_BATCH_FRAMES=0), median us per call over many calls, outputs compared bit for bit.
usage: host_latency.py [N ...]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from meyda_amd import capi  # noqa: E402


def plan(n, small):
    if small:
        os.environ.pop("MGX_SMALL_BATCH_FRAMES", None)
    else:
        os.environ["MGX_SMALL_BATCH_FRAMES"] = "0"
    p = capi.Plan(buffer_size=n, scalar_f64=True)
    os.environ.pop("MGX_SMALL_BATCH_FRAMES", None)
    return p


def bench(p, x, feats, calls):
    out, o = p._host_outputs(x.shape[0], feats)
    L = capi.lib()
    for _ in range(20):
        capi.check(L.mgx_extract_host(p._h, x.ctypes.data, x.shape[0], ctypes.byref(o)))
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        capi.check(L.mgx_extract_host(p._h, x.ctypes.data, x.shape[0], ctypes.byref(o)))
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6, out


def main():
    rng = np.random.default_rng(1)
    res = []
    for n in [int(v) for v in (sys.argv[1:] or ["512", "1024"])]:
        a, b = plan(n, True), plan(n, False)
        for F, feats in ((1, ["rms", "spectralCentroid"]), (1, capi.ALL_FEATURES), (64, capi.ALL_FEATURES),
                         (512, capi.ALL_FEATURES), (513, capi.ALL_FEATURES)):
            x = rng.uniform(-1, 1, (F, n)).astype(np.float32)
            calls = 2000 if F <= 64 else 300
            ta, oa = bench(a, x, feats, calls)
            tb, ob = bench(b, x, feats, calls)
            same = all(np.array_equal(oa[k].view(np.uint8), ob[k].view(np.uint8)) for k in oa)
            r = {"n": n, "frames": F, "features": len(feats), "small_us": ta, "staged_us": tb, "identical": same}
            print(json.dumps(r), flush=True)
            res.append(r)
    assert all(r["identical"] for r in res)


if __name__ == "__main__":
    main()
