#!/usr/bin/env python3
"""A/B timing of library builds in ONE process, interleaved rounds (cdna_hip_programming.md
§5.4 rule 24): each build (abl/libabl_*.so or any libmeyda_gpu.so copy) is loaded with its
own ctypes handle; per round, every variant times 20 launches of the all-feature batch
(262,144 x N=1024 unless --n/--frames); prints the median and min per variant.
usage: ab_libs.py [--n N] [--frames F] [--rounds R] [--compare] NAME=PATH[:flags] ...   (PATH 'base' = the tree's library)"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    L.mgx_plan_create.argtypes = [ctypes.POINTER(capi.PlanDesc), ctypes.POINTER(ctypes.c_void_p)]
    L.mgx_extract_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.POINTER(capi.Outputs), ctypes.c_void_p]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--features", default="all")
    ap.add_argument("--mel", type=int, default=26, help="mel bands of every plan")
    ap.add_argument("--precision", default="faithful", choices=["faithful", "fast"])
    ap.add_argument("--compare", action="store_true", help="also check every variant's outputs against the first's, bit for bit")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    n, F = a.n, a.frames
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    feats = capi.ALL_FEATURES if a.features == "all" else a.features.split(",")
    plan0 = capi.Plan(buffer_size=n, precision=a.precision, num_mel_bands=a.mel)
    outs, o = plan0.alloc_outputs(F, feats)
    vs = []
    for spec in a.variants:
        name, path = spec.split("=", 1)
        flags = 0
        if ":" in path:
            path, fl = path.split(":", 1)
            flags = int(fl, 0)
        path = capi.LIB_PATH if path == "base" else path
        L = load(path)
        d = capi.make_desc(buffer_size=n, precision=a.precision, num_mel_bands=a.mel)
        d.flags = flags
        h = ctypes.c_void_p()
        rc = L.mgx_plan_create(ctypes.byref(d), ctypes.byref(h))
        assert rc == 0, (name, rc)
        vs.append((name, L, h))
    s = torch.cuda.current_stream()
    res = {name: [] for name, _, _ in vs}
    for _ in range(3):  # clock settle
        for name, L, h in vs:
            for _ in range(20):
                L.mgx_extract_device(h, ctypes.c_void_p(x.data_ptr()), F, ctypes.byref(o), ctypes.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, L, h in vs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                L.mgx_extract_device(h, ctypes.c_void_p(x.data_ptr()), F, ctypes.byref(o), ctypes.c_void_p(s.cuda_stream))
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 20)
    if a.compare:
        first = None
        for name, L, h in vs:
            got, og = plan0.alloc_outputs(F, feats)
            for t in got.values():
                t.fill_(float("nan"))
            L.mgx_extract_device(h, ctypes.c_void_p(x.data_ptr()), F, ctypes.byref(og), ctypes.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            bits = {k: t.view(torch.int32 if t.element_size() == 4 else torch.int64) for k, t in got.items()}
            if first is None:
                first = bits
                continue
            diff = [k for k in bits if not torch.equal(bits[k], first[k])]
            print("%-14s outputs %s" % (name, "identical to %s" % vs[0][0] if not diff else "DIFFER in %s" % diff))
    base = np.median(res[vs[0][0]])
    for name, _, _ in vs:
        m = np.median(res[name])
        print("%-14s median %.4f ms  min %.4f ms  (%+.1f %% vs %s)  %.1f M frames/s" %
              (name, m, np.min(res[name]), (m / base - 1) * 100, vs[0][0], F / m / 1e3))


if __name__ == "__main__":
    main()
