#!/usr/bin/env python3
"""Cost of MGX_FLAG_MFCC_REFERENCE (the mel sums as chains in the reference's order) against the
default plan, interleaved in one process: each round times 20 launches of each plan over the
same device batch (262,144 frames unless --frames), one stream; prints median / min per plan and
the ratio. usage: mfcc_cost.py [--n N ...] [--features all|mfcc|c4] [--rounds R]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1024, 512])
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--features", default="all")
    a = ap.parse_args()
    s = torch.cuda.current_stream()
    for n in a.n:
        F = a.frames if n <= 1024 else a.frames // 2
        x = torch.empty(F, n, dtype=torch.float32, device="cuda")
        capi.synth_frames_device(x, 0x6D657964)
        bands = 40 if a.features == "c4" else 26
        feats = capi.ALL_FEATURES if a.features == "all" else ["mfcc"]
        plans = {"default": capi.Plan(buffer_size=n, num_mel_bands=bands),
                 "reference": capi.Plan(buffer_size=n, num_mel_bands=bands, mfcc_reference=True)}
        outs = {k: p.alloc_outputs(F, feats) for k, p in plans.items()}

        def run(k, reps):
            for _ in range(reps):
                plans[k].extract_device(x.data_ptr(), F, outs[k][1], s.cuda_stream)
        for _ in range(3):
            for k in plans:
                run(k, 20)
        torch.cuda.synchronize()
        res = {k: [] for k in plans}
        for _ in range(a.rounds):
            for k in plans:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run(k, 20)
                e1.record(s)
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) / 20)
        m0 = np.median(res["default"])
        for k in plans:
            m = np.median(res[k])
            print("N=%d F=%d %s bands=%d %-9s median %.4f ms  min %.4f ms  (%+.1f %%)  %.1f M frames/s" %
                  (n, F, a.features, bands, k, m, np.min(res[k]), (m / m0 - 1) * 100, F / m / 1e3), flush=True)


if __name__ == "__main__":
    main()
