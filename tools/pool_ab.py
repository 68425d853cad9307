#!/usr/bin/env python3
"""The N = 2048 tail pool (MGX_POOL_PCT, read at plan creation; kernels.hip): plans with different pool
shares in ONE process, interleaved rounds of 20 launches of the all-feature batch (262,144 x N unless
--frames), each plan's outputs compared bit for bit with the pool-less plan's.
usage: pool_ab.py [--n 2048] [--frames F] [--rounds R] PCT ..."""
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
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("pcts", nargs="+", type=int)
    a = ap.parse_args()
    n, F = a.n, a.frames
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    plans = []
    for pct in [0] + a.pcts:
        os.environ["MGX_POOL_PCT"] = str(pct)
        plans.append((pct, capi.Plan(buffer_size=n)))
    os.environ.pop("MGX_POOL_PCT")
    s = torch.cuda.current_stream()
    ref = None
    for pct, p in plans:  # outputs, twice in a row (the ticket base carries over between launches)
        for _ in range(2):
            got = p.extract_torch(x, capi.ALL_FEATURES)
        torch.cuda.synchronize()
        bits = {k: t.view(torch.int32 if t.element_size() == 4 else torch.int64) for k, t in got.items()}
        if ref is None:
            ref = bits
        else:
            diff = [k for k in bits if not torch.equal(bits[k], ref[k])]
            print("pool %2d %%  outputs %s" % (pct, "identical to no pool" if not diff else "DIFFER in %s" % diff))
    outs = {pct: p.alloc_outputs(F, capi.ALL_FEATURES)[1] for pct, p in plans}
    res = {pct: [] for pct, _ in plans}
    for _ in range(3):
        for pct, p in plans:
            for _ in range(20):
                p.extract_device(x.data_ptr(), F, outs[pct], s.cuda_stream)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for pct, p in plans:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                p.extract_device(x.data_ptr(), F, outs[pct], s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            res[pct].append(e0.elapsed_time(e1) / 20)
    base = np.median(res[0])
    for pct, _ in plans:
        m = np.median(res[pct])
        print("pool %2d %%  median %.4f ms  min %.4f ms  (%+.1f %% vs no pool)  %.1f M frames/s" %
              (pct, m, np.min(res[pct]), (m / base - 1) * 100, F / m / 1e3))


if __name__ == "__main__":
    main()
