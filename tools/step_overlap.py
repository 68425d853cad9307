#!/usr/bin/env python3
"""Where the time between extraction launches goes (262,144 x N=1024, all features): K
back-to-back steps timed by the host clock around device synchronisations, (a) with a HIP
event pair around every step (bench.py's run_mode), (b) without events, (c) consecutive
steps alternating between two streams with two output sets, so step i+1's workgroups start
while step i drains. Prints ms per step for each, interleaved over several rounds.
usage: step_overlap.py [--n N] [--frames F] [--steps K] [--rounds R]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n, F, K = a.n, a.frames, a.steps
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    plan = capi.Plan(buffer_size=n, device=0)
    _, o0 = plan.alloc_outputs(F, capi.ALL_FEATURES)
    _, o1 = plan.alloc_outputs(F, capi.ALL_FEATURES)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]

    def events():
        for i in range(K):
            ev[i][0].record(s0)
            plan.extract_device(x.data_ptr(), F, o0, s0.cuda_stream)
            ev[i][1].record(s0)

    def plain():
        for _ in range(K):
            plan.extract_device(x.data_ptr(), F, o0, s0.cuda_stream)

    def two_streams():
        e = torch.cuda.Event()
        e.record(s0)
        s1.wait_event(e)
        for i in range(K):
            if i & 1:
                plan.extract_device(x.data_ptr(), F, o1, s1.cuda_stream)
            else:
                plan.extract_device(x.data_ptr(), F, o0, s0.cuda_stream)
        e2 = torch.cuda.Event()
        e2.record(s1)
        s0.wait_event(e2)

    H = F // 2
    _, oa = plan.alloc_outputs(H, capi.ALL_FEATURES)
    _, ob = plan.alloc_outputs(F - H, capi.ALL_FEATURES)
    xb = x[H:]

    def split2():
        # one step = two half launches on the two streams, joined at the step's end (what an
        # internal split of one call would do)
        for _ in range(K):
            e = torch.cuda.Event()
            e.record(s0)
            s1.wait_event(e)
            plan.extract_device(x.data_ptr(), H, oa, s0.cuda_stream)
            plan.extract_device(xb.data_ptr(), F - H, ob, s1.cuda_stream)
            e2 = torch.cuda.Event()
            e2.record(s1)
            s0.wait_event(e2)

    modes = {"events": events, "plain": plain, "two_streams": two_streams, "split2": split2}
    res = {m: [] for m in modes}
    for m in modes.values():  # warm up every mode (clock settle)
        for _ in range(3):
            m()
        torch.cuda.synchronize()
    for r in range(a.rounds):
        for name, m in modes.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / K * 1e3)
        print("round %d: %s" % (r, "  ".join("%s %.4f" % (k, v[-1]) for k, v in res.items())), flush=True)
    ev_ms = float(np.mean([p.elapsed_time(q) for p, q in ev]))
    base = np.median(res["events"])
    for k, v in res.items():
        print("%-12s median %.4f ms/step  min %.4f  (%+.2f %% vs events)  %.1f M frames/s"
              % (k, np.median(v), np.min(v), 100 * (np.median(v) / base - 1), F / np.median(v) / 1e3))
    print("event-timed kernel mean (last events round) %.4f ms" % ev_ms)

    # Per launch on the two streams (an extra, untimed pass of the two_streams schedule with an event pair
    # around every launch): each stream's launch durations, and how far launch k+1 (the other stream) starts
    # before launch k ends (its overlap into k's drain) -- what bench.py's pipelined period rests on.
    pe = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    e = torch.cuda.Event()
    e.record(s0)
    s1.wait_event(e)
    for i in range(K):
        st = s1 if i & 1 else s0
        pe[i][0].record(st)
        plan.extract_device(x.data_ptr(), F, o1 if i & 1 else o0, st.cuda_stream)
        pe[i][1].record(st)
    torch.cuda.synchronize()
    t0 = pe[0][0]
    starts = np.array([t0.elapsed_time(p) for p, _ in pe])
    ends = np.array([t0.elapsed_time(q) for _, q in pe])
    dur = ends - starts
    ov = ends[:-1] - starts[1:]  # > 0: launch k+1 began before launch k ended
    period = (ends[-1] - starts[0]) / K
    print("per launch, two streams (event pair around each launch, untimed pass of %d launches):" % K)
    print("  stream 0 launch %.4f ms (mean of %d), stream 1 %.4f ms (%d); period %.4f ms"
          % (dur[0::2].mean(), len(dur[0::2]), dur[1::2].mean(), len(dur[1::2]), period))
    print("  launch k+1 starts before launch k ends by: median %.4f ms, min %.4f, max %.4f (0: no overlap)"
          % (np.median(ov), ov.min(), ov.max()))
    print("  first launches: durations %s; overlaps %s" % (np.round(dur[:4], 4).tolist(), np.round(ov[:3], 4).tolist()))


if __name__ == "__main__":
    main()
