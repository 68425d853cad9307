#!/usr/bin/env python3
"""Cost of the group's chunked extraction on one GPU (no transfers): one plan launch over
262,144 x 1024 frames vs a one-rank group at 1, 2, 4 and 8 chunks (all features)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402


def timeit(step, reps=20):
    s = torch.cuda.current_stream()
    for _ in range(30):
        step(s.cuda_stream)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        step(s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


n, F = 1024, 262144
x = torch.empty(F, n, dtype=torch.float32, device="cuda")
capi.synth_frames_device(x, 0x6D657964)
plan = capi.Plan(buffer_size=n)
outs, o = plan.alloc_outputs(F, capi.ALL_FEATURES)
mask = capi.output_mask(o)
g = capi.Group(buffer_size=n, rank=0, nranks=1, device=0)
print("plan          %.4f ms" % timeit(lambda s: plan.extract_device(x.data_ptr(), F, o, s)))
for nch in (1, 2, 4, 8):
    print("group %d chunk %.4f ms" % (nch, timeit(lambda s: g.extract_device([x.data_ptr()], [F], o, mask, nch, [s]))))
