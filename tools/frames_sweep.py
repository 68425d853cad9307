"""Kernel time vs batch size (N=1024, all features): fixed per-launch cost (ramp-up, tail)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import time
import torch
from meyda_amd import SEED, capi

n = 1024
for F in (32768, 65536, 131072, 262144, 524288, 1048576):
    frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, SEED)
    plan = capi.Plan(buffer_size=n)
    _, o = plan.alloc_outputs(F, capi.ALL_FEATURES)
    s = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
        plan.extract_device(frames.data_ptr(), F, o, s.cuda_stream)
        torch.cuda.synchronize()
    reps = max(5, int(20 * 262144 / F))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        plan.extract_device(frames.data_ptr(), F, o, s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print("F=%8d  %.4f ms  %.3f ns/frame" % (F, ms, ms * 1e6 / F), flush=True)
    del frames, o, plan
