#!/usr/bin/env python3
"""Every BASELINE.json config on one GPU (informational; bench.py is the contract line).

C2: 65,536 x N=512, amplitudeSpectrum + spectralCentroid (C2-2GiB: 1,048,576 frames, beyond the MALL)
C3: 262,144 x N=1024, spectral* + loudness (+ perceptual)
C4: 262,144 x N=1024, 40-band mel + 13-coefficient MFCC
C5: 262,144 x N=2048 per GPU (the 8-GPU config's shard), all features incl. MFCC
C34-tone: the bench workload (all features, N=1024) on a 440 Hz tone + noise
Bytes per frame follow SURVEY.md §8(d): 4N in + 4 bytes per output float.
Each row: back-to-back launches on one stream (kernel_ms, the launch on its own) and the same
launches pipelined over two streams and two output sets as bench.py runs its steps
(pipelined_ms, the launch period).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from meyda_amd import SEED, capi  # noqa: E402

SPECTRAL = ["spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff", "spectralSpread",
            "spectralSkewness", "spectralKurtosis"]
CONFIGS = {
    "C2": dict(n=512, F=65536, feats=["amplitudeSpectrum", "spectralCentroid"], out_floats=256 + 1, mel=26),
    # C2 again with a batch 8x the 256 MiB MALL (2 GiB of frames): the 128 MiB C2 batch stays
    # resident in the MALL between launches, so only this row is an HBM fraction
    "C2-2GiB": dict(n=512, F=1048576, feats=["amplitudeSpectrum", "spectralCentroid"], out_floats=256 + 1, mel=26),
    "C3": dict(n=1024, F=262144, feats=SPECTRAL + ["loudness", "perceptualSpread", "perceptualSharpness"],
               out_floats=7 + 25 + 2, mel=26),
    "C4": dict(n=1024, F=262144, feats=["mfcc"], out_floats=13, mel=40),
    "C5": dict(n=2048, F=262144, feats=capi.ALL_FEATURES, out_floats=50, mel=26),
    # SURVEY §8(d) sanity variant: the bench workload on a tone + noise signal instead of
    # uniform noise (data-dependent paths: range checks, small bins)
    "C34-tone": dict(n=1024, F=262144, feats=capi.ALL_FEATURES, out_floats=50, mel=26, tone=True),
}


def tone_frames(frames, n):
    """0.5 sin(2 pi 440 t / 44100) over the whole stream, plus 1e-2 x the seeded noise."""
    F = frames.shape[0]
    t = torch.arange(n, device=frames.device, dtype=torch.float64)[None, :]
    t = t + torch.arange(F, device=frames.device, dtype=torch.float64)[:, None] * n
    sig = 0.5 * torch.sin(2 * torch.pi * 440.0 * t / 44100.0)
    frames.mul_(1e-2).add_(sig.to(torch.float32))


S2 = []  # the second stream, created once


def run(name, cfg, reps=20):
    n, F = cfg["n"], cfg["F"]
    frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(frames, SEED)
    if cfg.get("tone"):
        tone_frames(frames, n)
    plan = capi.Plan(buffer_size=n, num_mel_bands=cfg["mel"])
    _, o = plan.alloc_outputs(F, cfg["feats"])
    _, o2 = plan.alloc_outputs(F, cfg["feats"])
    s = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:  # clock settle
        plan.extract_device(frames.data_ptr(), F, o, s.cuda_stream)
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        plan.extract_device(frames.data_ptr(), F, o, s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    s2 = S2[0] if S2 else S2.append(torch.cuda.Stream()) or S2[0]

    def piped(k):
        e = torch.cuda.Event()
        e.record(s)
        s2.wait_event(e)
        for i in range(k):
            st, oo = (s2, o2) if i & 1 else (s, o)
            plan.extract_device(frames.data_ptr(), F, oo, st.cuda_stream)
        e = torch.cuda.Event()
        e.record(s2)
        s.wait_event(e)
    piped(8)  # (the first launches on a stream's hardware queue carry a one-time cost of milliseconds)
    torch.cuda.synchronize()
    a.record(s)
    piped(reps)
    b.record(s)
    torch.cuda.synchronize()
    pms = a.elapsed_time(b) / reps
    bpf = 4 * n + 4 * cfg["out_floats"]
    gbs = F * bpf / (ms * 1e-3) / 1e9
    r = {"config": name, "n": n, "frames": F, "features": cfg["feats"], "mel_bands": cfg["mel"], "kernel_ms": ms,
         "frames_per_s": F / (ms * 1e-3), "bytes_per_frame": bpf, "achieved_GBs": gbs, "hbm_frac": gbs / 8000.0,
         "pipelined_ms": pms, "pipelined_frames_per_s": F / (pms * 1e-3),
         "pipelined_hbm_frac": F * bpf / (pms * 1e-3) / 1e9 / 8000.0}
    print(json.dumps(r), flush=True)
    return r


if __name__ == "__main__":
    names = sys.argv[1:] or list(CONFIGS)
    out = [run(k, CONFIGS[k]) for k in names]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "configs.json"), "w"), indent=1)
