#!/usr/bin/env python3
"""Time the extraction kernel for several feature sets / precisions (ablation by request)."""
import os
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from meyda_amd import capi  # noqa: E402

SETS = {
    "time_only": ["rms", "energy", "zcr"],
    "centroid": ["spectralCentroid"],
    "spectral": ["spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff", "spectralSpread",
                 "spectralSkewness", "spectralKurtosis"],
    "spectral+loud": ["spectralCentroid", "spectralFlatness", "spectralSlope", "spectralRolloff", "spectralSpread",
                      "spectralSkewness", "spectralKurtosis", "loudness", "perceptualSpread", "perceptualSharpness"],
    "mfcc": ["mfcc"],
    "all": capi.ALL_FEATURES,
    "amp+centroid": ["amplitudeSpectrum", "spectralCentroid"],
}


def time_it(plan, frames, o, reps=10):
    s = torch.cuda.current_stream()
    for _ in range(2):
        plan.extract_device(frames.data_ptr(), frames.shape[0], o, s.cuda_stream)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        plan.extract_device(frames.data_ptr(), frames.shape[0], o, s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    res = {}
    for n in [int(v) for v in (sys.argv[1:] or ["1024"])]:
        F = 262144 if n <= 1024 else 131072
        frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
        capi.synth_frames_device(frames, 0x6D657964)
        for prec in ["faithful", "fast"]:
            plan = capi.Plan(buffer_size=n, precision=prec)
            for name, feats in SETS.items():
                _, o = plan.alloc_outputs(F, feats)
                ms = time_it(plan, frames, o)
                key = "N%d/%s/%s" % (n, prec, name)
                res[key] = {"ms": ms, "Mframes_s": F / ms / 1e3}
                print("%-34s %8.3f ms  %8.1f Mframes/s" % (key, ms, F / ms / 1e3), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
