#!/usr/bin/env python3
"""Run a few extraction launches of one configuration (for rocprofv3 --pmc passes)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from meyda_amd import capi  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prof_variants import SETS  # noqa: E402

n = int(os.environ.get("PROBE_N", "1024"))
feats = SETS[os.environ.get("PROBE_SET", "time_only")]
prec = os.environ.get("PROBE_PREC", "faithful")
F = 262144
frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
capi.synth_frames_device(frames, 0x6D657964)
plan = capi.Plan(buffer_size=n, precision=prec, num_mel_bands=int(os.environ.get("PROBE_BANDS", "26")),
                 dct_sequential=bool(int(os.environ.get("MGX_PROBE_FLAGS", "0")) & 1))
_, o = plan.alloc_outputs(F, feats)
for _ in range(int(os.environ.get("PROBE_REPS", "3"))):
    plan.extract_device(frames.data_ptr(), F, o, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("done", n, feats, prec)
