import sys, numpy as np, torch
sys.path.insert(0, '.')
from meyda_amd import capi
from oracle import oracle
n = 1024
for feats in (["mfcc", "amplitudeSpectrum", "spectralCentroid"], ["mfcc", "amplitudeSpectrum"], ["mfcc"]):
    for F in (40, 4096, 65549):
        x = torch.empty(F, n, dtype=torch.float32, device="cuda")
        capi.synth_frames_device(x, 0x5EED)
        plan = capi.Plan(buffer_size=n, mfcc_reference=True)
        out = plan.extract_torch(x, feats)
        torch.cuda.synchronize()
        m = out["mfcc"].cpu().numpy()
        ref = oracle.extract(x[:8].cpu().numpy())
        print(feats, F, "nan frac", np.isnan(m).mean(), "first equal", np.array_equal(m[:8], ref["mfcc"]), flush=True)
