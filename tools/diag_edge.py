import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch  # noqa
from meyda_amd import capi
from oracle import oracle
from test_gpu_edge import edge_frames
for n in (256, 1024):
    x = edge_frames(n)
    ref = oracle.extract(x)
    out = capi.Plan(buffer_size=n, scalar_f64=True).extract(x, ["amplitudeSpectrum"])
    a, r = out["amplitudeSpectrum"], ref["amp"]
    for f in range(len(x)):
        dn = np.nonzero(np.isnan(a[f]) != np.isnan(r[f]))[0]
        di = np.nonzero(np.isinf(a[f]) != np.isinf(r[f]))[0]
        if len(dn) or len(di):
            print(n, f, "nan-diff bins", dn[:10], len(dn), "inf-diff", di[:10], len(di),
                  "gpu", a[f][dn[:4]], "ref", r[f][dn[:4]], "nan counts", np.isnan(a[f]).sum(), np.isnan(r[f]).sum())
