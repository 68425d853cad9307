#!/usr/bin/env python3
"""Dynamic instruction budget by ablation: every library given (abl/ or ab/ builds of
tools/ablate.py, 'base' = the tree's library) runs REPS launches of the all-feature batch
(262,144 x N = 1024) in ONE process, in the order given, so one rocprofv3 --pmc pass per
counter set covers every variant; dispatch k of the extract kernel belongs to variant
k // REPS (tools/gpu_budget.sh maps them back).
usage: pmc_budget.py NAME=PATH[:flags] ...  (prints the variant order)
       pmc_budget.py --report DIR NAME ...  (reads DIR/*/run_counter_collection.csv)"""
import csv
import ctypes
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPS = int(os.environ.get("PROBE_REPS", "2"))
F = 262144


def run(specs):
    import torch
    from meyda_amd import capi
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from ab_libs import load
    n = int(os.environ.get("PROBE_N", "1024"))
    x = torch.empty(F, n, dtype=torch.float32, device="cuda")
    capi.synth_frames_device(x, 0x6D657964)
    prec = os.environ.get("PROBE_PRECISION", "faithful")  # "fast": the f32-butterfly kernels
    plan0 = capi.Plan(buffer_size=n)
    _, o = plan0.alloc_outputs(F, capi.ALL_FEATURES)
    s = torch.cuda.current_stream()
    for spec in specs:
        name, path = spec.split("=", 1)
        flags = 0
        if ":" in path:
            path, fl = path.split(":", 1)
            flags = int(fl, 0)
        L = load(capi.LIB_PATH if path == "base" else os.path.join(ROOT, path))
        d = capi.make_desc(buffer_size=n, precision=prec)
        d.flags = flags
        h = ctypes.c_void_p()
        assert L.mgx_plan_create(ctypes.byref(d), ctypes.byref(h)) == 0, name
        for _ in range(REPS):
            L.mgx_extract_device(h, ctypes.c_void_p(x.data_ptr()), F, ctypes.byref(o), ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        print("variant", name)


def report(d, names):
    per = defaultdict(lambda: defaultdict(list))  # counter -> variant -> values
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if "extract_kernel" in r.get("Kernel_Name", "")]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        order = {di: i // REPS for i, di in enumerate(ids)}
        acc = defaultdict(float)
        for r in rows:
            acc[(order[int(r["Dispatch_Id"])], r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
        for (vi, cn, _), v in acc.items():
            if vi < len(names):
                per[cn][names[vi]].append(v)
    cols = sorted(per)
    print("# per frame (counter sum over the dispatch / 262,144 frames; SQ_INSTS_* count wave instructions)")
    def short(c):  # unique column names of at most 10 characters
        for a, b in (("SQ_INSTS_VALU_", "V_"), ("SQ_INSTS_", ""), ("SQ_ACTIVE_INST_", "ACT_"), ("SQ_WAIT_INST_", "WAITI_"), ("SQ_", "")):
            c = c.replace(a, b)
        return c.replace("_CYCLES", "_CYC")[:10]
    print("%-22s" % "variant" + "".join("%11s" % short(c) for c in cols))
    for nm in names:
        vals = []
        for c in cols:
            v = per[c].get(nm)
            vals.append("%11.1f" % (sum(v) / len(v) / F) if v else "%11s" % "-")
        print("%-22s" % nm + "".join(vals))


if __name__ == "__main__":
    if sys.argv[1] == "--report":
        report(sys.argv[2], sys.argv[3:])
    else:
        run(sys.argv[1:])
