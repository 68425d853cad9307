#!/usr/bin/env python3
"""VALU instruction mix of the bench kernel from the rocprofv3 PMC passes of
tools/gpu_pmc_cur.sh (gpurun_out/pmc/base/*), per frame, weighted by the measured issue
costs of tools/ubench/op_rates (profiles/r01_op_rates.log) into an estimate of the VALU
busy fraction. Writes profiles/pmc_valu.json (a report; bench.py takes its own counters live).
Counter durations under PMC collection are not used: the busy estimate divides by the
kernel time measured without the profiler (the launch duration of the committed bench line,
profiles/r04_bench.log)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = 262144
# SIMD cycles per wave64 instruction (profiles/r01_op_rates.log)
COST = {"SQ_INSTS_VALU_FMA_F64": 5.07, "SQ_INSTS_VALU_MUL_F64": 4.99, "SQ_INSTS_VALU_ADD_F64": 4.75,
        "SQ_INSTS_VALU_CVT": 4.19, "SQ_INSTS_VALU_TRANS_F64": 16.3, "SQ_INSTS_VALU_TRANS_F32": 8.1,
        "SQ_INSTS_VALU_FMA_F32": 2.73, "SQ_INSTS_VALU_ADD_F32": 2.69, "SQ_INSTS_VALU_MUL_F32": 2.7}
OTHER = 3.5  # the remaining VALU instructions (int, moves, compares, selects 4.5, DPP 4.4, packed 5)


def main():
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(ROOT, "gpurun_out/pmc/base/*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row["Kernel_Name"]:
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not agg:
        sys.exit("no extract_kernel PMC rows under gpurun_out/pmc/base")
    per = {k: sum(v) / len(v) / F for k, v in agg.items()}
    valu = per["SQ_INSTS_VALU"]
    known = sum(per.get(k, 0.0) for k in COST)
    cycles = sum(per.get(k, 0.0) * c for k, c in COST.items()) + (valu - known) * OTHER
    bench = json.loads(open(os.path.join(ROOT, "profiles/r04_bench.log")).read().strip().splitlines()[-1])
    kms = bench["roofline"]["kernel_ms"]
    frame_cycles = kms * 1e-3 * 2.4e9 * 1024 / F  # SIMD cycles per frame: 1,024 SIMDs at 2.4 GHz (GRBM_GUI_ACTIVE)
    f64 = sum(per.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                         "SQ_INSTS_VALU_TRANS_F64"))
    out = {"faithful_n1024_f262144": {
        "valu_instr_per_frame": valu, "f64_instr_per_frame": f64, "cvt_instr_per_frame": per["SQ_INSTS_VALU_CVT"],
        "lds_instr_per_frame": per.get("SQ_INSTS_LDS"), "vmem_rd_per_frame": per.get("SQ_INSTS_VMEM_RD"),
        "est_valu_cycles_per_frame": cycles, "frame_cycles": frame_cycles,
        "est_valu_busy": cycles / frame_cycles,
        "est_fp64_pipe_busy": (sum(per.get(k, 0.0) * COST[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                                     "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64",
                                                                     "SQ_INSTS_VALU_CVT"))) / frame_cycles,
        "kernel_ms": kms, "counters_per_frame": per}}
    json.dump(out, open(os.path.join(ROOT, "profiles/pmc_valu.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out["faithful_n1024_f262144"].items() if k != "counters_per_frame"}, indent=1))


if __name__ == "__main__":
    main()
