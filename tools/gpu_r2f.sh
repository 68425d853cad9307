#!/bin/bash
# Full GPU suite; A/B default (MFMA DCT) vs MGX_FLAG_DCT_SEQUENTIAL; MFMA PMC counters of both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2f
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "equals the seq|passed|failed|Error" $O/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_libs.py --rounds 7 mfma_dct=base sequential_dct=base:1 > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp PROBE_SET=all
set="SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in mfma seq; do
  if [ $v = seq ]; then export MGX_PROBE_FLAGS=1; else unset MGX_PROBE_FLAGS; fi
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc/$v -o run -- python3 $R/tools/pmc_probe.py > $O/pmc_$v.log 2>&1 || { echo "pmc failed $v"; tail -5 $O/pmc_$v.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for v in ("mfma", "seq"):
    agg = collections.defaultdict(list)
    dur = []
    for f in glob.glob(f"{O}/pmc/{v}/run_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row.get("Kernel_Name", ""):
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", v, "(per launch of 262,144 frames, N=1024, all features)")
    for k in sorted(agg):
        print("  %-28s %14.6g" % (k, sum(agg[k]) / len(agg[k])))
PY
