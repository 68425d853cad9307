#!/bin/bash
# DCT-on-MFMA parity; A/B timings of the ablations and the MFMA DCT; PMC: clock and MFMA counters.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2d
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "dct_on_matrix" -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/dct_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|equals" $O/dct_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
A=$R/abl
timeout -k 10 400 python tools/ab_libs.py base=base dct_mfma=base:1 no_phase2=$A/libabl_no_phase2.so no_loud2=$A/libabl_no_loud2.so no_ln=$A/libabl_no_ln.so no_dct=$A/libabl_no_dct.so no_scalars=$A/libabl_no_scalars.so no_mel=$A/libabl_no_mel.so > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp PROBE_SET=all
for set in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES"; do
  tag=$(echo $set | cut -d' ' -f1)
  for v in base dct; do
    if [ $v = dct ]; then export MGX_PROBE_FLAGS=1; else unset MGX_PROBE_FLAGS; fi
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc/$v/$tag -o run -- python3 $R/tools/pmc_probe.py > $O/pmc_${v}_$tag.log 2>&1 || { echo "pmc failed $v $set"; tail -5 $O/pmc_${v}_$tag.log; exit 1; }
  done
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for v in ("base", "dct"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{O}/pmc/{v}/*/run_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row.get("Kernel_Name", ""):
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", v)
    for k in sorted(agg):
        vals = agg[k]
        print("  %-28s %14.6g  (n=%d)" % (k, sum(vals) / len(vals), len(vals)))
PY
