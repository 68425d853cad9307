#!/bin/bash
# PMC passes (kernel-trace only, no sys/runtime trace) for the libs given as args.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then unset MEYDA_AMD_LIB; else export MEYDA_AMD_LIB=$R/abl/libabl_$v.so; fi
  IFS='|' read -ra SETS <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS|SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES|SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64}"
  for set in "${SETS[@]}"; do
    tag=$(echo $set | tr ' ' '_' | cut -c1-40)
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$v/$tag -o run -- python3 $R/tools/pmc_probe.py > /dev/null 2>&1 || { echo "pmc failed $v $set"; exit 1; }
  done
done
python3 - "$R" "$@" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
for v in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{R}/gpurun_out/pmc/{v}/*/run_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row.get("Kernel_Name", ""):
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", v)
    for k in sorted(agg):
        vals = agg[k]
        print("  %-28s %14.4g  (n=%d)" % (k, sum(vals) / len(vals) * 1.0, len(vals)))
PY
