#!/bin/bash
# Where a wave's cycles go (MI355X_MICROARCH.md PMC table: WAIT_ANY = parked at s_waitcnt /
# barrier, WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing; the three add up to
# WAVE_CYCLES), plus VALU/LDS/SALU activity, for the all-feature N=1024 launch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/stall
mkdir -p $O && cd /tmp && export TMPDIR=/tmp PROBE_SET=all
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/pmc_probe.py > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{O}/p*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if "extract_kernel" in row.get("Kernel_Name", ""):
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
F = 262144
print("per launch of 262,144 frames x N=1024, all features (mean over the probe's launches); per frame = / 262,144")
for k in sorted(agg):
    v = sum(agg[k]) / len(agg[k])
    print("  %-24s %16.6g   per frame %10.2f" % (k, v, v / F))
w = sum(agg["SQ_WAVE_CYCLES"]) / len(agg["SQ_WAVE_CYCLES"])
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
    print("  %-24s %.3f of SQ_WAVE_CYCLES" % (k, (sum(agg[k]) / len(agg[k])) / w))
PY
