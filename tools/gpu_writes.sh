#!/bin/bash
# WRITE_SIZE (PMC) of the extraction kernel per feature set and work-share layout: the default
# resident grid (rank-weighted shares at N = 1024) against MGX_GRID_CAP=1020 (equal shares).
# Output: gpurun_out/writes/<set>.<cap>.log and the counter CSVs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/writes
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
for set in ${WRITE_SETS:-time_only all}; do
  for cap in ${WRITE_CAPS:-default 1020}; do
    if [ "$cap" = default ]; then unset MGX_GRID_CAP; else export MGX_GRID_CAP=$cap; fi
    PROBE_SET=$set PROBE_N=${PROBE_N:-1024} timeout -k 10 120 \
      rocprofv3 --pmc ${WRITE_CTR:-WRITE_SIZE} --kernel-trace --output-format csv -d $O/$set.$cap -o run \
      -- python3 $R/tools/pmc_probe.py > $O/$set.$cap.log 2>&1 || { echo "pmc failed $set $cap"; exit 1; }
  done
done
unset MGX_GRID_CAP
python3 - "$O" <<'PY'
import csv, glob, sys
O = sys.argv[1]
for d in sorted(glob.glob(O + "/*.*/")):
    xs = {}
    for f in glob.glob(d + "**/run_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row.get("Kernel_Name", ""):
                xs.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for k, v in xs.items():
        print(d.rstrip("/").split("/")[-1], k, "mean %.1f KB over %d dispatches" % (sum(v) / len(v), len(v)))
PY
