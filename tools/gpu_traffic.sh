#!/bin/bash
# HBM traffic of the extraction kernel from PMC counters (MI355X_MICROARCH.md, HBM section):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel-trace only). The time-only
# feature set reads exactly the frames and writes 3 scalars per frame, which calibrates
# FETCH_SIZE for this kernel's access pattern (gfx950 reports 1/2 of wide streaming reads).
# Output: gpurun_out/traffic/summary.json  (copied into profiles/pmc_traffic.json by hand)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out/traffic && cd /tmp && export TMPDIR=/tmp
for prec in ${TRAFFIC_PRECS:-faithful}; do
  for set in time_only all; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      PROBE_SET=$set PROBE_PREC=$prec PROBE_N=${PROBE_N:-1024} timeout -k 10 180 \
        rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/traffic/$prec/$set/$ctr -o run \
        -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/traffic/$prec.$set.$ctr.log 2>&1 \
        || { echo "pmc failed $prec $set $ctr"; exit 1; }
    done
  done
done
python3 - "$R" <<'PY'
import csv, glob, json, os, sys
R = sys.argv[1]
n = int(os.environ.get("PROBE_N", "1024"))
F = 262144
out = {}
for prec in os.environ.get("TRAFFIC_PRECS", "faithful").split():
    vals = {}
    for s in ("time_only", "all"):
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            xs = []
            for f in glob.glob(f"{R}/gpurun_out/traffic/{prec}/{s}/{ctr}/**/run_counter_collection.csv", recursive=True):
                for row in csv.DictReader(open(f)):
                    if "extract_kernel" in row.get("Kernel_Name", "") and row["Counter_Name"] == ctr:
                        xs.append(float(row["Counter_Value"]))
            vals[(s, ctr)] = sum(xs) / len(xs) if xs else None
    # FETCH_SIZE and WRITE_SIZE are in KB
    frames_bytes = F * n * 4
    fetch_t = vals[("time_only", "FETCH_SIZE")] * 1024
    cal = frames_bytes / fetch_t  # true bytes per counted byte for this read pattern
    fetch_all = vals[("all", "FETCH_SIZE")] * 1024 * cal
    write_all = vals[("all", "WRITE_SIZE")] * 1024
    key = "%s_n%d_f%d" % (prec, n, F)
    out[key] = {
        "hbm_bytes_per_launch": fetch_all + write_all,
        "read_bytes": fetch_all, "write_bytes": write_all,
        "fetch_size_kb_raw": vals[("all", "FETCH_SIZE")], "write_size_kb_raw": vals[("all", "WRITE_SIZE")],
        "calibration": {"time_only_fetch_kb": vals[("time_only", "FETCH_SIZE")],
                        "time_only_write_kb": vals[("time_only", "WRITE_SIZE")],
                        "frames_bytes": frames_bytes, "factor": cal},
        "algorithmic_bytes_per_launch": F * (4 * n + 4 * 50),
    }
    print(key, json.dumps(out[key], indent=1))
os.makedirs(f"{R}/gpurun_out/traffic", exist_ok=True)
json.dump(out, open(f"{R}/gpurun_out/traffic/summary.json", "w"), indent=1)
PY
