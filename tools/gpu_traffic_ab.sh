#!/bin/bash
# HBM traffic and launch time of library variants side by side (the tree's library and ab/lib_NAME.so
# builds, tools/variant.sh): per library, FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (kernel-trace only) over the time-only set (the read calibration, as tools/gpu_traffic.sh) and the
# all-feature set at N = $PROBE_N, then tools/ab_libs.py timing every library in one process with a
# bit-for-bit output comparison.  usage: tools/gpu_traffic_ab.sh NAME=PATH ...   (PATH 'base' = the tree's)
# Output: gpurun_out/traffic_ab/summary.json and ab.log
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/traffic_ab
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
N=${PROBE_N:-1024}
for spec in "$@"; do
  name=${spec%%=*}; path=${spec#*=}
  [ "$path" = base ] && path=$R/meyda_amd/libmeyda_gpu.so || path=$R/$path
  for set in time_only all; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      echo "pmc $name $set $ctr"
      MEYDA_AMD_LIB=$path PROBE_SET=$set PROBE_N=$N timeout -k 10 180 \
        rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name/$set/$ctr -o run \
        -- python3 $R/tools/pmc_probe.py > $O/$name.$set.$ctr.log 2>&1 || { echo "pmc failed $name $set $ctr"; exit 1; }
    done
  done
done
python3 - "$O" "$N" "$@" <<'PY'
import csv, glob, json, sys
O, n, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
F = 262144
out = {}
for spec in specs:
    name = spec.split("=", 1)[0]
    v = {}
    for s in ("time_only", "all"):
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            xs = [float(r["Counter_Value"]) for f in glob.glob(f"{O}/{name}/{s}/{ctr}/**/run_counter_collection.csv", recursive=True)
                  for r in csv.DictReader(open(f)) if "extract_kernel" in r.get("Kernel_Name", "") and r["Counter_Name"] == ctr]
            v[s + "." + ctr] = sum(xs) / len(xs) if xs else None
    cal = F * n * 4 / (v["time_only.FETCH_SIZE"] * 1024)
    rd, wr = v["all.FETCH_SIZE"] * 1024 * cal, v["all.WRITE_SIZE"] * 1024
    alg = F * (4 * n + 4 * 50)
    out[name] = {"read_bytes": rd, "write_bytes": wr, "traffic_over_algorithmic": (rd + wr) / alg, "raw_kb": v,
                 "read_calibration": cal, "algorithmic_bytes": alg}
    print(name, json.dumps(out[name]))
json.dump(out, open(f"{O}/summary.json", "w"), indent=1)
PY
[ $? -eq 0 ] || exit 1
args=()
for spec in "$@"; do
  name=${spec%%=*}; path=${spec#*=}
  [ "$path" = base ] && args+=("$spec") || args+=("$name=$R/$path")
done
timeout -k 10 300 python3 $R/tools/ab_libs.py --n $N --rounds 7 --compare "${args[@]}" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
