#!/bin/bash
# The per-group workgroup barrier every K groups (ab/libgsync{,2,4}.so: -DMGX_GROUP_SYNC=1/2/4) against the
# tree: outputs bit for bit, interleaved timing, WRITE_SIZE (PMC) of the all-feature and time-only sets.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/gsync2
mkdir -p $O && cd $R
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_libs.py --rounds 7 --compare "$@" BASE=base K1=ab/libgsync.so K2=ab/libgsync2.so K4=ab/libgsync4.so > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; grep -v amdgpu.ids $O/$tag.log | sed "s/^/$tag /"; }
run all1024 --n 1024
run time1024 --n 1024 --features rms,energy,zcr
run all2048 --n 2048 --frames 131072
run c3 --n 1024 --features spectralCentroid,spectralFlatness,spectralSlope,spectralRolloff,spectralSpread,spectralSkewness,spectralKurtosis,loudness,perceptualSpread,perceptualSharpness
cd /tmp && export TMPDIR=/tmp
for lib in gsync2 gsync4; do
  export MEYDA_AMD_LIB=$R/ab/lib$lib.so
  for set in time_only all; do
    PROBE_SET=$set timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w.$set.$lib -o run \
      -- python3 $R/tools/pmc_probe.py > $O/w.$set.$lib.log 2>&1 || { echo "pmc failed $set $lib"; tail -5 $O/w.$set.$lib.log; exit 1; }
  done
done
unset MEYDA_AMD_LIB
python3 - "$O" <<'PY'
import csv, glob, sys
O = sys.argv[1]
for d in sorted(glob.glob(O + "/w.*/")):
    xs = {}
    for f in glob.glob(d + "**/run_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "extract_kernel" in row.get("Kernel_Name", ""):
                xs.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for k, v in xs.items():
        print(d.rstrip("/").split("/")[-1], k, "mean %.1f KiB over %d dispatches" % (sum(v) / len(v), len(v)))
PY
