#!/bin/bash
# A workgroup barrier after each full group of 16 frames (-DMGX_GROUP_SYNC=1, ab/libgsync.so) against
# the tree: outputs bit for bit and interleaved timing per feature set, then WRITE_SIZE (PMC) of both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/gsync
mkdir -p $O && cd $R
run() { tag=$1; shift; timeout -k 10 200 python tools/ab_libs.py --rounds 5 --compare "$@" BASE=base GSYNC=ab/libgsync.so > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; grep -v amdgpu.ids $O/$tag.log | sed "s/^/$tag /"; }
run all1024 --n 1024
run time1024 --n 1024 --features rms,energy,zcr
run c3 --n 1024 --features spectralCentroid,spectralFlatness,spectralSlope,spectralRolloff,spectralSpread,spectralSkewness,spectralKurtosis,loudness,perceptualSpread,perceptualSharpness
run all512 --n 512
run all2048 --n 2048 --frames 131072
run c2 --n 512 --frames 65536 --features amplitudeSpectrum,spectralCentroid
cd /tmp && export TMPDIR=/tmp
for lib in base gsync; do
  if [ $lib = gsync ]; then export MEYDA_AMD_LIB=$R/ab/libgsync.so; else unset MEYDA_AMD_LIB; fi
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
        print(d.rstrip("/").split("/")[-1], k, "mean %.1f KB over %d dispatches" % (sum(v) / len(v), len(v)))
PY
