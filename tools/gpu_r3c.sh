#!/bin/bash
# Round-3 evidence refresh of the current tree: precision report, the bench line, a rocprofv3
# --kernel-trace --stats run of the same bench command with --single-stream (whole, non-overlapping
# launches: the stats' AverageNs is a launch duration) and the PMC traffic.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/${R3_TAG:-r3c}
mkdir -p $O && cd $R
echo "[r3c] precision"
timeout -k 10 300 python tools/precision_report.py 512 1024 2048 > $O/precision.log 2>&1 || { tail -20 $O/precision.log; exit 1; }
echo "[r3c] bench"
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
echo "[r3c] rocprof (single stream)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --single-stream --steps 100 --warmup 20 --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c3 --no-c4 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -c 400 $O/prof_bench.log
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 20 > $O/prof_summary.txt && cat $O/prof_summary.txt
echo "[r3c] traffic"
$R/tools/gpu_traffic.sh > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp $R/gpurun_out/traffic/summary.json $O/pmc_traffic.json
echo "[r3c] done"
