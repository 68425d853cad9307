#!/bin/bash
# rocprofv3 --kernel-trace --stats of the headline bench with its launches on one stream (per-launch
# AverageNs), the headline kernel only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/prof1
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --single-stream --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c3 --no-c4 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 20 > $O/prof_summary.txt; cat $O/prof_summary.txt; cat $O/prof/run_kernel_stats.csv | head -4
