#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/prof2 && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-host-path --no-pmc --no-every-output > $O/prof_bench.log 2>&1
rc=$?; tail -1 $O/prof_bench.log; [ $rc -ne 0 ] && exit $rc
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 20
