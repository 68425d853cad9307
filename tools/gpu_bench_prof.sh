#!/bin/bash
# The bench line (with its live PMC passes and CPU baseline), a rocprofv3 kernel trace + stats
# of a bench run (summary over the timed launches), and every BASELINE config on one GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/bench
mkdir -p $O && cd $R
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-host-path --no-pmc --no-every-output > $O/prof_bench.log 2>&1
rc=$?; tail -1 $O/prof_bench.log; [ $rc -ne 0 ] && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py $f 100 > $O/prof_summary.txt && cat $O/prof_summary.txt
cd $R
timeout -k 10 300 python tools/configs_bench.py > $O/configs.log 2>&1
rc=$?; cat $O/configs.log | grep config; [ $rc -ne 0 ] && exit $rc
exit 0
