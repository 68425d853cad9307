#!/bin/bash
# Full GPU tests, smoke, bench (with the JS CPU baseline), and the rocprofv3 kernel trace
# of a bench run; each GPU step under its own limit, stop at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2c
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -6 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
rc=$?; tail -2 $O/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-path > $O/prof_bench.log 2>&1
rc=$?; tail -1 $O/prof_bench.log; [ $rc -ne 0 ] && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py $f 20 > $O/prof_summary.txt && cat $O/prof_summary.txt
