#!/bin/bash
# Round-2 GPU round trip: parity tests, smoke, bench. Each GPU step has its own limit;
# the script stops at the first failing step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} > $O/gpu_tests.log 2>&1
rc=$?; tail -15 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 3 > $O/bench.log 2>&1
rc=$?; tail -3 $O/bench.log; exit $rc
