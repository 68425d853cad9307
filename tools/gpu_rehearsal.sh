#!/bin/bash
# Round-end rehearsal: what the driver runs on a fresh box (every GPU test, smoke, the
# default bench line), each step under its own limit; stop at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/rehearsal
mkdir -p $O && cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log; exit $rc
