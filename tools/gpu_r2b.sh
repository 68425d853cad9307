#!/bin/bash
# Group tests + facade + group chunk overhead.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2b
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_js_facade.py tests/test_wav.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; tail -25 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/group_overhead.py > $O/group_overhead.log 2>&1
rc=$?; cat $O/group_overhead.log; exit $rc
