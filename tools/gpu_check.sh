#!/bin/bash
# GPU check of a change: the GPU tests selected by $1 (pytest -k expression, "all" = every GPU
# test), then an interleaved A/B timing (tools/ab_libs.py) of the variants given as the other
# arguments. Each GPU step under its own limit; stop at the first failure.
# usage: tools/gpu_check.sh 'K_EXPR' [NAME=PATH[:flags] ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/check
mkdir -p $O && cd $R
sel=$1; shift
if [ "$sel" = all ]; then k=(); else k=(-k "$sel"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu "${k[@]}" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|bit-exact|Error" $O/gpu_tests.log | tail -40; [ $rc -ne 0 ] && exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 300 python tools/ab_libs.py --rounds 7 "$@" > $O/ab.log 2>&1
  rc=$?; cat $O/ab.log; [ $rc -ne 0 ] && exit $rc
fi
exit 0
