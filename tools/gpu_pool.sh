#!/bin/bash
# The N = 2048 tail pool: timing and bit-for-bit outputs per pool share (tools/pool_ab.py), then the GPU suite
# with every plan of the process using a 10 % pool (MGX_POOL_PCT=10).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/pool
mkdir -p $O && cd $R
timeout -k 10 300 python tools/pool_ab.py 5 10 15 25 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
MGX_POOL_PCT=10 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
