#!/bin/bash
# Parity (full GPU suite) of the current tree, then A/B: VALU DCT vs the 4x4x4 MFMA DCT.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r2e
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "equals the VALU|passed|failed|Error" $O/gpu_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_libs.py --rounds 7 base=base dct_mfma=base:1 > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; exit $rc
