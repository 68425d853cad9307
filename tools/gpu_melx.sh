#!/bin/bash
# The default mel sums on the matrix cores (mel_mfma): parity tests on the tree's library, then A/B
# timing against the round-3 build (ab/libbase_head.so, segmented scan) and the variant without the
# window held in registers (ab/libmelx_b.so); outputs compared (only mfcc may differ from BASE).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/melx
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 1024 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 5 --compare BASE=ab/libbase_head.so MXA=ab/libmelx_a.so MXB=ab/libmelx_b.so NO_MEL=ab/libabl_no_mel.so > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
