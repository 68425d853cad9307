#!/bin/bash
# Reference-order MFCC (MGX_FLAG_MFCC_REFERENCE) with the power rows stored lane-contiguously from the LDS
# amplitude row (tree) against the previous per-lane stores (ab/lib_head.so): the chain parity tests, then
# launch times with outputs compared bit for bit at N = 1024 / 2048 / 512 / 256 and C4 (40 bands, mfcc
# alone), the default plan beside them. Output: gpurun_out/chain_rows/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_rows
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfcc_chain.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 1024 2048 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare head=ab/lib_head.so:2 tree=base:2 default=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  echo "N=$n"; grep -v amdgpu.ids $O/ab_$n.log
done
timeout -k 10 300 python tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare head=ab/lib_head.so:2 tree=base:2 default=base > $O/ab_c4.log 2>&1 || { tail -20 $O/ab_c4.log; exit 1; }
echo "C4"; grep -v amdgpu.ids $O/ab_c4.log
