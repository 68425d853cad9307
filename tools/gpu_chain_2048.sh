#!/bin/bash
# Reference-order MFCC at N = 2048 on the packed-track chains (the tree) against round 2's one-frame
# reference order (ab/libref_old.so) and the default plan: the chain GPU tests (now with N = 2048),
# then interleaved timing with outputs compared bit for bit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_2048
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfcc_chain.py tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/ab_libs.py --n 2048 --frames 131072 --rounds 7 --compare OLD=ab/libref_old.so:2 NEW=base:2 DEF=base > $O/ab_2048.log 2>&1 || { tail -20 $O/ab_2048.log; exit 1; }
grep -v amdgpu.ids $O/ab_2048.log | sed "s/^/N=2048 /"
timeout -k 10 300 python tools/ab_libs.py --n 2048 --frames 131072 --mel 40 --features mfcc --rounds 7 --compare OLD=ab/libref_old.so:2 NEW=base:2 DEF=base > $O/ab_2048_c4.log 2>&1 || { tail -20 $O/ab_2048_c4.log; exit 1; }
grep -v amdgpu.ids $O/ab_2048_c4.log | sed "s/^/N=2048 40 bands /"
