#!/bin/bash
# Mel chains on packed tracks (the tree) against the round-3 phase schedule (ab/libchain_phase.so) and
# the default plan: the chain and MFCC GPU tests first, then A/B timing with outputs compared bit for bit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_t
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfcc_chain.py tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for n in 1024 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare PH=ab/libchain_phase.so:2 TR=base:2 DEF=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
timeout -k 10 300 python tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare PH=ab/libchain_phase.so:2 TR=base:2 DEF=base > $O/ab_c4.log 2>&1 || { tail -20 $O/ab_c4.log; exit 1; }
grep -v amdgpu.ids $O/ab_c4.log | sed "s/^/c4 /"
