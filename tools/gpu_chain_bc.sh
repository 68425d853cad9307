#!/bin/bash
# Packed-track chains with the weights broadcast inside each track (ds_swizzle) and the next group's
# weights and rows loaded during the current group (ab/libchain_bc.so, -DMGX_CHAIN_BCAST=1) against the
# tree: outputs compared bit for bit (edge frames included), interleaved timing.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_bc
mkdir -p $O && cd $R
V="TR=base:2 BC=ab/libchain_bc.so:2 DEF=base"
for n in 1024 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare $V > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
timeout -k 10 300 python tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare $V > $O/ab_c4.log 2>&1 || { tail -20 $O/ab_c4.log; exit 1; }
grep -v amdgpu.ids $O/ab_c4.log | sed "s/^/c4 /"
MEYDA_AMD_LIB=$R/ab/libchain_bc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mfcc_chain.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
