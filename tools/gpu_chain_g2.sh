#!/bin/bash
# Paired-batch chains: software-pipelined loads (tree) against the first paired build (ab/libchain_g1.so),
# the round-3 LDS-row chains (ab/libchain_lds.so) and the default plan; chain tests first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_g2
mkdir -p $O && cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfcc_chain.py tests/test_gpu_parity.py -k "chain or mfcc_reference" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 1024 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 5 --compare REF_L=ab/libchain_lds.so:2 G1=ab/libchain_g1.so:2 G2=base:2 DEF=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
