#!/bin/bash
# Packed-track mel chains: non-temporal frame loads in the CHAIN kernels (ab/libchain_nt.so, -DMGX_CHAIN_NT=1: the
# ring keeps more of the L2), the next group's rows in flight (ab/libchain_pf.so, -DMGX_CHAIN_PF=1) and both
# (ab/libchain_pfnt.so) against the tree: outputs compared bit for bit, interleaved timing.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_nt
mkdir -p $O && cd $R
V="TR=base:2 NT=ab/libchain_nt.so:2 PF=ab/libchain_pf.so:2 PFNT=ab/libchain_pfnt.so:2 DEF=base"
for n in 1024 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare $V > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
timeout -k 10 300 python tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare $V > $O/ab_c4.log 2>&1 || { tail -20 $O/ab_c4.log; exit 1; }
grep -v amdgpu.ids $O/ab_c4.log | sed "s/^/c4 /"
