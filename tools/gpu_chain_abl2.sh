#!/bin/bash
# Where the packed-track chains' time goes (timing ablations, wrong values): NOLOAD (no weight / row
# loads), NODEP (the 8 steps of a group independent), NONE (the chains skipped) against the tree (TR) and
# the default plan (DEF), interleaved, N = 1024 and 512.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_abl2
mkdir -p $O && cd $R
V="TR=base:2 NOLOAD=ab/libabl_chain_noload.so:2 NODEP=ab/libabl_chain_nodep.so:2 NONE=ab/libabl_chain_none.so:2 DEF=base"
for n in 1024 512; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 $V > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log | sed "s/^/N=$n /"
done
