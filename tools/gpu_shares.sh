#!/bin/bash
# Rank shares of the four workgroups of a CU at N = 1024 (kernels.hip, "shares 22 / 18 / 14 / 10"):
# the tree's against flatter, steeper and equal shares, one stream, interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/shares
mkdir -p $O && cd $R
for r in 1 2; do
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 7 --compare BASE=base S20_17_15_12=ab/libr20_17_15_12.so S24_18_13_9=ab/libr24_18_13_9.so S23_19_13_9=ab/libr23_19_13_9.so S16x4=ab/libr16_16_16_16.so > $O/ab$r.log 2>&1 || { tail -20 $O/ab$r.log; exit 1; }
grep -v amdgpu.ids $O/ab$r.log
done
