#!/bin/bash
# Where the matrix-core mel's time goes (N = 1024, timing only: the variants compute wrong mfcc).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/melx2
mkdir -p $O && cd $R
for n in 1024 512; do timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 5 BASE=ab/libbase_head.so MXB=ab/libmelx_b.so MXB2=ab/libmelx_b2.so MXA2=ab/libmelx_a.so NO_MEL=ab/libabl_no_mel.so >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }; done
grep -v amdgpu.ids $O/ab.log
