#!/bin/bash
# Cost of two workgroup barriers per frame at the mel step (tools/ablate.py bar2), with and without
# the mel scan; 262,144 frames (every wave of a workgroup gets the same number of frames).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/bar
mkdir -p $O && cd $R
timeout -k 10 200 python tools/ab_libs.py --n 1024 --rounds 5 BASE=base BAR2=ab/libabl_bar2.so NO_MEL=ab/libabl_no_mel.so BAR2_NO_MEL=ab/libabl_bar2_no_mel.so > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
