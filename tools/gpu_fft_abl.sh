#!/bin/bash
# What the FFT costs: the passes after pass 0 / the whole FFT after stage 0 skipped (tools/ablate.py
# no_passes / no_fft; wrong values, timing only), beside phase 2 and the mel scan, both precisions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/fft_abl
mkdir -p $O && cd $R
for prec in faithful fast; do
  echo "== $prec N=1024"
  timeout -k 10 200 python tools/ab_libs.py --precision $prec --rounds 5 --n 1024 --frames 262144 BASE=base no_passes=ab/libabl_no_passes.so \
    no_fft=ab/libabl_no_fft.so no_phase2=ab/libabl_no_phase2.so no_mel=ab/libabl_no_mel.so > $O/$prec.log 2>&1 || { tail -20 $O/$prec.log; exit 1; }
  grep -v amdgpu.ids $O/$prec.log
done
