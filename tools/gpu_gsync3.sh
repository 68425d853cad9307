#!/bin/bash
# The per-second-group workgroup barrier (the tree, Geo::GROUP_SYNC = 2 at N <= 1024) against none
# (ab/libgs0.so) at N = 512 and 256 and config C2: outputs bit for bit, interleaved timing.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/gsync3
mkdir -p $O && cd $R
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_libs.py --rounds 7 --compare "$@" K0=ab/libgs0.so K2=base > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; grep -v amdgpu.ids $O/$tag.log | sed "s/^/$tag /"; }
run all512 --n 512
run all256 --n 256
run c2 --n 512 --frames 65536 --features amplitudeSpectrum,spectralCentroid
run all1024 --n 1024
