#!/bin/bash
# The time-only requests' next-frame prefetch issued after their reductions (so the prefetched and
# the current frame share registers: no per-frame copy, fewer spills) against the round-3 build:
# outputs compared bit for bit, several feature sets and sizes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/pf
mkdir -p $O && cd $R
run() { tag=$1; shift; timeout -k 10 200 python tools/ab_libs.py --rounds 5 --compare "$@" BASE=ab/libbase_head.so PF=ab/libpf.so LOG4=ab/liblog4.so > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; grep -v amdgpu.ids $O/$tag.log | sed "s/^/$tag /"; }
run all1024 --n 1024
run all512 --n 512
run all2048 --n 2048 --frames 131072
run time1024 --n 1024 --features rms,energy,zcr
run c2 --n 512 --frames 65536 --features amplitudeSpectrum,spectralCentroid
run c3 --n 1024 --features spectralCentroid,spectralFlatness,spectralSlope,spectralRolloff,spectralSpread,spectralSkewness,spectralKurtosis,loudness,perceptualSpread,perceptualSharpness
run mfcc1024 --n 1024 --features mfcc
