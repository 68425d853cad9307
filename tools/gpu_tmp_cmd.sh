#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/shares3 && mkdir -p $O && cd $R
bash tools/gpu_check.sh all > $O/check.log 2>&1
rc=$?; tail -2 $O/check.log; [ $rc -ne 0 ] && exit $rc
C3=spectralCentroid,spectralFlatness,spectralSlope,spectralRolloff,spectralSpread,spectralSkewness,spectralKurtosis,loudness,perceptualSpread,perceptualSharpness
timeout -k 10 200 python tools/ab_libs.py --rounds 5 --features $C3 eq=abl/libabl_eq.so base=base > $O/c3.log 2>&1 || exit 1
echo C3; grep median $O/c3.log
timeout -k 10 200 python tools/ab_libs.py --rounds 5 --features mfcc eq=abl/libabl_eq.so base=base > $O/c4.log 2>&1 || exit 1
echo mfcc; grep median $O/c4.log
