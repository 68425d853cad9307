#!/bin/bash
# Cumulative timing ablations (tools/ablate.py a+b+...): what is left of the N = 1024 launch
# without the FFT, phase 2, the mel scan, the amplitude and the prefix row; and the time-only set.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/cum_abl
mkdir -p $O && cd $R
timeout -k 10 300 python tools/ab_libs.py --rounds 5 --n 1024 --frames 262144 BASE=base no_fft=ab/libabl_no_fft.so \
  fft+p2=ab/libabl_no_fft_no_phase2.so fft+p2+mel=ab/libabl_no_fft_no_phase2_no_mel.so \
  fft+p2+mel+amp+pref=ab/libabl_no_fft_no_phase2_no_mel_no_amp_no_prefix.so amp+pref+mel=ab/libabl_no_amp_no_prefix_no_mel.so \
  > $O/cum.log 2>&1 || { tail -20 $O/cum.log; exit 1; }
grep -v amdgpu.ids $O/cum.log
timeout -k 10 200 python tools/ab_libs.py --rounds 5 --n 1024 --frames 262144 --features rms,energy,zcr BASE=base > $O/time_only.log 2>&1 || { tail -20 $O/time_only.log; exit 1; }
grep -v amdgpu.ids $O/time_only.log | sed 's/^/time-only: /'
timeout -k 10 200 python tools/ab_libs.py --rounds 5 --n 1024 --frames 262144 --features spectralCentroid BASE=base > $O/centroid.log 2>&1 || { tail -20 $O/centroid.log; exit 1; }
grep -v amdgpu.ids $O/centroid.log | sed 's/^/centroid: /'
