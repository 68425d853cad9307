#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/shares5 && mkdir -p $O && cd $R
bash tools/gpu_check.sh all > $O/check.log 2>&1
rc=$?; tail -1 $O/check.log; [ $rc -ne 0 ] && exit $rc
for n in 256 512 1024 2048; do
  timeout -k 10 200 python tools/ab_libs.py --n $n --rounds 5 --compare r0=abl/libabl_eq.so base=base > $O/n$n.log 2>&1 || { tail $O/n$n.log; exit 1; }
  echo "N=$n"; grep -E "median|outputs" $O/n$n.log
done
timeout -k 10 200 python tools/ab_libs.py --n 512 --frames 65536 --features amplitudeSpectrum,spectralCentroid --rounds 5 r0=abl/libabl_eq.so base=base > $O/c2.log 2>&1 || exit 1
echo C2; grep median $O/c2.log
