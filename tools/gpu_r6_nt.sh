#!/bin/bash
# Non-temporal frame loads for batches larger than the MALL (plan.cpp nt_frames) against the round-6 tree
# (ab/lib_head.so = tools/build_rev.sh HEAD head): HBM traffic at N = 1024 (tools/gpu_traffic_ab.sh), launch
# times with outputs compared bit for bit at every config size (tools/ab_libs.py), then the -m gpu suite.
# Output: gpurun_out/nt/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/nt
mkdir -p $O && cd $R
AB="timeout -k 10 300 python3 $R/tools/ab_libs.py --rounds 7 --compare head=$R/ab/lib_head.so nt=base"
bash tools/gpu_traffic_ab.sh head=ab/lib_head.so nt=base > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp gpurun_out/traffic_ab/summary.json $O/traffic_summary.json
tail -4 $O/traffic.log
for c in "--n 2048" "--n 512" "--n 512 --frames 65536 --features amplitudeSpectrum,spectralCentroid" \
         "--n 1024 --features rms,energy,zcr" "--n 1024 --features spectralCentroid,spectralRolloff,spectralFlatness,loudness" \
         "--n 1024 --features mfcc --mel 40" "--n 256"; do
  echo "[nt] $c" | tee -a $O/ab.log
  $AB $c >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  tail -3 $O/ab.log
done
echo "[nt] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
