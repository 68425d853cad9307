#!/bin/bash
# Every BASELINE config on the current tree, and the MFCC reference-order cost at N = 2048.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/configs
mkdir -p $O && cd $R
timeout -k 10 400 python tools/configs_bench.py > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
grep -v amdgpu.ids $O/configs.log | tail -12
timeout -k 10 300 python tools/mfcc_cost.py --n 2048 --rounds 5 > $O/cost_2048.log 2>&1 || { tail -20 $O/cost_2048.log; exit 1; }
grep -v amdgpu.ids $O/cost_2048.log
