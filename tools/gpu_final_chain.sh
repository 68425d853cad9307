#!/bin/bash
# The final tree: the whole GPU suite, smoke, the bench line, then the reference-order MFCC cost at
# every N (and C4's 40 bands) against the default plan, interleaved in one process.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
bash tools/gpu_full.sh || exit 1
O=$R/gpurun_out/mfcc_cost
mkdir -p $O
timeout -k 10 400 python tools/mfcc_cost.py --n 256 512 1024 2048 > $O/all.log 2>&1 || { tail -20 $O/all.log; exit 1; }
grep -v amdgpu.ids $O/all.log
timeout -k 10 300 python tools/mfcc_cost.py --n 1024 2048 --features c4 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
grep -v amdgpu.ids $O/c4.log
