#!/bin/bash
# Round 5's dynamic VALU budget per frame of extract_kernel<1024> (all features, 262,144 frames): the tree's
# library and tools/ablate.py variants (copied to ab/lib_b_*.so) through tools/gpu_budget.sh's PMC passes,
# then their launch times in one process (tools/ab_libs.py). Output: gpurun_out/r5_budget/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
V="BASE=base"
for v in no_fft no_phase2 no_mel no_amp no_prefix no_scalars no_loud2 no_fft_no_phase2_no_mel_no_amp_no_prefix; do V="$V $v=$R/ab/lib_b_$v.so"; done
BUDGET_TAG=r5_budget BUDGET_VARIANTS="$V" timeout -k 10 900 bash tools/gpu_budget.sh || exit 1
timeout -k 10 600 python tools/ab_libs.py --n 1024 --rounds 7 $V > gpurun_out/r5_budget/times.log 2>&1 || { tail -20 gpurun_out/r5_budget/times.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_budget/times.log
