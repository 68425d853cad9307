#!/bin/bash
# The last round-5 GPU call: the driver's round-end steps on the final tree (tools/gpu_full.sh: the -m gpu suite,
# smoke(), the bench line), then the N = 2048 tail-pool sweep (tools/pool_ab.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
FULL_TAG=full3 bash tools/gpu_full.sh || exit 1
timeout -k 10 300 python tools/pool_ab.py 15 20 30 40 > gpurun_out/pool3.log 2>&1 || { tail -20 gpurun_out/pool3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pool3.log
