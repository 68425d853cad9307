#!/bin/bash
# parity tests + variant timings (N=1024, 2048)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/prof_variants.py ${VARIANT_NS:-1024 2048} > gpurun_out/variants.log 2>&1
rc=$?; grep -v "^{" gpurun_out/variants.log | grep -v amdgpu.ids; exit $rc
