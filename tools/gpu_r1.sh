#!/bin/bash
# Round-1 measurement bundle: parity, variants, bench, rocprof stats, PMC traffic.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/prof_variants.py ${VARIANT_NS:-1024} > gpurun_out/variants.log 2>&1
rc=$?; grep -v "^{" gpurun_out/variants.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_PROF" ] && exit 0
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -2 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1
rc=$?; tail -1 $R/gpurun_out/prof_bench.log; [ $rc -ne 0 ] && exit $rc
$R/tools/gpu_traffic.sh
