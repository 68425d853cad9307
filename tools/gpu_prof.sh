#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_variants.py 1024 512 2048 > gpurun_out/variants.log 2>&1
rc=$?; cat gpurun_out/variants.log | grep -v "^{" ; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; find $GRAFT_REPO_ROOT/gpurun_out/prof_r1 -name "*stats*" | head; exit $rc
