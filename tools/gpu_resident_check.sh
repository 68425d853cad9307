#!/bin/bash
# MGX_FLAG_RESIDENT on the GPU: its tests (Python C ABI and the facade), the C-ABI latency microbenchmark
# (tools/ubench/small_latency.hip: K = a resident plan) and the facade's real-time latency (tools/latency.js).
# Output: gpurun_out/res/
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/res
mkdir -p $O && cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -h 'beside a resident' $O/tests.log; tail -1 $O/tests.log
timeout -k 10 300 node --expose-gc tests/js/facade_gpu.js > $O/facade.log 2>&1 || { tail -20 $O/facade.log; exit 1; }
tail -2 $O/facade.log
timeout -k 10 120 ./tools/ubench/small_latency 512 3000 > $O/small_latency.log 2>&1 || { tail -5 $O/small_latency.log; exit 1; }
grep -v amdgpu.ids $O/small_latency.log
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 node tools/latency.js > $O/latency.log 2>&1 || { tail -5 $O/latency.log; exit 1; }
grep -v amdgpu.ids $O/latency.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c1', d['c1']['us_per_call'], d['c1']['us_p90'], 'c1_resident', d['c1_resident']['us_per_call'], d['c1_resident']['us_p90'])
print('c1_gap', d['c1_gap']['us_per_call'], d['c1_gap']['us_p90'], 'c1_resident_gap', d['c1_resident_gap']['us_per_call'], d['c1_resident_gap']['us_p90'])
for s in d['stream']: print(s['bufferSize'], s['batchFrames'], s['resident'], s['us_per_launch'], s['us_per_buffer'])"
