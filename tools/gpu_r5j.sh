#!/bin/bash
# Round 5: one-frame host calls without spectrum outputs wait on their output words instead of a released
# completion word: the -m gpu suite, smoke, the real-time path and the launch-floor microbenchmark.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5j
mkdir -p $O && cd $R
step() { echo "[r5j] $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
grep -v amdgpu.ids $O/host_latency.log | head -3
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
timeout -k 10 120 ./tools/ubench/small_latency 512 3000 > $O/small_latency.log 2>&1 || { tail -20 $O/small_latency.log; exit 1; }
grep -v amdgpu.ids $O/small_latency.log
step done
