#!/bin/bash
# Round 5: the facade over extractInto (GPU facade tests, latency) and where a one-frame call's kernel time goes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_js_facade.py tests/test_gpu_parity.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider -k "facade or small or alternate" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 node tools/latency.js > $O/latency.log 2>&1 || { tail -20 $O/latency.log; exit 1; }
tail -1 $O/latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']['us_per_call']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
timeout -k 10 300 python tools/small_stamps.py ab/lib_wt.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
