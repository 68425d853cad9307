#!/bin/bash
# Round 5: get() without per-feature closures and re-dispatch: the facade's GPU tests, then tools/latency.js twice.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5m
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_js_facade.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 node tools/latency.js > $O/latency_$i.log 2>&1 || { tail -20 $O/latency_$i.log; exit 1; }
  tail -1 $O/latency_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
done
