#!/bin/bash
# Round 5: get() extracts into a reused scratch buffer per output layout: the facade's GPU tests, the one-frame
# parity tests (incl. outputs equal to the word-wait preset), then the real-time path.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5k
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_js_facade.py tests/test_gpu_parity.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 node tools/latency.js > $O/latency.log 2>&1 || { tail -20 $O/latency.log; exit 1; }
tail -1 $O/latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
