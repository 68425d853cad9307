#!/bin/bash
# Round 5: the facade's kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0 unless set): the facade's GPU
# tests, then tools/latency.js with the environment forcing device-memory arguments (the HIP default) and with
# the facade's own setting.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5l
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_js_facade.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 facade; do
  if [ $v = 1 ]; then HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 node tools/latency.js > $O/latency_$v.log 2>&1 || { tail -20 $O/latency_$v.log; exit 1; }
  else timeout -k 10 300 node tools/latency.js > $O/latency_$v.log 2>&1 || { tail -20 $O/latency_$v.log; exit 1; }; fi
  echo "== $v"; tail -1 $O/latency_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
done
