#!/bin/bash
# Round 5: the plan-built LDS image and the prologue's kernel arguments in one burst of scalar loads
# against the previous tree (ab/lib_prev.so): the -m gpu suite, one-frame phase stamps, the real-time
# path, launch times at N = 256 ... 2048 with outputs compared. Results in gpurun_out/r5f/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5f
mkdir -p $O && cd $R
step() { echo "[r5f] $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step stamps
timeout -k 10 300 python tools/small_stamps.py ab/lib_wt.so > $O/small_stamps.log 2>&1 || { tail -20 $O/small_stamps.log; exit 1; }
grep -v amdgpu.ids $O/small_stamps.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
grep -v amdgpu.ids $O/host_latency.log | head -3
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']['us_per_call']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
step ab
for n in 1024 2048 512 256; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare prev=ab/lib_prev.so tree=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log
done
step done
