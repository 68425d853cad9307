#!/bin/bash
# Round 5: one-frame launches at N <= 512 carry their frame in the kernel arguments (KernelArgsInline), and
# the output-pointer load goes first: the -m gpu suite, smoke, one-frame phase stamps, the real-time path,
# and launch times of 262,144-frame batches against the previous tree (ab/lib_head.so), outputs compared.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r5h
mkdir -p $O && cd $R
step() { echo "[r5h] $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step stamps
timeout -k 10 300 python tools/small_stamps.py ab/lib_wt.so > $O/small_stamps.log 2>&1 || { tail -20 $O/small_stamps.log; exit 1; }
grep -v amdgpu.ids $O/small_stamps.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
grep -v amdgpu.ids $O/host_latency.log | head -3
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
step ab
for n in 1024 512 2048; do
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare head=ab/lib_head.so tree=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  echo "N=$n"; grep -v amdgpu.ids $O/ab_$n.log
done
step done
