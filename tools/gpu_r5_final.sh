#!/bin/bash
# Round-5 measurement of the final tree, in one GPU call: the -m gpu suite and smoke(), the real-time
# path (C ABI, JS facade, one-frame phase stamps of the diagnostic build ab/lib_wt.so), the precision
# report, the bench line, its rocprofv3 kernel stats (bench.py --single-stream), PMC traffic and VALU mix.
# Results in gpurun_out/final/ (copied into profiles/r05_* after review).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/final
mkdir -p $O && cd $R
step() { echo "[final] $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']['us_per_call']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
timeout -k 10 300 python tools/small_stamps.py ab/lib_wt.so > $O/small_stamps.log 2>&1 || { tail -20 $O/small_stamps.log; exit 1; }
grep -v amdgpu.ids $O/small_stamps.log
step precision
timeout -k 10 300 python tools/precision_report.py 512 1024 2048 > $O/precision.log 2>&1 || { tail -20 $O/precision.log; exit 1; }
step bench
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_fp64']['frac'], d['roofline_fp64'].get('valu_busy_measured')); print('c5', d['c5']['kernel_ms'], d['c5']['roofline_frac'], 'mfcc_exact', d['mfcc_exact']['cost_vs_value_kernel'])"
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --single-stream --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c2 --no-c3 --no-c4 --no-c5 --no-mfcc-exact --no-latency > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 40 > $O/prof_summary.txt; head -6 $O/prof_summary.txt
cd $R
step traffic
timeout -k 10 600 $R/tools/gpu_traffic.sh > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp $R/gpurun_out/traffic/summary.json $O/pmc_traffic.json
step valu_pmc
timeout -k 10 600 $R/tools/gpu_pmc_cur.sh || { echo "pmc failed"; exit 1; }
cp $R/gpurun_out/pmc_cur.log $O/ 2>/dev/null
step done
