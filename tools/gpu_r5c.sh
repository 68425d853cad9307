#!/bin/bash
# Round 5 measurement of the current tree: the GPU suite, the real-time path (C ABI and facade), the
# bench line, its rocprofv3 kernel stats (bench.py --single-stream) and the PMC traffic / VALU passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c; mkdir -p $O
echo "[r5c] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
echo "[r5c] latency"
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
tail -1 $O/host_latency.log | cut -c1-1200
echo "[r5c] bench"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic']); print(json.dumps(d['roofline_fp64'])[:600]); print(json.dumps(d['cpu_baseline'].get('all_cores'))); print('mfcc_exact', d['mfcc_exact']['cost_vs_value_kernel'], d['c4']['mfcc_exact']['cost_vs_config_kernel'], d['c5']['mfcc_exact']['cost_vs_config_kernel']); print('c5', d['c5']['kernel_ms'], d['c5']['roofline_frac'], 'c2', d['c2']['kernel_ms'], 'c3', d['c3']['kernel_ms'], 'c4', d['c4']['kernel_ms'])"
echo "[r5c] rocprof"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --single-stream --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c2 --no-c3 --no-c4 --no-c5 --no-mfcc-exact --no-latency > $R/$O/prof_bench.log 2>&1 || { tail -20 $R/$O/prof_bench.log; exit 1; }
tail -1 $R/$O/prof_bench.log | cut -c1-300
python3 $R/tools/prof_summary.py $(ls $R/$O/prof/*/run_kernel_trace.csv $R/$O/prof/run_kernel_trace.csv 2>/dev/null | head -1) 100 "" 1 40 > $R/$O/prof_summary.txt; cat $R/$O/prof_summary.txt | head -20
