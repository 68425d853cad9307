#!/bin/bash
# Round 6's closing measurements of the final tree (after the non-temporal frame loads and the resident path), in
# one GPU call; results in gpurun_out/final6b/, copied into profiles/r06_*: the -m gpu suite and smoke(); the
# real-time path (C ABI small batches; the JS facade launched and resident, back to back and with idle gaps);
# the bench line; rocprofv3 --kernel-trace --stats of bench.py --single-stream; PMC traffic.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/final6b
mkdir -p $O && cd $R
step() { echo "[final6b] $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k]['us_per_call'] for k in ('c1', 'c1_resident', 'c1_gap', 'c1_resident_gap')})"
step bench
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_fp64']['frac'], d['roofline_fp64'].get('valu_busy_measured')); print('c5', d['c5']['kernel_ms'], d['c5']['roofline_frac'], d['c5']['value'], 'mfcc_exact', d['mfcc_exact']['cost_vs_value_kernel'])"
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --single-stream --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c2 --no-c3 --no-c4 --no-c5 --no-mfcc-exact --no-latency > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 40 > $O/prof_summary.txt; head -6 $O/prof_summary.txt
cd $R
step traffic
timeout -k 10 600 $R/tools/gpu_traffic.sh > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp $R/gpurun_out/traffic/summary.json $O/pmc_traffic.json
step done
