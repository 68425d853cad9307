#!/bin/bash
# Round 6's judged measurements of the final tree in one GPU call (results in gpurun_out/final6/, copied into profiles/r06_*):
# the -m gpu suite and smoke(); the real-time path (C ABI, JS facade with the application-set HIP_FORCE_DEV_KERNARG=0);
# the precision report; the bench line; rocprofv3 --kernel-trace --stats of bench.py --single-stream; PMC traffic and VALU
# mix; the dynamic VALU budget by ablation (ab/lib_b6_*.so) with launch times; the two-rank gather rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/final6
mkdir -p $O && cd $R
step() { echo "[final6] $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
tail -1 $O/host_latency.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['c1']['us_per_call']); [print(s['bufferSize'], s['batchFrames'], len(s['features']), round(s['us_per_launch'],1), round(s['us_per_buffer'],2)) for s in d['stream']]"
step precision
timeout -k 10 300 python tools/precision_report.py 512 1024 2048 > $O/precision.log 2>&1 || { tail -20 $O/precision.log; exit 1; }
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
step valu_pmc
timeout -k 10 600 $R/tools/gpu_pmc_cur.sh || { echo "pmc failed"; exit 1; }
cp $R/gpurun_out/pmc_cur.log $O/ 2>/dev/null
step budget
V="BASE=base"
for v in no_fft no_phase2 no_mel no_amp no_prefix no_scalars no_loud2 no_fft_no_phase2_no_mel_no_amp_no_prefix; do V="$V $v=ab/lib_b6_$v.so"; done
BUDGET_TAG=final6/budget BUDGET_VARIANTS="$V" timeout -k 10 900 bash tools/gpu_budget.sh > $O/budget.log 2>&1 || { tail -20 $O/budget.log; exit 1; }
cd $R
timeout -k 10 600 python tools/ab_libs.py --n 1024 --rounds 7 $V > $O/budget_times.log 2>&1 || { tail -20 $O/budget_times.log; exit 1; }
cat $O/budget/budget.txt; grep -v amdgpu.ids $O/budget_times.log
step rehearsal
timeout -k 10 900 bash tools/gpu_dist_rehearsal.sh > $O/dist.log 2>&1 || { tail -30 $O/dist.log; exit 1; }
cat $O/dist.log
cp -r $R/gpurun_out/dist $O/dist 2>/dev/null
step done
