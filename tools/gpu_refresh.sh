#!/bin/bash
# Regenerate every judged measurement of the current tree in one GPU call:
# parity tests, op-rate microbenchmark, variant timings, the BASELINE configs, precision
# report, the bench line, its rocprofv3 kernel stats and the PMC HBM traffic.
# Results land in gpurun_out/refresh/ (copied into profiles/ by hand after review).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/refresh
mkdir -p $O && cd $R
step() { echo "[refresh] $1"; }
step tests
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step latency
timeout -k 10 300 python tools/host_latency.py > $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
timeout -k 10 300 node tools/latency.js >> $O/host_latency.log 2>&1 || { tail -20 $O/host_latency.log; exit 1; }
step variants
timeout -k 10 300 python tools/prof_variants.py ${VARIANT_NS:-256 512 1024 2048} > $O/variants.log 2>&1 || exit 1
step configs
timeout -k 10 300 python tools/configs_bench.py > $O/configs.log 2>&1 || exit 1
step precision
timeout -k 10 300 python tools/precision_report.py 512 1024 2048 > $O/precision.log 2>&1 || exit 1
step bench
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --single-stream --no-cpu-baseline --no-host-path --no-pmc --no-every-output --no-fast --no-c2 --no-c3 --no-c4 --no-c5 --no-mfcc-exact --no-latency > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log
# the 100 timed (pipelined) launches' period, then the 20 single-stream launches after them
python3 $R/tools/prof_summary.py $O/prof/run_kernel_trace.csv 100 "" 1 40 > $O/prof_summary.txt
step traffic
$R/tools/gpu_traffic.sh > $O/traffic.log 2>&1 || { tail -20 $O/traffic.log; exit 1; }
cp $R/gpurun_out/traffic/summary.json $O/pmc_traffic.json
step valu_pmc
$R/tools/gpu_pmc_cur.sh || { echo "pmc failed"; exit 1; }
step done
