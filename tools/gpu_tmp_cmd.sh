#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/fin && mkdir -p $O && cd $R
timeout -k 10 300 python tools/configs_bench.py > $O/configs.log 2>&1 || { tail $O/configs.log; exit 1; }
timeout -k 10 120 python tools/step_overlap.py --rounds 3 --steps 50 > $O/overlap.log 2>&1 || exit 1
grep median $O/overlap.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
