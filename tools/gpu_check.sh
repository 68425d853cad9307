#!/bin/bash
# One GPU call for a tree change: the -m gpu suite (one process), smoke(), then the default bench line.
# Results in gpurun_out/check/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/check
mkdir -p $O && cd $R
echo "[check] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 160 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
echo "[check] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$NO_BENCH" ]; then
  echo "[check] bench"
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic']); print('c5', d['c5'].get('kernel_ms'), d['c5'].get('roofline_frac'), 'mfcc_exact', d['mfcc_exact'].get('cost_vs_value_kernel'))"
fi
echo "[check] done"
