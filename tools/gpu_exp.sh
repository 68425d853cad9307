#!/bin/bash
# One GPU call of the current experiment: optional pytest selection ($EXP_TESTS), then an
# interleaved A/B of the tree's library against ab/lib_*.so variants with a bit-for-bit output
# comparison (tools/ab_libs.py --compare) at each N in $EXP_NS (default 1024), all features.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/${EXP_TAG:-exp}
mkdir -p $O && cd $R
if [ -n "$EXP_TESTS" ]; then
  echo "[exp] tests: $EXP_TESTS"
  timeout -k 10 600 python -u -m pytest $EXP_TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if [ -n "$EXP_PRE" ]; then
  echo "[exp] pre: $EXP_PRE"
  timeout -k 10 300 bash -c "$EXP_PRE" > $O/pre.log 2>&1 || { tail -30 $O/pre.log; exit 1; }
  tail -20 $O/pre.log
fi
vars=""
for f in ab/lib_*.so; do [ -f "$f" ] || continue; b=$(basename $f .so); vars="$vars ${b#lib_}=$f"; done
for n in ${EXP_NS:-1024}; do
  echo "[exp] A/B N=$n:$vars"
  timeout -k 10 400 python tools/ab_libs.py --compare --rounds ${EXP_ROUNDS:-7} --n $n BASE=base $vars > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log
done
