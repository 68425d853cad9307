#!/bin/bash
# A/B of the previous build (ab/libabl_PREV.so, tools/build_prev.sh) against the tree, both
# precisions, with an output comparison.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/ab_fast
mkdir -p $O && cd $R
for prec in fast faithful; do
  for cfg in "1024 262144" "2048 131072" "512 262144"; do
    n=${cfg% *}; f=${cfg#* }
    echo "== $prec N=$n"
    timeout -k 10 200 python tools/ab_libs.py --precision $prec --compare --rounds 5 --n $n --frames $f PREV=ab/libabl_PREV.so NEW=base > $O/${prec}_$n.log 2>&1 || { tail -20 $O/${prec}_$n.log; exit 1; }
    grep -E "^(PREV|NEW)" $O/${prec}_$n.log
  done
done
