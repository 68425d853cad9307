#!/bin/bash
# Round-3: the frame / complex-output bases as wave-uniform pointers (no spill stores in the
# batch loop): WRITE_SIZE per set, interleaved A/B against the previous build with an output
# comparison, then the GPU parity suite.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r3b
mkdir -p $O && cd $R
WRITE_CAPS=default bash tools/gpu_writes.sh > $O/writes.log 2>&1 || { cat $O/writes.log; exit 1; }
tail -2 $O/writes.log
for cfg in "1024 262144" "2048 131072" "512 262144"; do
  n=${cfg% *}; f=${cfg#* }
  echo "== N=$n frames=$f"
  timeout -k 10 200 python tools/ab_libs.py --compare --rounds 7 --n $n --frames $f PREV=ab/libabl_PREV.so NEW=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  tail -4 $O/ab_$n.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
