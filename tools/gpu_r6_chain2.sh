#!/bin/bash
# Round 6: the reference-order MFCC (flag 2) with its power rows loaded one chain group ahead (ab/lib_r6_pf.so)
# and, on top, the matrix-core DCT (the tree), against the round-start library (ab/lib_r6a.so); the default plan
# beside them. Outputs compared bit for bit; the -m gpu suite first. Results in gpurun_out/r6c2/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r6c2
mkdir -p $O && cd $R
step() { echo "[r6c2] $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for n in 1024 2048 512 256; do
  step "ab N=$n"
  timeout -k 10 300 python tools/ab_libs.py --n $n --rounds 7 --compare old=ab/lib_r6a.so:2 pf=ab/lib_r6_pf.so:2 tree=base:2 default=base > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$n.log
done
step "ab C4"
timeout -k 10 300 python tools/ab_libs.py --n 1024 --mel 40 --features mfcc --rounds 7 --compare old=ab/lib_r6a.so:2 pf=ab/lib_r6_pf.so:2 tree=base:2 default=base > $O/ab_c4.log 2>&1 || { tail -20 $O/ab_c4.log; exit 1; }
grep -v amdgpu.ids $O/ab_c4.log
step done
