#!/bin/bash
# Where the CHAIN kernels' cost goes: the tree's library, the chains skipped, the weights from
# registers (tools/ablate.py chain_none / chain_noload), N = 1024 and 512, all features.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_abl
mkdir -p $O && cd $R
for v in base chain_none; do
  if [ $v = base ]; then unset MEYDA_AMD_LIB; else export MEYDA_AMD_LIB=$R/abl/libabl_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python tools/mfcc_cost.py --n 1024 512 --rounds 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep -v amdgpu.ids $O/$v.log
done
